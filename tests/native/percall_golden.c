/*
 * A libuinet-shaped consumer of the per-call ABI: compiled against
 * include/uinet_cksum.h and linked with -luinet_cksum (no torch, no Python in
 * the process), it defines struct mbuf with the reference layout
 * (sys/sys/mbuf.h:90-98,153-171: m_next @0, m_data @16, m_len @24, 256 B),
 * rebuilds golden chains from an input file and prints the engine's
 * in_cksum_skip / in_cksum_pseudo_header / in_cksum_hdr results.  The test
 * runs it with no visible GPU (tests/test_percall_host.py).
 *
 * Input (little-endian, written by the test):
 *   u64 arena_len, arena bytes
 *   u32 nseg, u32 npkt: seg_off u64[nseg], seg_len i32[nseg], pkt_seg u32[npkt+1],
 *       then per packet: kind u8 (0 skip, 1 pseudo), i32 a (len | plen),
 *       i32 b (skip | off0), u32 src, u32 dst, u8 proto
 *   u32 nhdr: hdr_off u64[nhdr]
 * Output: u16 per packet, then u32 per header, raw on stdout.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define IPVERSION 4
#include "uinet_cksum.h"

struct mbuf {
	struct mbuf *m_next;
	void *m_nextpkt;
	char *m_data;
	int m_len;
	int m_flags;
	short m_type;
	char m_pad[6];
	char m_rest[216];
};
_Static_assert(sizeof(struct mbuf) == 256, "MSIZE");

struct ip {
	unsigned char b[20];
};

static void
rd(void *p, size_t n, FILE *f)
{
	if (fread(p, 1, n, f) != n) {
		fprintf(stderr, "short input\n");
		exit(2);
	}
}

int
main(int argc, char **argv)
{
	FILE *f = fopen(argv[1], "rb");
	uint64_t alen;
	uint32_t nseg, npkt, nhdr, i;
	unsigned char *raw, *arena;
	uint64_t *seg_off, *hdr_off;
	int32_t *seg_len;
	uint32_t *pkt_seg;
	struct mbuf *mb;

	if (argc != 2 || !f)
		return 2;
	rd(&alen, 8, f);
	raw = malloc(alen + 8192);
	arena = raw + ((4096 - ((uintptr_t)raw & 4095)) & 4095); /* 4-KiB aligned, as generated */
	rd(arena, alen, f);
	rd(&nseg, 4, f);
	rd(&npkt, 4, f);
	seg_off = malloc(8 * (size_t)nseg + 8);
	seg_len = malloc(4 * (size_t)nseg + 4);
	pkt_seg = malloc(4 * ((size_t)npkt + 1));
	rd(seg_off, 8 * (size_t)nseg, f);
	rd(seg_len, 4 * (size_t)nseg, f);
	rd(pkt_seg, 4 * ((size_t)npkt + 1), f);
	mb = calloc(nseg + 1, sizeof(*mb));
	for (i = 0; i < npkt; i++) {
		uint32_t k;
		for (k = pkt_seg[i]; k < pkt_seg[i + 1]; k++) {
			mb[k].m_data = (char *)arena + seg_off[k];
			mb[k].m_len = seg_len[k];
			mb[k].m_next = k + 1 < pkt_seg[i + 1] ? &mb[k + 1] : NULL;
		}
	}
	for (i = 0; i < npkt; i++) {
		unsigned char kind, proto;
		int32_t a, b;
		uint32_t src, dst;
		uint16_t r;
		struct mbuf *m = pkt_seg[i] < pkt_seg[i + 1] ? &mb[pkt_seg[i]] : NULL;

		rd(&kind, 1, f);
		rd(&a, 4, f);
		rd(&b, 4, f);
		rd(&src, 4, f);
		rd(&dst, 4, f);
		rd(&proto, 1, f);
		if (kind == 0)
			r = b == 0 ? in_cksum(m, a) : in_cksum_skip(m, a, b);
		else
			r = in_cksum_pseudo_header(m, a, b, src, dst, proto);
		fwrite(&r, 2, 1, stdout);
	}
	rd(&nhdr, 4, f);
	hdr_off = malloc(8 * (size_t)nhdr + 8);
	rd(hdr_off, 8 * (size_t)nhdr, f);
	for (i = 0; i < nhdr; i++) {
		uint32_t r = in_cksum_hdr((const struct ip *)(arena + hdr_off[i]));
		fwrite(&r, 4, 1, stdout);
	}
	{	/* the reference-named inline, on a header at the last offset */
		struct ip h;
		memcpy(&h, arena, sizeof(h));
		in_cksum_update(&h);
	}
	return 0;
}
