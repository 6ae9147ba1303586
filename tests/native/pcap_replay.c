/*
 * Offline replay of a pcap capture through the checksum stages of libuinet's
 * IPv4 receive path, the consumer side of SURVEY.md section 8f item 3
 * (`multitool --pcap file://...`: uinet_if_pcap_host.c:227-228 and
 * uinet_if_pcap.c:690-715 feed each frame to the stack; the stack's bad-sum
 * counters, uinet_api.c:170, must stay 0 on the reference's own capture).
 *
 * libpcap and the stack itself cannot be built here (Next item 6),
 * so this harness reads the capture file itself and restates, frame by frame
 * and in the stack's order, the receive steps that decide a checksum verdict:
 *   ether_input       m_adj of the 14-B Ethernet header (type 0x0800 only)
 *   ip_input.c:460-471   CSUM_IP_CHECKED -> !CSUM_IP_VALID, else in_cksum_hdr
 *                        (hlen 20) / in_cksum(m, hlen); ips_badsum, drop
 *   ip_input.c:482-499   ip_len < hlen: ips_badlen; chain shorter: ips_tooshort
 *   ip_input.c:760-761   fragments go to ip_reass (counted, not verified)
 *   tcp_input.c:697-718  CSUM_DATA_VALID (| CSUM_PSEUDO_HDR) -> csum_data ^
 *                        0xffff, else in_cksum_pseudo_header(m, tlen, off0,
 *                        src, dst, TCP); tcps_rcvbadsum, drop
 *   udp_usrreq.c:404-449 uh_ulen checks (udps_badlen), uh_sum 0: udps_nosum,
 *                        else the same two ways; udps_badsum, drop
 *
 * Modes (argv[2]):
 *   offload    the whole capture first goes through uinet_cksum_rx_offload
 *              (the engine's GPU batch hook), then the stack reads the marks;
 *   software   no hook: every verdict from the engine's per-call functions;
 *   reference  no hook: every verdict from the reference's own functions
 *              (oracle/_ref/libref_cksum.so, loaded by path at run time).
 * argv[3] = K corrupts one bit in K frames (deterministic positions past the
 * Ethernet header).  Frames sit in 2-KiB clusters at a 0-3-B offset; every
 * third frame is split into two mbufs after its headers.
 * Output: one line of counters.
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define IPVERSION 4
#include "uinet_cksum.h"

/* the reference layout (sys/sys/mbuf.h:90-133): m_hdr, then m_pkthdr with
 * csum_flags @64 and csum_data @68 */
struct mbuf {
	struct mbuf *m_next;
	void *m_nextpkt;
	char *m_data;
	int m_len;
	int m_flags;
	short m_type;
	char m_pad[6];
	char m_pkthdr_head[24];
	int csum_flags;
	int csum_data;
	char m_rest[184];
};
_Static_assert(sizeof(struct mbuf) == 256, "MSIZE");
_Static_assert(__builtin_offsetof(struct mbuf, csum_flags) == 64, "csum_flags");

#define M_PKTHDR 0x2
#define CSUM_IP_CHECKED 0x100
#define CSUM_IP_VALID 0x200
#define CSUM_DATA_VALID 0x400
#define CSUM_PSEUDO_HDR 0x800

typedef unsigned short (*skip_fn)(struct mbuf *, int, int);
typedef uint16_t (*pseudo_fn)(struct mbuf *, int, int, uint32_t, uint32_t, uint8_t);
typedef unsigned int (*hdr_fn)(const void *);

static skip_fn f_skip;
static pseudo_fn f_pseudo;
static hdr_fn f_hdr;

static unsigned short
eng_skip(struct mbuf *m, int len, int skip)
{
	return in_cksum_skip(m, len, skip);
}

static uint16_t
eng_pseudo(struct mbuf *m, int plen, int off0, uint32_t s, uint32_t d, uint8_t p)
{
	return in_cksum_pseudo_header(m, plen, off0, s, d, p);
}

static unsigned int
eng_hdr(const void *ip)
{
	return in_cksum_hdr((const struct ip *)ip);
}

static uint32_t
rd32(const uint8_t *p, int swap)
{
	uint32_t v;
	memcpy(&v, p, 4);
	return swap ? __builtin_bswap32(v) : v;
}

static int
chain_len(const struct mbuf *m)
{
	int t = 0;
	for (; m; m = m->m_next)
		t += m->m_len;
	return t;
}

int
main(int argc, char **argv)
{
	FILE *f;
	long sz;
	uint8_t *file;
	int swap, nfr = 0, cap = 4096, i, corrupt = argc > 3 ? atoi(argv[3]) : 0;
	size_t o;
	uint8_t **fr;
	int *frlen;
	const char *mode = argc > 2 ? argv[2] : "software";
	long ipv4 = 0, tcp = 0, udp = 0, frags = 0, ips_badsum = 0, ips_badlen = 0,
	     ips_tooshort = 0, tcps_rcvbadsum = 0, udps_badsum = 0, udps_badlen = 0, udps_nosum = 0,
	     marked = 0;

	if (argc < 2 || !(f = fopen(argv[1], "rb")))
		return 2;
	fseek(f, 0, SEEK_END);
	sz = ftell(f);
	fseek(f, 0, SEEK_SET);
	file = malloc((size_t)sz);
	if (fread(file, 1, (size_t)sz, f) != (size_t)sz)
		return 2;
	fclose(f);
	if (sz < 24)
		return 2;
	if (rd32(file, 0) == 0xa1b2c3d4u || rd32(file, 0) == 0xa1b23c4du)
		swap = 0;
	else if (rd32(file, 1) == 0xa1b2c3d4u || rd32(file, 1) == 0xa1b23c4du)
		swap = 1;
	else
		return 3;
	if (rd32(file + 20, swap) != 1)
		return 3; /* LINKTYPE_ETHERNET */
	fr = malloc(sizeof(*fr) * (size_t)cap);
	frlen = malloc(sizeof(*frlen) * (size_t)cap);
	for (o = 24; o + 16 <= (size_t)sz && nfr < cap;) {
		uint32_t incl = rd32(file + o + 8, swap);
		if (o + 16 + incl > (size_t)sz || incl > 2000)
			break;
		fr[nfr] = file + o + 16;
		frlen[nfr++] = (int)incl;
		o += 16 + incl;
	}

	if (!strcmp(mode, "reference")) {
		void *h = dlopen(argc > 4 ? argv[4] : "oracle/_ref/libref_cksum.so", RTLD_NOW);
		if (!h)
			return 4;
		f_skip = (skip_fn)dlsym(h, "refh_in_cksum_skip");
		f_pseudo = (pseudo_fn)dlsym(h, "refh_in_cksum_pseudo_header");
		f_hdr = (hdr_fn)dlsym(h, "refh_in_cksum_hdr");
		if (!f_skip || !f_pseudo || !f_hdr)
			return 4;
	} else {
		f_skip = eng_skip;
		f_pseudo = eng_pseudo;
		f_hdr = eng_hdr;
	}

	/* the received frames: a 2-KiB cluster each, every third one split */
	char *clusters = aligned_alloc(4096, 2048 * (size_t)nfr + 4096);
	struct mbuf *mb = calloc(2 * (size_t)nfr, sizeof(struct mbuf));
	struct mbuf **mv = malloc(sizeof(*mv) * (size_t)nfr);
	for (i = 0; i < nfr; i++) {
		char *c = clusters + 2048 * (size_t)i + (i & 3);
		struct mbuf *m = &mb[2 * i];
		memcpy(c, fr[i], (size_t)frlen[i]);
		if (i < corrupt * 3 && i % 3 == 0 && frlen[i] > 15) {
			/* one bit past the Ethernet header, at a frame-dependent position */
			int pos = 14 + (int)((2654435761u * (unsigned)(i + 1)) % (unsigned)(frlen[i] - 14));
			c[pos] ^= (char)(1 << (i % 8));
		}
		m->m_data = c;
		m->m_len = frlen[i];
		m->m_flags = M_PKTHDR;
		if (i % 3 == 1 && frlen[i] > 60) {
			int cut = 54 + i % 7;
			struct mbuf *n2 = &mb[2 * i + 1];
			m->m_len = cut;
			n2->m_data = c + cut;
			n2->m_len = frlen[i] - cut;
			m->m_next = n2;
		}
		mv[i] = m;
	}
	if (!strcmp(mode, "offload")) {
		uint8_t *st = malloc((size_t)nfr);
		int rc = uinet_cksum_rx_offload(mv, nfr, -1, st);
		if (rc) {
			fprintf(stderr, "uinet_cksum_rx_offload: %s\n", uinet_cksum_strerror(rc));
			return 5;
		}
		for (i = 0; i < nfr; i++)
			marked += (mv[i]->csum_flags & CSUM_IP_CHECKED) != 0;
		free(st);
	}

	for (i = 0; i < nfr; i++) {
		struct mbuf *m = mv[i];
		const uint8_t *e = (const uint8_t *)m->m_data, *ip;
		int hlen, ip_len, sum, off0;
		uint32_t src, dst;

		if (m->m_len < 34 || (e[12] << 8 | e[13]) != 0x0800)
			continue;
		m->m_data += 14; /* ether_input: m_adj(m, ETHER_HDR_LEN) */
		m->m_len -= 14;
		ip = (const uint8_t *)m->m_data;
		ipv4++;
		hlen = (ip[0] & 15) << 2;
		if ((ip[0] >> 4) != 4 || hlen < 20 || hlen > m->m_len)
			continue; /* ips_badvers / ips_badhlen */
		if (m->csum_flags & CSUM_IP_CHECKED)
			sum = !(m->csum_flags & CSUM_IP_VALID);
		else if (hlen == 20)
			sum = (int)f_hdr(ip);
		else
			sum = f_skip(m, hlen, 0);
		if (sum) {
			ips_badsum++;
			continue;
		}
		ip_len = ip[2] << 8 | ip[3];
		if (ip_len < hlen) {
			ips_badlen++;
			continue;
		}
		if (chain_len(m) < ip_len) {
			ips_tooshort++;
			continue;
		}
		if ((ip[6] << 8 | ip[7]) & 0x3fff) {
			frags++;
			continue;
		}
		memcpy(&src, ip + 12, 4);
		memcpy(&dst, ip + 16, 4);
		off0 = hlen;
		if (ip[9] == 6) {
			int tlen = ip_len - off0, th_sum;
			tcp++;
			if (m->csum_flags & CSUM_DATA_VALID) {
				if (!(m->csum_flags & CSUM_PSEUDO_HDR))
					return 6; /* the hook always sets CSUM_PSEUDO_HDR */
				th_sum = m->csum_data ^ 0xffff;
			} else {
				th_sum = f_pseudo(m, tlen, off0, src, dst, 6);
			}
			if (th_sum)
				tcps_rcvbadsum++;
		} else if (ip[9] == 17) {
			uint8_t uh[8];
			int len, have = 0, uh_sum;
			struct mbuf *p;
			int skip = off0;
			for (p = m; p && have < 8; p = p->m_next) {
				int k;
				if (skip >= p->m_len) {
					skip -= p->m_len;
					continue;
				}
				k = p->m_len - skip < 8 - have ? p->m_len - skip : 8 - have;
				memcpy(uh + have, p->m_data + skip, (size_t)k);
				have += k;
				skip = 0;
			}
			if (have < 8)
				continue;
			udp++;
			len = uh[4] << 8 | uh[5];
			if (len != ip_len - hlen && (len > ip_len - hlen || len < 8)) {
				udps_badlen++;
				continue;
			}
			if (!(uh[6] | uh[7])) {
				udps_nosum++;
				continue;
			}
			if (m->csum_flags & CSUM_DATA_VALID) {
				if (!(m->csum_flags & CSUM_PSEUDO_HDR))
					return 6;
				uh_sum = m->csum_data ^ 0xffff;
			} else {
				uh_sum = f_pseudo(m, len, off0, src, dst, 17);
			}
			if (uh_sum)
				udps_badsum++;
		}
	}
	printf("frames=%d ipv4=%ld marked=%ld tcp=%ld udp=%ld frags=%ld ips_badsum=%ld "
	       "ips_badlen=%ld ips_tooshort=%ld tcps_rcvbadsum=%ld udps_badsum=%ld udps_badlen=%ld "
	       "udps_nosum=%ld\n",
	    nfr, ipv4, marked, tcp, udp, frags, ips_badsum, ips_badlen, ips_tooshort,
	    tcps_rcvbadsum, udps_badsum, udps_badlen, udps_nosum);
	return 0;
}
