/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * A from-scratch CPU restatement of libuinet's Internet-checksum path, used
 * as the parity checker for the HIP engine in libuinet_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library; the product never links it.
 *
 * Reference behaviour restated here (paths relative to /root/reference):
 *   sys/amd64/amd64/in_cksum.c:91-170   in_cksumdata  (address-aligned word sum)
 *   sys/amd64/amd64/in_cksum.c:172-179  in_addword
 *   sys/amd64/amd64/in_cksum.c:181-191  in_pseudo     (folded, NOT complemented)
 *   sys/amd64/amd64/in_cksum.c:193-232  in_cksum_skip (mbuf-chain walk)
 *   sys/amd64/amd64/in_cksum.c:241-276  in_cksum_pseudo_header
 *   sys/amd64/amd64/in_cksum.c:278-285  in_cksum_hdr
 *   sys/netinet/ip_output.c:962-963     UDP "0 -> 0xffff" rule (caller side)
 *   sys/netinet6/in6_cksum.c:86-357     in6_cksum / in6_cksum_pseudo (IPv6)
 *
 * Parity is pinned by tests/golden/ (vectors produced by oracle/_ref, the
 * reference object compiled from /root/reference/sys/amd64/amd64/in_cksum.c
 * with libuinet's kernel flags, see oracle/Makefile) and by the reference's
 * own fixture lib/libuinet_demo/passive_extract_test.pcap.
 *
 * Arithmetic model (not the reference's code shape): every byte at logical
 * position p contributes byte * 256^(p & 1) to a 64-bit sum (16-bit words in
 * little-endian memory order, the way the amd64 code sums them); the sum is
 * folded with end-around carry, which keeps "sum == 0" (only all-zero input)
 * apart from "sum == 0 mod 65535", exactly like REDUCE16
 * (in_cksum.c:65-71).  in_cksumdata weights by *address* parity and
 * in_cksum_skip re-aligns with "<< 8" when address and logical parity
 * differ (in_cksum.c:222-225); both collapse to the logical-position rule
 * above.  in_cksum_hdr has no such re-alignment, so its weights follow the
 * header's address parity.
 *
 * Out-of-contract inputs: a negative piece length (len < skip, or
 * m_len < off0 for the pseudo-header variant) makes the reference index
 * in_masks[] with a negative value when the address is not 4-byte aligned
 * (undefined behaviour).  Here such a piece contributes nothing, which is
 * what the reference computes for 4-byte-aligned addresses; the running
 * length/parity bookkeeping follows the reference exactly.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

#include "cksum_oracle.h"

/* ---- arithmetic core ---------------------------------------------------- */

/* Sum n bytes; the first byte sits at logical parity `par` (0 = low byte of
 * a little-endian 16-bit word). */
static uint64_t
weighted_sum(const uint8_t *p, long n, unsigned par)
{
	uint64_t lo = 0, hi = 0;
	long i = 0;

	if (n <= 0)
		return 0;
	if (par & 1) {
		hi += p[0];
		i = 1;
	}
	for (; i + 1 < n; i += 2) {
		lo += p[i];
		hi += p[i + 1];
	}
	if (i < n)
		lo += p[i];
	return lo + (hi << 8);
}

/* End-around-carry fold to 16 bits (REDUCE16, in_cksum.c:65-71). */
static uint32_t
fold16(uint64_t s)
{
	while (s >> 16)
		s = (s & 0xffff) + (s >> 16);
	return (uint32_t)s;
}

static uint16_t
bswap16(uint16_t x)
{
	return (uint16_t)((x << 8) | (x >> 8));
}

/* ---- per-call ABI restatement ------------------------------------------- */

/* Shared piece processing of in_cksum_skip / in_cksum_pseudo_header
 * (the `skip_start:` block, in_cksum.c:219-228 and :263-272). */
struct walk {
	uint64_t sum;
	long clen;   /* logical bytes summed so far   */
	long remain; /* bytes still wanted            */
};

static void
take_piece(struct walk *w, const uint8_t *addr, long mlen)
{
	if (w->remain < mlen)
		mlen = w->remain;
	w->sum += weighted_sum(addr, mlen, (unsigned)(w->clen & 1));
	w->clen += mlen;
	w->remain -= mlen;
}

static void
take_rest(struct walk *w, const struct oracle_mbuf *m)
{
	/* in_cksum.c:214-229: zero-length mbufs are passed over. */
	for (; m && w->remain; m = m->m_next) {
		if (m->m_len == 0)
			continue;
		take_piece(w, (const uint8_t *)m->m_data, m->m_len);
	}
}

uint16_t
oracle_cksum_skip(const struct oracle_mbuf *m, int len, int skip)
{
	struct walk w = { 0, 0, (long)len - skip };

	/* in_cksum.c:204-212: find the mbuf that holds byte `skip`. */
	while (skip && m) {
		if (m->m_len > skip) {
			take_piece(&w, (const uint8_t *)m->m_data + skip,
			    m->m_len - skip);
			m = m->m_next;
			skip = 0;
			break;
		}
		skip -= m->m_len;
		m = m->m_next;
	}
	if (skip == 0)
		take_rest(&w, m);
	return (uint16_t)(~fold16(w.sum) & 0xffff);
}

uint16_t
oracle_cksum_pseudo_header(const struct oracle_mbuf *m, int plen, int off0,
    uint32_t src, uint32_t dst, uint8_t proto)
{
	struct walk w;

	/* in_cksum.c:252-253: the seed is src + dst + htons(proto) +
	 * htons(plen), all as stored (network order) little-endian values. */
	w.sum = (uint64_t)src + dst + bswap16(proto) +
	    bswap16((uint16_t)plen);
	w.clen = 0;
	w.remain = plen;
	/* :254-256: the first piece starts off0 bytes into the first mbuf. */
	take_piece(&w, (const uint8_t *)m->m_data + off0, (long)m->m_len - off0);
	take_rest(&w, m->m_next);
	return (uint16_t)(~fold16(w.sum) & 0xffff);
}

unsigned
oracle_cksum_hdr(const void *ip)
{
	/* in_cksum.c:278-285: 20 bytes, weights follow the address parity. */
	uint64_t s = weighted_sum((const uint8_t *)ip, 20,
	    (unsigned)((uintptr_t)ip & 1));
	return ~fold16(s) & 0xffff;
}

uint16_t
oracle_in_pseudo(uint32_t a, uint32_t b, uint32_t c)
{
	return (uint16_t)fold16((uint64_t)a + b + c);
}

uint16_t
oracle_in_addword(uint16_t a, uint16_t b)
{
	return (uint16_t)fold16((uint64_t)a + b);
}

/* ---- IPv6 (sys/netinet6/in6_cksum.c) ------------------------------------ */

/* The zone index KAME embeds in word 1 of a link-local unicast or a link- /
 * interface-local multicast address; in6_cksum leaves it out of the sum
 * (in6_cksum.c:110-124 with scope6.c:502-509, netinet6/in6.h:294-356). */
static uint64_t
in6_scope_word(const uint8_t *a)
{
	int ll = a[0] == 0xfe && (a[1] & 0xc0) == 0x80;
	int mc = a[0] == 0xff && ((a[1] & 0x0f) == 0x02 || (a[1] & 0x0f) == 0x01);

	return (ll || mc) ? (uint64_t)(a[2] | a[3] << 8) : 0;
}

/* in6_cksum.c:86-126: the pseudo header (htonl(len), three zero bytes,
 * nxt) and both addresses as little-endian 16-bit words, minus the embedded
 * scopes.  Unfolded. */
static uint64_t
in6_pseudo_sum(const uint8_t *ip6, uint32_t len, uint8_t nxt)
{
	uint64_t s = ((len >> 24) & 0xff) | ((len >> 16) & 0xff) << 8;
	int i;

	s += ((len >> 8) & 0xff) | (len & 0xff) << 8;
	s += (uint64_t)nxt << 8;
	for (i = 0; i < 32; i += 2)
		s += (uint64_t)(ip6[8 + i] | ip6[8 + i + 1] << 8);
	return s - in6_scope_word(ip6 + 8) - in6_scope_word(ip6 + 24);
}

int
oracle_in6_cksum_pseudo(const void *ip6, uint32_t len, uint8_t nxt, uint16_t csum)
{
	/* in6_cksum.c:129-140: REDUCE, not complemented */
	return (int)fold16(in6_pseudo_sum(ip6, len, nxt) + csum);
}

uint16_t
oracle_in6_cksum(const struct oracle_mbuf *m, uint8_t nxt, uint32_t off, uint32_t len)
{
	/* in6_cksum.c:150-357: "m MUST contain a contiguous IP6 header"; off
	 * counts from the chain start, len bytes of transport segment follow. */
	struct walk w = { in6_pseudo_sum((const uint8_t *)m->m_data, len, nxt), 0, (long)len };

	/* :208-214 skip whole mbufs, then :215-219 the rest of the first one */
	while (off > 0 && m) {
		if ((uint32_t)m->m_len <= off) {
			off -= (uint32_t)m->m_len;
			m = m->m_next;
			continue;
		}
		break;
	}
	if (m) {
		take_piece(&w, (const uint8_t *)m->m_data + off, (long)m->m_len - off);
		/* :292-350 the following mbufs, zero-length ones passed over;
		 * running out of data panics there (:351-352) */
		take_rest(&w, m->m_next);
	}
	return (uint16_t)(~fold16(w.sum) & 0xffff);
}

void
oracle_in6_cksum_batch(struct oracle_mbuf *const *m, const uint8_t *nxt,
    const uint32_t *off, const uint32_t *len, uint16_t *out, int n)
{
	int i;

	for (i = 0; i < n; i++)
		out[i] = oracle_in6_cksum(m[i], nxt[i], off[i], len[i]);
}

/* ---- flat batch helpers (what the GPU descriptor APIs compute) ---------- */

static uint16_t
finish(uint64_t sum, uint32_t flags)
{
	uint32_t f = fold16(sum);
	uint16_t r;

	if (flags & ORACLE_F_NO_COMPLEMENT)
		return (uint16_t)f;
	r = (uint16_t)(~f & 0xffff);
	if ((flags & ORACLE_F_UDP) && r == 0)
		r = 0xffff; /* ip_output.c:962-963 */
	return r;
}

void
oracle_spans(const uint8_t *base, const uint64_t *off, const uint32_t *len,
    const uint32_t *seed, const uint8_t *parity, uint16_t *out, uint64_t n,
    uint32_t flags)
{
	for (uint64_t i = 0; i < n; i++) {
		uint64_t s = seed ? seed[i] : 0;

		s += weighted_sum(base + off[i], len[i],
		    parity ? (parity[i] & 1u) : 0u);
		out[i] = finish(s, flags);
	}
}

/* in_cksum_skip over chains given as segment lists (segment k = the bytes
 * base[seg_off[k] .. + seg_len[k]), packet i = segments
 * [pkt_seg[i], pkt_seg[i+1])); len NULL = whole chain, skip NULL = 0.  The
 * walk is in_cksum.c:203-229 with segments in the role of mbufs. */
void
oracle_chains(const uint8_t *base, const uint64_t *seg_off,
    const uint32_t *seg_len, const uint64_t *pkt_seg, const int64_t *len,
    const int64_t *skip, const uint32_t *seed, uint16_t *out, uint64_t n,
    uint32_t flags)
{
	for (uint64_t i = 0; i < n; i++) {
		int64_t sk = skip ? skip[i] : 0;
		int64_t want = len ? len[i] : INT64_MAX / 2;
		struct walk w = { seed ? seed[i] : 0, 0, (long)(want - sk) };
		uint64_t k = pkt_seg[i], end = pkt_seg[i + 1];

		while (sk && k < end) {
			if ((int64_t)seg_len[k] > sk) {
				take_piece(&w, base + seg_off[k] + sk,
				    (long)seg_len[k] - sk);
				k++;
				sk = 0;
				break;
			}
			sk -= seg_len[k];
			k++;
		}
		if (sk == 0) {
			for (; k < end && w.remain; k++) {
				if (seg_len[k] == 0)
					continue;
				take_piece(&w, base + seg_off[k], seg_len[k]);
			}
		}
		out[i] = finish(w.sum, flags);
	}
}

/* ---- threaded per-call batches (tests over large mbuf sets) ------------- */

struct skip_job {
	struct oracle_mbuf *const *m;
	const int *len, *skip;
	uint16_t *out;
	int lo, hi;
};

static void *
skip_worker(void *arg)
{
	struct skip_job *j = arg;

	for (int i = j->lo; i < j->hi; i++)
		j->out[i] = oracle_cksum_skip(j->m[i], j->len[i], j->skip[i]);
	return NULL;
}

void
oracle_cksum_skip_batch(struct oracle_mbuf *const *m, const int *len,
    const int *skip, uint16_t *out, int n, int nthreads)
{
	pthread_t tid[64];
	struct skip_job job[64];

	if (nthreads < 1)
		nthreads = 1;
	if (nthreads > 64)
		nthreads = 64;
	for (int t = 0; t < nthreads; t++) {
		job[t] = (struct skip_job){ m, len, skip, out,
			(int)((long)n * t / nthreads),
			(int)((long)n * (t + 1) / nthreads) };
		pthread_create(&tid[t], NULL, skip_worker, &job[t]);
	}
	for (int t = 0; t < nthreads; t++)
		pthread_join(tid[t], NULL);
}

void
oracle_cksum_pseudo_header_batch(struct oracle_mbuf *const *m,
    const int *plen, const int *off0, const uint32_t *src,
    const uint32_t *dst, const uint8_t *proto, uint16_t *out, int n)
{
	for (int i = 0; i < n; i++)
		out[i] = oracle_cksum_pseudo_header(m[i], plen[i], off0[i],
		    src[i], dst[i], proto[i]);
}

void
oracle_cksum_hdr_batch(const void *const *ip, unsigned *out, int n)
{
	for (int i = 0; i < n; i++)
		out[i] = oracle_cksum_hdr(ip[i]);
}
