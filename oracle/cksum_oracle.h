/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see cksum_oracle.c).
 */
#ifndef CKSUM_ORACLE_H
#define CKSUM_ORACLE_H

#include <stdint.h>

/* Layout-compatible with the fields the reference reads from struct mbuf
 * (sys/sys/mbuf.h:90-98,153-171): m_next@0, m_data@16, m_len@24; MSIZE 256
 * (sys/sys/param.h:159). */
struct oracle_mbuf {
	struct oracle_mbuf *m_next;
	struct oracle_mbuf *m_nextpkt;
	char *m_data;
	int m_len;
	int m_flags;
	short m_type;
	char m_pad[256 - 34];
};

#define ORACLE_F_UDP           0x1u /* map a 0 result to 0xffff */
#define ORACLE_F_NO_COMPLEMENT 0x2u /* return the folded sum      */

uint16_t oracle_cksum_skip(const struct oracle_mbuf *m, int len, int skip);
uint16_t oracle_cksum_pseudo_header(const struct oracle_mbuf *m, int plen,
    int off0, uint32_t src, uint32_t dst, uint8_t proto);
unsigned oracle_cksum_hdr(const void *ip);
uint16_t oracle_in_pseudo(uint32_t a, uint32_t b, uint32_t c);
uint16_t oracle_in_addword(uint16_t a, uint16_t b);

void oracle_spans(const uint8_t *base, const uint64_t *off,
    const uint32_t *len, const uint32_t *seed, const uint8_t *parity,
    uint16_t *out, uint64_t n, uint32_t flags);
void oracle_chains(const uint8_t *base, const uint64_t *seg_off,
    const uint32_t *seg_len, const uint64_t *pkt_seg, const int64_t *len,
    const int64_t *skip, const uint32_t *seed, uint16_t *out, uint64_t n,
    uint32_t flags);
void oracle_cksum_skip_batch(struct oracle_mbuf *const *m, const int *len,
    const int *skip, uint16_t *out, int n, int nthreads);
void oracle_cksum_pseudo_header_batch(struct oracle_mbuf *const *m,
    const int *plen, const int *off0, const uint32_t *src,
    const uint32_t *dst, const uint8_t *proto, uint16_t *out, int n);
void oracle_cksum_hdr_batch(const void *const *ip, unsigned *out, int n);

/* IPv6: sys/netinet6/in6_cksum.c */
uint16_t oracle_in6_cksum(const struct oracle_mbuf *m, uint8_t nxt, uint32_t off,
    uint32_t len);
int oracle_in6_cksum_pseudo(const void *ip6, uint32_t len, uint8_t nxt, uint16_t csum);
void oracle_in6_cksum_batch(struct oracle_mbuf *const *m, const uint8_t *nxt,
    const uint32_t *off, const uint32_t *len, uint16_t *out, int n);

/* offload_oracle.c: the driver batch offload hooks, restated packet by
 * packet (mutates pkthdr csum fields, and packet bytes on TX). */
void oracle_rx_offload(struct oracle_mbuf *const *m, int n, int l2len,
    uint8_t *status);
void oracle_tx_offload(struct oracle_mbuf *const *m, int n, int l2len,
    uint8_t *status);

#endif
