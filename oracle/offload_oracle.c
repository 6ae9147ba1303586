/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see cksum_oracle.c).
 *
 * CPU restatement of the driver batch offload hooks of include/uinet_cksum.h
 * section 2d, written as the software stack itself would proceed, one packet
 * at a time, with the oracle's in_cksum_* (pinned to the reference object):
 *
 *   RX  ether_input strips the link header (m_adj), then
 *       sys/netinet/ip_input.c:460-471    header sum: in_cksum_hdr when
 *                                         hlen == 20, else in_cksum(m, hlen)
 *       sys/netinet/tcp_input.c:697-718   th_sum = in_cksum_pseudo_header(m,
 *                                         ip_len - off0, off0, src, dst, TCP)
 *       sys/netinet/udp_usrreq.c:404-449  uh_ulen checks, then the same over
 *                                         uh_ulen bytes when uh_sum != 0
 *     and records each verdict the way the offloaded stack reads it back:
 *     CSUM_IP_CHECKED (| CSUM_IP_VALID), CSUM_DATA_VALID | CSUM_PSEUDO_HDR
 *     with csum_data = sum ^ 0xffff.
 *   TX  sys/netinet/ip_output.c:953-976   in_delayed_cksum
 *       sys/netinet/ip_output.c:665-667   ip_sum = 0; ip_sum = in_cksum(m, hlen)
 *
 * Chains whose link header reaches past the first mbuf are viewed through
 * a private copy of their mbuf headers (what m_adj would leave).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cksum_oracle.h"

#define O_M_PKTHDR 0x2
#define O_CSUM_IP 0x1
#define O_CSUM_TCP 0x2
#define O_CSUM_UDP 0x4
#define O_CSUM_TSO 0x20
#define O_CSUM_IP_CHECKED 0x100
#define O_CSUM_IP_VALID 0x200
#define O_CSUM_DATA_VALID 0x400
#define O_CSUM_PSEUDO_HDR 0x800

/* status bits, as include/uinet_cksum.h defines them */
#define S_RX_IPV4 0x01
#define S_RX_IP_OK 0x02
#define S_RX_L4 0x04
#define S_RX_L4_OK 0x08
#define S_RX_NOSUM 0x10
#define S_RX_FRAG 0x20
#define S_TX_L4 0x01
#define S_TX_IP 0x02
#define S_TX_L4_LOST 0x04
#define S_TX_SKIP 0x08

/* struct pkthdr's checksum fields (sys/sys/mbuf.h:116-133) */
static int *
csum_flags(struct oracle_mbuf *m)
{
	return (int *)((char *)m + 64);
}

static int *
csum_data(struct oracle_mbuf *m)
{
	return (int *)((char *)m + 68);
}

/* The chain with its first `off` bytes trimmed (m_adj), in `tmp`. */
static struct oracle_mbuf *
adj_view(const struct oracle_mbuf *m, int off, struct oracle_mbuf **tmp)
{
	int n = 0, i;
	const struct oracle_mbuf *p;
	struct oracle_mbuf *v;

	for (p = m; p; p = p->m_next)
		n++;
	v = calloc((size_t)n, sizeof(*v));
	for (i = 0, p = m; p; p = p->m_next, i++) {
		v[i] = *p;
		v[i].m_next = p->m_next ? &v[i + 1] : NULL;
		if (off > 0 && v[i].m_len > 0) {
			int k = off < v[i].m_len ? off : v[i].m_len;
			v[i].m_data += k;
			v[i].m_len -= k;
			off -= k;
		}
	}
	*tmp = v;
	return v;
}

static int
chain_bytes(const struct oracle_mbuf *m, int off, uint8_t *dst, int n)
{
	int got = 0;

	for (; m && got < n; m = m->m_next) {
		int l = m->m_len, k;
		if (l <= 0)
			continue;
		if (off >= l) {
			off -= l;
			continue;
		}
		k = l - off < n - got ? l - off : n - got;
		memcpy(dst + got, m->m_data + off, (size_t)k);
		got += k;
		off = 0;
	}
	return got;
}

static long
chain_total(const struct oracle_mbuf *m)
{
	long t = 0;

	for (; m; m = m->m_next)
		if (m->m_len > 0)
			t += m->m_len;
	return t;
}

/* Offset of the IPv4 header (l2len -1: Ethernet, optional 802.1Q), or -1. */
static int
ip_offset(const struct oracle_mbuf *m, int l2len)
{
	uint8_t e[18];
	int got, type;

	if (l2len >= 0)
		return l2len;
	got = chain_bytes(m, 0, e, 18);
	if (got < 14)
		return -1;
	type = e[12] << 8 | e[13];
	if (type == 0x8100) {
		if (got < 18)
			return -1;
		type = e[16] << 8 | e[17];
		if (type == 0x0800)
			return 18;
		return -1;
	}
	return type == 0x0800 ? 14 : -1;
}

void
oracle_rx_offload(struct oracle_mbuf *const *mv, int n, int l2len, uint8_t *status)
{
	int i;

	for (i = 0; i < n; i++) {
		struct oracle_mbuf *m = mv[i], *tmp = NULL, *ipm;
		uint8_t h[60 + 8], st = 0;
		int l3, got, hlen, ip_len, frag, proto, sum;
		uint32_t src, dst;

		if (!m || (l3 = ip_offset(m, l2len)) < 0)
			goto done;
		got = chain_bytes(m, l3, h, (int)sizeof(h));
		if (got < 20 || (h[0] >> 4) != 4)
			goto done;
		hlen = (h[0] & 15) << 2;
		if (hlen < 20 || got < hlen)
			goto done;
		st |= S_RX_IPV4;
		ipm = adj_view(m, l3, &tmp);
		if (hlen == 20 && ipm->m_len >= 20)
			sum = (int)oracle_cksum_hdr(ipm->m_data);
		else
			sum = oracle_cksum_skip(ipm, hlen, 0);
		if (sum == 0)
			st |= S_RX_IP_OK;
		if (m->m_flags & O_M_PKTHDR)
			*csum_flags(m) |= O_CSUM_IP_CHECKED | (sum == 0 ? O_CSUM_IP_VALID : 0);
		ip_len = h[2] << 8 | h[3];
		frag = ((h[6] << 8 | h[7]) & 0x3fff) != 0;
		proto = h[9];
		memcpy(&src, h + 12, 4);
		memcpy(&dst, h + 16, 4);
		if (frag) {
			st |= S_RX_FRAG;
			goto done;
		}
		if (ip_len < hlen || chain_total(m) < (long)l3 + ip_len)
			goto done;
		if (proto == 6) {
			sum = oracle_cksum_pseudo_header(ipm, ip_len - hlen, hlen, src, dst, 6);
		} else if (proto == 17) {
			int ulen;
			if (got < hlen + 8)
				goto done;
			if ((h[hlen + 6] | h[hlen + 7]) == 0) {
				st |= S_RX_NOSUM;
				goto done;
			}
			ulen = h[hlen + 4] << 8 | h[hlen + 5];
			if (ulen > ip_len - hlen || ulen < 8)
				goto done;
			sum = oracle_cksum_pseudo_header(ipm, ulen, hlen, src, dst, 17);
		} else {
			goto done;
		}
		st |= S_RX_L4 | (sum == 0 ? S_RX_L4_OK : 0);
		if (m->m_flags & O_M_PKTHDR) {
			*csum_flags(m) |= O_CSUM_DATA_VALID | O_CSUM_PSEUDO_HDR;
			*csum_data(m) = sum ^ 0xffff;
		}
done:
		free(tmp);
		if (status)
			status[i] = st;
	}
}

void
oracle_tx_offload(struct oracle_mbuf *const *mv, int n, int l2len, uint8_t *status)
{
	int i;

	for (i = 0; i < n; i++) {
		struct oracle_mbuf *m = mv[i], *tmp = NULL, *ipm;
		uint8_t h[20], st = 0;
		int l3, hlen, ip_len, fl;

		if (!m || !(m->m_flags & O_M_PKTHDR)) {
			st = S_TX_SKIP;
			goto done;
		}
		fl = *csum_flags(m);
		if ((fl & O_CSUM_TSO) || !(fl & (O_CSUM_IP | O_CSUM_TCP | O_CSUM_UDP)) ||
		    (l3 = ip_offset(m, l2len)) < 0 || chain_bytes(m, l3, h, 20) < 20 ||
		    (h[0] >> 4) != 4 || (hlen = (h[0] & 15) << 2) < 20) {
			st = S_TX_SKIP;
			goto done;
		}
		if ((fl & O_CSUM_IP) && l3 + 12 > m->m_len) {
			st = S_TX_SKIP;
			goto done;
		}
		ip_len = h[2] << 8 | h[3];
		ipm = adj_view(m, l3, &tmp);
		if (fl & (O_CSUM_TCP | O_CSUM_UDP)) {
			/* in_delayed_cksum, ip_output.c:953-976 */
			uint16_t csum = oracle_cksum_skip(ipm, ip_len, hlen);
			int offset = hlen + *csum_data(m);
			if ((fl & O_CSUM_UDP) && csum == 0)
				csum = 0xffff;
			if (offset + 2 > ipm->m_len) {
				st |= S_TX_L4_LOST;
			} else {
				memcpy(ipm->m_data + offset, &csum, 2);
				st |= S_TX_L4;
			}
			*csum_flags(m) &= ~(O_CSUM_TCP | O_CSUM_UDP);
		}
		if (fl & O_CSUM_IP) {
			/* ip_output.c:665-667 */
			uint16_t s;
			memset(ipm->m_data + 10, 0, 2);
			s = oracle_cksum_skip(ipm, hlen, 0);
			memcpy(ipm->m_data + 10, &s, 2);
			st |= S_TX_IP;
			*csum_flags(m) &= ~O_CSUM_IP;
		}
done:
		free(tmp);
		if (status)
			status[i] = st;
	}
}
