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
 * IPv6 frames (Ethernet type 0x86dd, or version 6 at l2len) go the IPv6 way:
 *   RX  sys/netinet6/ip6_input.c          short chains and embedded zones
 *                                         (:658-661) are dropped; hop-by-hop
 *                                         options first (:906-913), then the
 *                                         next-header loop (:986-1019):
 *       sys/netinet6/dest6.c:62-123       destination options skipped
 *       sys/netinet6/route6.c:59-108      routing header skipped when its
 *                                         segments left is 0, else dropped
 *       sys/netinet6/frag6.c:165          reassembly first (no verdict here)
 *       sys/netinet/tcp_input.c:627-639   th_sum = in6_cksum(m, TCP, off0,
 *                                         40 + ip6_plen - off0)
 *       sys/netinet6/udp6_usrreq.c:216-246 uh_ulen == that length, uh_sum
 *                                         != 0, in6_cksum(m, UDP, off, ulen)
 *     with the same CSUM_DATA_VALID(_IPV6) | CSUM_PSEUDO_HDR marks;
 *   TX  sys/netinet6/ip6_output.c:188-209,966-981  in6_delayed_cksum(m,
 *                                         transport length, transport offset)
 *                                         -- the transport found past the
 *                                         extension headers, as a NIC that
 *                                         advertises CSUM_*_IPV6 must
 *
 * Chains whose link header reaches past the first mbuf are viewed through
 * a private copy of their mbuf headers (what m_adj would leave), and RX
 * transport sums see the chain the way the stack's m_pullup calls leave it:
 * headers contiguous in the first mbuf (pulled_up, below).
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
#define O_CSUM_UDP_IPV6 0x2000
#define O_CSUM_TCP_IPV6 0x4000

/* status bits, as include/uinet_cksum.h defines them */
#define S_RX_IPV4 0x01
#define S_RX_IP_OK 0x02
#define S_RX_L4 0x04
#define S_RX_L4_OK 0x08
#define S_RX_NOSUM 0x10
#define S_RX_FRAG 0x20
#define S_RX_IPV6 0x40
#define S_TX_L4 0x01
#define S_TX_IP 0x02
#define S_TX_L4_LOST 0x04
#define S_TX_SKIP 0x08
#define S_TX_IPV6 0x10

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

/*
 * The chain as the transport's checksum sees it after the stack's pull-ups:
 * ip_input.c:426,443 (the IP header), tcp_input.c:686 (IP header + TCP
 * header), udp_usrreq.c:378 (+ UDP header), ip6_input.c:519 and
 * IP6_EXTHDR_CHECK at tcp_input.c:535 / udp6_usrreq.c:200 (IPv6 header
 * through the transport header) make the first `need` bytes contiguous before
 * in_cksum_pseudo_header / in6_cksum read the headers from the first mbuf.
 * When the first mbuf is shorter, the chain is viewed as one contiguous copy
 * in `one` (m_pullup moves only the first `need` bytes; the sums do not see
 * the difference); *buf is the caller's to free.
 */
static const struct oracle_mbuf *
pulled_up(const struct oracle_mbuf *ipm, int need, struct oracle_mbuf *one, uint8_t **buf)
{
	long total;

	*buf = NULL;
	if (ipm->m_len >= need)
		return ipm;
	total = chain_total(ipm);
	*buf = malloc(total > 0 ? (size_t)total : 1);
	chain_bytes(ipm, 0, *buf, (int)total);
	*one = *ipm;
	one->m_next = NULL;
	one->m_data = (char *)*buf;
	one->m_len = (int)total;
	return one;
}

/* Offset of the network header (l2len -1: Ethernet, optional 802.1Q), or -1;
 * *ver = 4 or 6 (ether_demux's type switch, or the version nibble at l2len). */
static int
ip_offset(const struct oracle_mbuf *m, int l2len, int *ver)
{
	uint8_t e[18];
	int got, type, l3 = 14;

	*ver = 0;
	if (l2len >= 0) {
		if (chain_bytes(m, l2len, e, 1) < 1)
			return -1;
		*ver = e[0] >> 4;
		return (*ver == 4 || *ver == 6) ? l2len : -1;
	}
	got = chain_bytes(m, 0, e, 18);
	if (got < 14)
		return -1;
	type = e[12] << 8 | e[13];
	if (type == 0x8100) {
		if (got < 18)
			return -1;
		type = e[16] << 8 | e[17];
		l3 = 18;
	}
	*ver = type == 0x0800 ? 4 : type == 0x86dd ? 6 : 0;
	return *ver ? l3 : -1;
}

/* in6_clearscope's test (ip6_input.c:658): a link-local unicast or link- /
 * interface-local multicast address with a nonzero zone word. */
static int
zone_embedded(const uint8_t *a)
{
	int ll = a[0] == 0xfe && (a[1] & 0xc0) == 0x80;
	int mc = a[0] == 0xff && ((a[1] & 0x0f) == 0x02 || (a[1] & 0x0f) == 0x01);

	return (ll || mc) && (a[2] || a[3]);
}

/*
 * The header chain after the fixed IPv6 header of `ipm` (m_data at the IPv6
 * header, payload length plen): hop-by-hop (0) only as the first header,
 * destination options (60) and routing (43) headers are (len + 1) * 8 bytes,
 * a routing header with segments left is dropped on receive, at most 15
 * headers after hop-by-hop (the transport included).  Returns 1 and the transport's offset / protocol, 0 at a fragment
 * header (44), -1 for a dropped packet.
 */
static int
walk6(const struct oracle_mbuf *ipm, int plen, int first, int rx, int *off, int *nxt)
{
	int o = 40, x = first, k;
	/* ip6_input.c:986-990 counts the loop's headers (transport included)
	 * against ip6_hdrnestlimit (15, in6_proto.c:406); hop-by-hop (:906-913)
	 * runs before the loop and does not count */
	int lim = x == 0 ? 16 : 15;
	uint8_t e[4];

	for (k = 0; k < lim; k++) {
		if (x == 0 && k > 0)
			return -1;
		if (x == 44) {
			*off = o;
			*nxt = x;
			return o <= 40 + plen ? 0 : -1;
		}
		if (x != 0 && x != 60 && x != 43) {
			if (o > 40 + plen)
				return -1;
			*off = o;
			*nxt = x;
			return 1;
		}
		if (o + 8 > 40 + plen || chain_bytes(ipm, o, e, 4) < 4)
			return -1;
		if (rx && x == 43 && e[3] != 0)
			return -1;	/* route6.c:99-105 */
		x = e[0];
		o += 8 * (e[1] + 1);
	}
	return -1;
}

/* One received IPv6 frame, m_data at the IPv6 header in `ipm`. */
static uint8_t
rx6(struct oracle_mbuf *m, struct oracle_mbuf *ipm, const uint8_t *h, int got, long avail)
{
	uint8_t st = S_RX_IPV6, u[8];
	int plen = h[4] << 8 | h[5], nxt = h[6], off = 40, w = -1, tlen, sum;

	(void)got;
	if (plen)
		w = walk6(ipm, plen, h[6], 1, &off, &nxt);
	if (w == 0 || h[6] == 44)
		st |= S_RX_FRAG;	/* frag6_input reassembles first */
	if (w != 1 || avail < 40 + (long)plen)
		return st;		/* dropped, jumbogram (hop-by-hop), ip6s_tooshort */
	if (zone_embedded(h + 8) || zone_embedded(h + 24))
		return st;		/* ip6s_badscope */
	tlen = 40 + plen - off;
	if (nxt == 17) {
		if (chain_bytes(ipm, off, u, 8) < 8 || (u[4] << 8 | u[5]) != tlen)
			return st;	/* udps_badlen */
		if ((u[6] | u[7]) == 0)
			return st | S_RX_NOSUM;
	} else if (nxt != 6) {
		return st;
	}
	{
		struct oracle_mbuf one;
		uint8_t *buf;
		const struct oracle_mbuf *p = pulled_up(ipm, off + (nxt == 6 ? 20 : 8), &one, &buf);

		sum = oracle_in6_cksum(p, (uint8_t)nxt, (uint32_t)off, (uint32_t)tlen);
		free(buf);
	}
	st |= S_RX_L4 | (sum == 0 ? S_RX_L4_OK : 0);
	if (m->m_flags & O_M_PKTHDR) {
		*csum_flags(m) |= O_CSUM_DATA_VALID | O_CSUM_PSEUDO_HDR;
		*csum_data(m) = sum ^ 0xffff;
	}
	return st;
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
		int ver;

		if (!m || (l3 = ip_offset(m, l2len, &ver)) < 0)
			goto done;
		got = chain_bytes(m, l3, h, (int)sizeof(h));
		if (ver == 6) {
			if (got < 40 || (h[0] >> 4) != 6)
				goto done;
			ipm = adj_view(m, l3, &tmp);
			st = rx6(m, ipm, h, got, chain_total(m) - l3);
			goto done;
		}
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
			struct oracle_mbuf one;
			uint8_t *buf;
			const struct oracle_mbuf *p = pulled_up(ipm, hlen + 20, &one, &buf);

			sum = oracle_cksum_pseudo_header(p, ip_len - hlen, hlen, src, dst, 6);
			free(buf);
		} else if (proto == 17) {
			struct oracle_mbuf one;
			uint8_t *buf;
			const struct oracle_mbuf *p;
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
			p = pulled_up(ipm, hlen + 8, &one, &buf);
			sum = oracle_cksum_pseudo_header(p, ulen, hlen, src, dst, 17);
			free(buf);
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
		uint8_t h[40], st = 0;
		int l3, hlen, ip_len, fl, ver = 0;

		if (!m || !(m->m_flags & O_M_PKTHDR)) {
			st = S_TX_SKIP;
			goto done;
		}
		fl = *csum_flags(m);
		if (!(fl & O_CSUM_TSO) && (l3 = ip_offset(m, l2len, &ver)) >= 0 && ver == 6) {
			/* in6_delayed_cksum(m, transport length, transport offset) */
			uint16_t csum;
			int plen, offset, l4 = 40, nxt;

			if (!(fl & (O_CSUM_TCP_IPV6 | O_CSUM_UDP_IPV6)) ||
			    chain_bytes(m, l3, h, 40) < 40 || (h[0] >> 4) != 6 ||
			    (plen = h[4] << 8 | h[5]) == 0) {
				st = S_TX_SKIP;
				goto done;
			}
			ipm = adj_view(m, l3, &tmp);
			if (walk6(ipm, plen, h[6], 0, &l4, &nxt) != 1) {
				st = S_TX_SKIP;
				goto done;
			}
			csum = oracle_cksum_skip(ipm, 40 + plen, l4);
			if ((fl & O_CSUM_UDP_IPV6) && csum == 0)
				csum = 0xffff;
			offset = l4 + *csum_data(m);
			st = S_TX_IPV6;
			if (offset + 2 > ipm->m_len) {
				st |= S_TX_L4_LOST;
			} else {
				memcpy(ipm->m_data + offset, &csum, 2);
				st |= S_TX_L4;
			}
			*csum_flags(m) &= ~(O_CSUM_TCP_IPV6 | O_CSUM_UDP_IPV6);
			goto done;
		}
		if ((fl & O_CSUM_TSO) || !(fl & (O_CSUM_IP | O_CSUM_TCP | O_CSUM_UDP)) ||
		    ver != 4 || chain_bytes(m, l3, h, 20) < 20 ||
		    (h[0] >> 4) != 4 || (hlen = (h[0] & 15) << 2) < 20 ||
		    chain_total(m) - l3 < hlen) {
			/* a header the chain cuts short is left alone (the stack
			 * never builds one; in_cksum would sum what is there) */
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
