// The driver hooks' header parse (SURVEY.md 8f items 1-2, IPv6 with item 4),
// written once for the host (cksum_offload.hip, on the host pool) and the
// device (cksum_hookdev.hip, one lane per packet over registered memory).
//
// Every function reads the packet through a View:
//   uint64_t addr()                 the head mbuf's address (0 = none)
//   int read(off, dst, n)           up to n bytes at chain offset off (count read)
//   const uint8_t* bytes(off, tmp, n, &got)
//                                   the same bytes, in place when the view holds
//                                   them contiguously (first mbuf / window), else
//                                   read into tmp
//   long length()                   the chain's byte count
//   int m_flags(), m_len()          the first mbuf's m_flags / m_len
//   int csum_flags(), csum_data()   its m_pkthdr.csum_flags / csum_data
//   uint32_t take_ip_sum(off)       TX: ip_sum at chain offset off (first mbuf)
//                                   must not count in the header sum: the host
//                                   zeroes it (ip_output.c:665-667) and returns
//                                   seed 0; the device leaves the packet alone
//                                   and returns the seed ~ip_sum that cancels it
// and returns the checksum jobs (in_cksum_skip form, PJob) the GPU folds.
//
//   RX  ip_input.c:460-471 (CSUM_IP_CHECKED / CSUM_IP_VALID),
//       tcp_input.c:697-718 and udp_usrreq.c:404-449 (CSUM_DATA_VALID |
//       CSUM_PSEUDO_HDR); IPv6: tcp_input.c:627-639, udp6_usrreq.c:216-246.
//   TX  ip_output.c:645-667 (deferred ip_sum), :953-976 (in_delayed_cksum);
//       IPv6: ip6_output.c:188-209, :966-988.
#pragma once

#include <stdint.h>
#include <string.h>

#include "uinet_cksum.h"
#include "walk_xlate.h"  // UINET_HD

namespace uinet {
namespace hook {

// sys/sys/mbuf.h:182,281-293; sys/netinet/ip.h:63-65.
constexpr int kMPktHdr = 0x2;
constexpr int kCsumIp = 0x1, kCsumTcp = 0x2, kCsumUdp = 0x4, kCsumTso = 0x20;
constexpr int kCsumUdpIpv6 = 0x2000, kCsumTcpIpv6 = 0x4000;  // mbuf.h:295-296
constexpr int kCsumIpChecked = 0x100, kCsumIpValid = 0x200, kCsumDataValid = 0x400,
              kCsumPseudoHdr = 0x800;
constexpr int kIpMf = 0x2000, kIpOffMask = 0x1fff;

// One checksum job: in_cksum_skip(m, len, skip) plus seed; m == 0: none.
struct PJob {
  uint64_t m;
  int len;
  int skip;
  uint32_t seed;
};

UINET_HD inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
UINET_HD inline uint16_t bswap16(uint16_t x) { return (uint16_t)((x << 8) | (x >> 8)); }
UINET_HD inline uint32_t fold16(uint64_t s) {
  while (s >> 16) s = (s & 0xffff) + (s >> 16);
  return (uint32_t)s;
}

struct Ip4 {
  int l3 = 0;       // chain offset of the IP header
  int hl = 0;       // header length
  int ip_len = 0;   // total length
  int proto = 0;
  bool frag = false;
  uint32_t src = 0, dst = 0;  // as stored (network order read as a native u32)
  uint8_t l4[8] = {};         // first 8 bytes after the IP header (if present)
  int l4_have = 0;
};

// The fixed IPv6 header and the first 8 bytes after it.
struct Ip6 {
  int l3 = 0;
  int plen = 0;  // ip6_plen
  int nxt = 0;
  uint8_t addr[32] = {};  // source, destination
  uint8_t l4[8] = {};
  int l4_have = 0;
};

// Packet k owns jobs 2k (IP header) and 2k + 1 (TCP / UDP).
struct RxPlan {
  bool ip_job = false, l4_job = false;
  uint8_t st = 0;
};

struct TxPlan {
  int ip_l3 = 0;  // chain offset of the IPv4 header (ip_sum at +10)
  bool ip_job = false, l4_job = false;
  int l4_store = 0;  // chain offset of th_sum / uh_sum
  bool udp = false;
  int clear = 0;  // csum_flags bits the hook takes over
  uint8_t st = 0;
};

// The network header's offset and IP version (4 or 6; 0 = neither).
// l2len -1: Ethernet (0x0800 / 0x86dd, or one 802.1Q tag first); l2len >= 0:
// the header sits at l2len and its version nibble tells.
template <class V>
UINET_HD int l3_locate(const V& v, int l2len, int* l3) {
  uint8_t t[18];
  int got = 0;
  if (l2len >= 0) {
    *l3 = l2len;
    const uint8_t* b = v.bytes(l2len, t, 1, &got);
    if (got < 1) return 0;
    return (b[0] >> 4) == 4 ? 4 : (b[0] >> 4) == 6 ? 6 : 0;
  }
  const uint8_t* b = v.bytes(0, t, 18, &got);
  if (got < 14) return 0;
  uint16_t et = be16(b + 12);
  *l3 = 14;
  if (et == 0x8100) {
    if (got < 18) return 0;
    et = be16(b + 16);
    *l3 = 18;
  }
  return et == 0x0800 ? 4 : et == 0x86dd ? 6 : 0;
}

// The header, and with want_l4 the first 8 bytes after it (RX's UDP checks;
// TX never looks at them).  Reads no byte it does not use: past the first
// mbuf the device view pays two more host lines per frame (the next mbuf's
// header and data), so the header length is read first.
template <class V>
UINET_HD bool parse_ip4(const V& v, int l3, Ip4* o, bool want_l4) {
  uint8_t t[60 + 8];
  int got = 0;
  const uint8_t* b = v.bytes(l3, t, 20, &got);
  if (got < 20 || (b[0] >> 4) != 4) return false;
  const int hl = (b[0] & 15) * 4;
  if (hl < 20) return false;
  if (hl + (want_l4 ? 8 : 0) > 20) b = v.bytes(l3, t, hl + (want_l4 ? 8 : 0), &got);
  if (got < hl) return false;
  o->l3 = l3;
  o->hl = hl;
  o->ip_len = be16(b + 2);
  o->frag = (be16(b + 6) & (kIpMf | kIpOffMask)) != 0;
  o->proto = b[9];
  memcpy(&o->src, b + 12, 4);
  memcpy(&o->dst, b + 16, 4);
  o->l4_have = got - hl < 8 ? got - hl : 8;
  for (int i = 0; i < o->l4_have; i++) o->l4[i] = b[hl + i];
  return true;
}

template <class V>
UINET_HD bool parse_ip6(const V& v, int l3, Ip6* o, bool want_l4) {
  uint8_t t[40 + 8];
  int got = 0;
  const uint8_t* b = v.bytes(l3, t, 40 + (want_l4 ? 8 : 0), &got);
  if (got < 40 || (b[0] >> 4) != 6) return false;
  o->l3 = l3;
  o->plen = be16(b + 4);
  o->nxt = b[6];
  for (int i = 0; i < 32; i++) o->addr[i] = b[8 + i];
  o->l4_have = got - 40;
  for (int i = 0; i < o->l4_have; i++) o->l4[i] = b[40 + i];
  return true;
}

// A link-local unicast, or link- / interface-local multicast, address whose
// second 16-bit word (KAME's embedded zone) is nonzero.  ip6_input drops such
// packets before any transport input (ip6_input.c:658-661, "badscope"), so
// the RX hook leaves them unmarked.
UINET_HD inline bool ip6_zone_embedded(const uint8_t* a) {
  const bool ll = a[0] == 0xfe && (a[1] & 0xc0) == 0x80;
  const bool mc = a[0] == 0xff && ((a[1] & 0x0f) == 0x02 || (a[1] & 0x0f) == 0x01);
  return (ll || mc) && (a[2] | a[3]) != 0;
}

// The extension headers between the fixed IPv6 header and the transport, as
// the stack walks them: hop-by-hop only first (ip6_input.c:906-913), then the
// next-header loop (:986-1019) through destination options (dest6.c:62-123)
// and routing headers (route6.c:59-108: segments left 0 is skipped, anything
// else dropped on receive).  The loop counts every header it handles, the
// transport included, against ip6_hdrnestlimit = 15 (:986-990,
// in6_proto.c:406); hop-by-hop is handled before the loop and does not count,
// so a packet may carry hop-by-hop + 14 more headers + the transport.  A
// fragment header (frag6.c:165) stops the walk: the stack reassembles first.
// Returns 1 with *off (the transport header's offset from the IPv6 header)
// and *nxt at the first other header, 0 at a fragment header, -1 when the
// stack would drop the packet or the walk leaves the payload (ip6_plen).
template <class V>
UINET_HD int ip6_walk(const V& v, const Ip6& ip, bool rx, int* off, int* nxt) {
  int o = 40, x = ip.nxt;
  const int lim = x == 0 ? 16 : 15;  // + the uncounted hop-by-hop header
  for (int k = 0; k < lim; k++) {
    if (x == 0 && k != 0) return -1;  // hop-by-hop after the first header
    if (x != 0 && x != 43 && x != 60) {
      if (o > 40 + ip.plen) return -1;
      *off = o;
      *nxt = x;
      return x == 44 ? 0 : 1;
    }
    if (o + 8 > 40 + ip.plen) return -1;
    uint8_t t[4];
    int got = 0;
    const uint8_t* e = v.bytes(ip.l3 + o, t, 4, &got);
    if (got < 4) return -1;
    if (rx && x == 43 && e[3] != 0) return -1;  // segments left: route6.c:99-105
    x = e[0];
    o += (e[1] + 1) * 8;
  }
  return -1;
}

// in6_cksum.c:86-126 for wire addresses (no embedded zone): htonl(len),
// three zero bytes and the transport's nxt, then both addresses, as
// little-endian 16-bit words; folded so it fits a job seed.
UINET_HD inline uint32_t pseudo6_seed(const Ip6& ip, uint32_t len, int nxt) {
  uint64_t s = (uint64_t)bswap16((uint16_t)(len >> 16)) + bswap16((uint16_t)len) +
               bswap16((uint16_t)nxt);
  for (int i = 0; i < 32; i += 2) s += (uint64_t)(ip.addr[i] | ip.addr[i + 1] << 8);
  return fold16(s);
}

// in_cksum.c:252-253, folded so it fits a job seed.
UINET_HD inline uint32_t pseudo_seed(uint32_t src, uint32_t dst, int proto, int plen) {
  return fold16((uint64_t)src + dst + bswap16((uint16_t)proto) + bswap16((uint16_t)plen));
}

// RX IPv6: tcp_input.c:627-639 (tlen = 40 + ip6_plen - off0, the transport
// after the extension headers) and udp6_usrreq.c:216-246 (uh_ulen must equal
// that length, uh_sum 0 is an error).  Returns the L4 job, or m == 0 for none.
template <class V>
UINET_HD PJob rx6_job(const V& v, const Ip6& ip, uint8_t* st) {
  const PJob none{0, 0, 0, 0u};
  int off = 40, nxt = ip.nxt;
  const int w = ip.plen ? ip6_walk(v, ip, true, &off, &nxt) : -1;
  if (w == 0 || ip.nxt == 44) *st |= UINET_RX_FRAG;
  if (w != 1) return none;
  if (v.length() < (long)ip.l3 + 40 + ip.plen) return none;  // ip6s_tooshort
  if (ip6_zone_embedded(ip.addr) || ip6_zone_embedded(ip.addr + 16)) return none;
  const int tlen = 40 + ip.plen - off;
  if (nxt == 17) {
    uint8_t u[8];
    const uint8_t* uh = ip.l4;
    if (off != 40) {
      int got = 0;
      uh = v.bytes(ip.l3 + off, u, 8, &got);
      if (got < 8) return none;
    } else if (ip.l4_have < 8) {
      return none;
    }
    if (be16(uh + 4) != tlen) return none;  // udps_badlen
    if (be16(uh + 6) == 0) {                // udps_nosum
      *st |= UINET_RX_NOSUM;
      return none;
    }
  } else if (nxt != 6) {
    return none;
  }
  return PJob{v.addr(), ip.l3 + 40 + ip.plen, ip.l3 + off, pseudo6_seed(ip, (uint32_t)tlen, nxt)};
}

// RX: ip_input.c:460-471, tcp_input.c:697-718, udp_usrreq.c:404-449 and the
// IPv6 forms (rx6_job).  Returns the IP-header job; the L4 job goes to *l4.
template <class V>
UINET_HD PJob rx_parse(const V& v, int l2len, RxPlan& p, PJob* l4) {
  const PJob none{0, 0, 0, 0u};
  p = RxPlan();
  *l4 = none;
  int l3 = 0;
  const int ver = v.addr() ? l3_locate(v, l2len, &l3) : 0;
  if (ver == 6) {
    Ip6 ip6;
    if (!parse_ip6(v, l3, &ip6, true)) return none;
    p.st |= UINET_RX_IPV6;
    const PJob j = rx6_job(v, ip6, &p.st);
    if (j.m) {
      p.l4_job = true;
      *l4 = j;
    }
    return none;
  }
  Ip4 ip;
  if (ver != 4 || !parse_ip4(v, l3, &ip, true)) return none;
  p.st |= UINET_RX_IPV4;
  p.ip_job = true;  // in_cksum(m, hlen) over the header (ip_input.c:463-467)
  const PJob hdr{v.addr(), ip.l3 + ip.hl, ip.l3, 0u};
  if (ip.frag) {
    p.st |= UINET_RX_FRAG;
    return hdr;
  }
  if (ip.ip_len < ip.hl || v.length() < (long)ip.l3 + ip.ip_len) return hdr;
  int plen = ip.ip_len - ip.hl;
  if (ip.proto == 6) {  // tcp_input.c:711-713: tlen = ip_len - off0
  } else if (ip.proto == 17) {
    if (ip.l4_have < 8) return hdr;
    if (be16(ip.l4 + 6) == 0) {  // uh_sum 0: no checksum (udp_usrreq.c:427,450)
      p.st |= UINET_RX_NOSUM;
      return hdr;
    }
    const int ulen = be16(ip.l4 + 4);  // udp_usrreq.c:404-412
    if (ulen > plen || ulen < 8) return hdr;
    plen = ulen;
  } else {
    return hdr;
  }
  p.l4_job = true;
  *l4 = PJob{v.addr(), ip.l3 + ip.hl + plen, ip.l3 + ip.hl,
             pseudo_seed(ip.src, ip.dst, ip.proto, plen)};
  return hdr;
}

// TX: ip_output.c:645-667,953-976 and ip6_output.c:188-209,966-988.  ip_sum
// does not count in the header job (take_ip_sum, above).
template <class V>
UINET_HD PJob tx_parse(V& v, int l2len, TxPlan& p, PJob* l4) {
  const PJob none{0, 0, 0, 0u};
  p = TxPlan();
  *l4 = none;
  if (!v.addr() || !(v.m_flags() & kMPktHdr)) {
    p.st = UINET_TX_SKIP;
    return none;
  }
  const int fl = v.csum_flags();
  int l3 = 0;
  const int ver = (fl & kCsumTso) ? 0 : l3_locate(v, l2len, &l3);
  if (ver == 6) {  // in6_delayed_cksum, ip6_output.c:188-209,978-981
    // As an offloading NIC must (ip6_output.c:966-981 leaves CSUM_*_IPV6 to a
    // driver that advertises it, extension headers or not), the transport is
    // found past the extension headers; the seed already in its checksum
    // field holds the final destination.
    Ip6 ip6;
    int off = 40, nxt = 0;
    if (!(fl & (kCsumTcpIpv6 | kCsumUdpIpv6)) || !parse_ip6(v, l3, &ip6, false) || ip6.plen == 0 ||
        ip6_walk(v, ip6, false, &off, &nxt) != 1) {
      p.st = UINET_TX_SKIP;
      return none;
    }
    p.st = UINET_TX_IPV6;
    p.udp = (fl & kCsumUdpIpv6) != 0;
    p.clear = kCsumTcpIpv6 | kCsumUdpIpv6;
    p.l4_store = l3 + off + v.csum_data();
    p.l4_job = true;
    *l4 = PJob{v.addr(), l3 + 40 + ip6.plen, l3 + off, 0u};
    return none;
  }
  Ip4 ip;
  if (ver != 4 || !(fl & (kCsumIp | kCsumTcp | kCsumUdp)) || !parse_ip4(v, l3, &ip, false)) {
    p.st = UINET_TX_SKIP;
    return none;
  }
  if ((fl & kCsumIp) && ip.l3 + 12 > v.m_len()) {
    p.st = UINET_TX_SKIP;  // header not in the first mbuf: leave it to the stack
    return none;
  }
  if (fl & (kCsumTcp | kCsumUdp)) {  // in_delayed_cksum, ip_output.c:958-963
    p.udp = (fl & kCsumUdp) != 0;
    p.clear = kCsumTcp | kCsumUdp;
    p.l4_store = ip.l3 + ip.hl + v.csum_data();
    p.l4_job = true;
    *l4 = PJob{v.addr(), ip.l3 + ip.ip_len, ip.l3 + ip.hl, 0u};
  }
  if (fl & kCsumIp) {  // ip_output.c:665-667: ip_sum = 0, then in_cksum(m, hlen)
    const uint32_t seed = v.take_ip_sum(ip.l3 + 10);
    p.ip_l3 = ip.l3;
    p.ip_job = true;
    return PJob{v.addr(), ip.l3 + ip.hl, ip.l3, seed};
  }
  return none;
}

}  // namespace hook
}  // namespace uinet
