// Driver batch offload (SURVEY.md 8f items 1-2, IPv6 with item 4): whole RX /
// TX batches of IPv4 and IPv6 packets checksummed in one GPU batch, with the
// results recorded the way the stack consumes a checksum-offloading NIC's
// work.
//
//   RX  ip_input.c:460-471 (CSUM_IP_CHECKED / CSUM_IP_VALID),
//       tcp_input.c:697-718 and udp_usrreq.c:428-449 (CSUM_DATA_VALID |
//       CSUM_PSEUDO_HDR: th_sum = csum_data ^ 0xffff must be 0);
//       IPv6: tcp_input.c:627-639 and udp6_usrreq.c:216-246 read the same
//       marks (CSUM_DATA_VALID_IPV6 == CSUM_DATA_VALID, mbuf.h:302).
//   TX  ip_output.c:645-667 (deferred ip_sum) and :953-976 (in_delayed_cksum:
//       in_cksum_skip(m, ip_len, hlen) over the in_pseudo seed already in
//       th_sum, UDP 0 -> 0xffff, stored at hlen + csum_data);
//       IPv6: ip6_output.c:966-988 and :188-209 (in6_delayed_cksum:
//       in_cksum_skip(m, 40 + plen, 40) over the in6_cksum_pseudo seed that
//       tcp_output.c:1069-1071 / udp6_usrreq.c:786 put in the checksum field).
//
// The host parses headers (a few bytes per packet, already in cache from the
// driver) and writes flags; every byte sum is a GPU job (host_batch.h).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

#include <vector>

#include "cksum_internal.h"
#include "host_batch.h"
#include "host_pool.h"

namespace uinet {
namespace {

// sys/sys/mbuf.h:182,281-293; sys/netinet/ip.h:63-65.
constexpr int kMPktHdr = 0x2;
constexpr int kCsumIp = 0x1, kCsumTcp = 0x2, kCsumUdp = 0x4, kCsumTso = 0x20;
constexpr int kCsumUdpIpv6 = 0x2000, kCsumTcpIpv6 = 0x4000;  // mbuf.h:295-296
constexpr int kCsumIpChecked = 0x100, kCsumIpValid = 0x200, kCsumDataValid = 0x400,
              kCsumPseudoHdr = 0x800;
constexpr int kIpMf = 0x2000, kIpOffMask = 0x1fff;

// Copies up to n bytes at chain offset `off`; returns the count copied.
int chain_read(const MbufHdr* m, int off, uint8_t* dst, int n) {
  int got = 0;
  for (; m && got < n; m = m->m_next) {
    const int l = m->m_len;
    if (l <= 0) continue;
    if (off >= l) {
      off -= l;
      continue;
    }
    const int k = (l - off < n - got) ? l - off : n - got;
    memcpy(dst + got, m->m_data + off, (size_t)k);
    got += k;
    off = 0;
  }
  return got;
}

long chain_len(const MbufHdr* m) {
  long t = 0;
  for (; m; m = m->m_next) t += m->m_len > 0 ? m->m_len : 0;
  return t;
}

inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
inline uint16_t bswap16(uint16_t x) { return (uint16_t)((x << 8) | (x >> 8)); }

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

// The network header's offset and IP version (4 or 6; 0 = neither).
// l2len -1: Ethernet (0x0800 / 0x86dd, or one 802.1Q tag first); l2len >= 0:
// the header sits at l2len and its version nibble tells.
int l3_locate(const MbufHdr* m, int l2len, int* l3) {
  uint8_t b[18];
  if (l2len >= 0) {
    *l3 = l2len;
    if (chain_read(m, l2len, b, 1) < 1) return 0;
    return (b[0] >> 4) == 4 ? 4 : (b[0] >> 4) == 6 ? 6 : 0;
  }
  const int got = chain_read(m, 0, b, 18);
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

bool parse_ip4(const MbufHdr* m, int l3, Ip4* o) {
  uint8_t b[60 + 8];
  const int got = chain_read(m, l3, b, 60 + 8);
  if (got < 20 || (b[0] >> 4) != 4) return false;
  const int hl = (b[0] & 15) * 4;
  if (hl < 20 || got < hl) return false;
  o->l3 = l3;
  o->hl = hl;
  o->ip_len = be16(b + 2);
  o->frag = (be16(b + 6) & (kIpMf | kIpOffMask)) != 0;
  o->proto = b[9];
  memcpy(&o->src, b + 12, 4);
  memcpy(&o->dst, b + 16, 4);
  o->l4_have = got - hl < 8 ? got - hl : 8;
  memcpy(o->l4, b + hl, (size_t)o->l4_have);
  return true;
}

uint32_t fold16(uint64_t s) {
  while (s >> 16) s = (s & 0xffff) + (s >> 16);
  return (uint32_t)s;
}

// The fixed IPv6 header and the first 8 bytes after it.
struct Ip6 {
  int l3 = 0;
  int plen = 0;  // ip6_plen
  int nxt = 0;
  uint8_t addr[32] = {};  // source, destination
  uint8_t l4[8] = {};
  int l4_have = 0;
};

bool parse_ip6(const MbufHdr* m, int l3, Ip6* o) {
  uint8_t b[40 + 8];
  const int got = chain_read(m, l3, b, 40 + 8);
  if (got < 40 || (b[0] >> 4) != 6) return false;
  o->l3 = l3;
  o->plen = be16(b + 4);
  o->nxt = b[6];
  memcpy(o->addr, b + 8, 32);
  o->l4_have = got - 40;
  memcpy(o->l4, b + 40, (size_t)o->l4_have);
  return true;
}

// A link-local unicast, or link- / interface-local multicast, address whose
// second 16-bit word (KAME's embedded zone) is nonzero.  ip6_input drops such
// packets before any transport input (ip6_input.c:658-661, "badscope"), so
// the RX hook leaves them unmarked.
bool ip6_zone_embedded(const uint8_t* a) {
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
int ip6_walk(const MbufHdr* m, const Ip6& ip, bool rx, int* off, int* nxt) {
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
    uint8_t e[4];
    if (o + 8 > 40 + ip.plen || chain_read(m, ip.l3 + o, e, 4) < 4) return -1;
    if (rx && x == 43 && e[3] != 0) return -1;  // segments left: route6.c:99-105
    x = e[0];
    o += (e[1] + 1) * 8;
  }
  return -1;
}

// in6_cksum.c:86-126 for wire addresses (no embedded zone): htonl(len),
// three zero bytes and the transport's nxt, then both addresses, as
// little-endian 16-bit words; folded so it fits a job seed.
uint32_t pseudo6_seed(const Ip6& ip, uint32_t len, int nxt) {
  uint64_t s = (uint64_t)bswap16((uint16_t)(len >> 16)) + bswap16((uint16_t)len) +
               bswap16((uint16_t)nxt);
  for (int i = 0; i < 32; i += 2) s += (uint64_t)(ip.addr[i] | ip.addr[i + 1] << 8);
  return fold16(s);
}

// in_cksum.c:252-253, folded so it fits a job seed.
uint32_t pseudo_seed(uint32_t src, uint32_t dst, int proto, int plen) {
  return fold16((uint64_t)src + dst + bswap16((uint16_t)proto) + bswap16((uint16_t)plen));
}

// Packet i owns jobs 2i (IP header) and 2i+1 (TCP/UDP); an unused job has
// m == nullptr and walks nothing.
struct RxPlan {
  Ip4 ip;
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

// RX IPv6: tcp_input.c:627-639 (tlen = 40 + ip6_plen - off0, the transport
// after the extension headers) and udp6_usrreq.c:216-246 (uh_ulen must equal
// that length, uh_sum 0 is an error).  Returns the L4 job, or m == nullptr
// for none.
Job rx6_job(const MbufHdr* m, const Ip6& ip, uint8_t* st) {
  const Job none{nullptr, 0, 0, 0u};
  int off = 40, nxt = ip.nxt;
  const int w = ip.plen ? ip6_walk(m, ip, true, &off, &nxt) : -1;
  if (w == 0 || ip.nxt == 44) *st |= UINET_RX_FRAG;
  if (w != 1) return none;
  if (chain_len(m) < (long)ip.l3 + 40 + ip.plen) return none;  // ip6s_tooshort
  if (ip6_zone_embedded(ip.addr) || ip6_zone_embedded(ip.addr + 16)) return none;
  const int tlen = 40 + ip.plen - off;
  if (nxt == 17) {
    uint8_t u[8];
    const uint8_t* uh = ip.l4;
    if (off != 40) {
      if (chain_read(m, ip.l3 + off, u, 8) < 8) return none;
      uh = u;
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
  return Job{m, ip.l3 + 40 + ip.plen, ip.l3 + off, pseudo6_seed(ip, (uint32_t)tlen, nxt)};
}

// UINET_CKSUM_TRACE_HOST=1: the hooks' phase times on stderr (tools only;
// run_jobs prints its own walk / pack / launch split under the same switch).
// The parse runs inside the batch walk (run_jobs_made), so it is part of
// "walk+fold"; "setup" is the per-call plan allocation before it.
struct PhaseTrace {
  using clk = std::chrono::steady_clock;
  const char* what;
  bool on;
  clk::time_point t0, t1, t2;
  explicit PhaseTrace(const char* w) : what(w), on(enabled()) {
    if (on) t0 = clk::now();
  }
  static bool enabled() {
    static const bool e = getenv("UINET_CKSUM_TRACE_HOST") != nullptr;  // read once
    return e;
  }
  void set_up() {
    if (on) t1 = clk::now();
  }
  void summed() {
    if (on) t2 = clk::now();
  }
  void done(int n) {
    if (!on) return;
    const clk::time_point t3 = clk::now();
    auto ms = [](clk::time_point a, clk::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    fprintf(stderr,
            "uinet_cksum offload %s: n=%d | setup %.3f ms, parse+walk+fold %.3f ms, apply %.3f ms\n",
            what, n, ms(t0, t1), ms(t1, t2), ms(t2, t3));
  }
};

thread_local std::vector<Job> t_l4;
thread_local std::vector<uint16_t> t_res;
thread_local std::vector<RxPlan> t_rx;
thread_local std::vector<TxPlan> t_tx;

// f(i0, i1) over chunks of consecutive packets, on the host pool.
template <typename F>
void for_chunks(int n, F&& f) {
  const int threads = tuning().host_threads;
  int cs = (n + threads * 4 - 1) / (threads * 4);
  if (cs < 1024) cs = 1024;
  const int nch = (n + cs - 1) / cs;
  host_pool().run(nch, threads, [&](int j) { f(j * cs, j * cs + cs < n ? j * cs + cs : n); },
                  tuning().host_pin != 0);
}

// Packet k of a hook's batch owns jobs 2k (IP header) and 2k + 1 (TCP / UDP);
// the hook's parse runs when the batch walk reaches job 2k (run_jobs_made), so
// each packet's headers are read once, on the thread that then walks its
// chains.  Parsing is idempotent (a staged re-walk parses again).
struct HookCtx {
  struct mbuf* const* mv;
  int n;
  int l2len;
  void* plan;  // RxPlan* or TxPlan*
  Job* l4;     // job 2k + 1 of packet k, made with job 2k
};
// The RX parse reads each packet's first data line(s) (link, IP and transport
// headers, in a cluster apart from the mbuf): request packet k + 4's while
// packet k is parsed.  Its mbuf header was requested 4 packets earlier (the
// walk's prefetch runs 8 packets ahead).  RX 17 % faster (r04hk3).
constexpr int kDataAhead = 4;
inline void prefetch_headers(const HookCtx& c, int k) {
  const int a = k + kDataAhead;
  if (a >= c.n || !c.mv[a]) return;
  const uint8_t* d = reinterpret_cast<const MbufHdr*>(c.mv[a])->m_data;
  __builtin_prefetch(d, 0, 3);
  __builtin_prefetch(d + 64, 0, 3);
}
const MbufHdr* hook_first(void* ctx, int i) {
  return reinterpret_cast<const MbufHdr*>(static_cast<HookCtx*>(ctx)->mv[i >> 1]);
}

// RX: ip_input.c:460-471, tcp_input.c:697-718, udp_usrreq.c:404-449 and the
// IPv6 forms (rx6_job).  Returns the IP-header job; the L4 job goes to *l4.
Job rx_parse(const MbufHdr* m, int l2len, RxPlan& p, Job* l4) {
  const Job none{nullptr, 0, 0, 0u};
  p = RxPlan();
  *l4 = none;
  int l3 = 0;
  const int ver = m ? l3_locate(m, l2len, &l3) : 0;
  if (ver == 6) {
    Ip6 ip6;
    if (!parse_ip6(m, l3, &ip6)) return none;
    p.st |= UINET_RX_IPV6;
    const Job j = rx6_job(m, ip6, &p.st);
    if (j.m) {
      p.l4_job = true;
      *l4 = j;
    }
    return none;
  }
  if (ver != 4 || !parse_ip4(m, l3, &p.ip)) return none;
  const Ip4& ip = p.ip;
  p.st |= UINET_RX_IPV4;
  p.ip_job = true;  // in_cksum(m, hlen) over the header (ip_input.c:463-467)
  const Job hdr{m, ip.l3 + ip.hl, ip.l3, 0u};
  if (ip.frag) {
    p.st |= UINET_RX_FRAG;
    return hdr;
  }
  if (ip.ip_len < ip.hl || chain_len(m) < (long)ip.l3 + ip.ip_len) return hdr;
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
  *l4 = Job{m, ip.l3 + ip.hl + plen, ip.l3 + ip.hl, pseudo_seed(ip.src, ip.dst, ip.proto, plen)};
  return hdr;
}
Job rx_make(void* ctx, int i) {
  HookCtx& c = *static_cast<HookCtx*>(ctx);
  const int k = i >> 1;
  if (i & 1) return c.l4[k];
  prefetch_headers(c, k);
  return rx_parse(reinterpret_cast<const MbufHdr*>(c.mv[k]), c.l2len,
                  static_cast<RxPlan*>(c.plan)[k], &c.l4[k]);
}

// TX: ip_output.c:645-667,953-976 and ip6_output.c:188-209,966-988.  Zeroes
// ip_sum before the header job reads it (ip_output.c:665-667).
Job tx_parse(MbufHdr* m, int l2len, TxPlan& p, Job* l4) {
  const Job none{nullptr, 0, 0, 0u};
  p = TxPlan();
  *l4 = none;
  if (!m || !(m->m_flags & kMPktHdr)) {
    p.st = UINET_TX_SKIP;
    return none;
  }
  const int fl = pkthdr_of(m)->csum_flags;
  int l3 = 0;
  const int ver = (fl & kCsumTso) ? 0 : l3_locate(m, l2len, &l3);
  if (ver == 6) {  // in6_delayed_cksum, ip6_output.c:188-209,978-981
    // As an offloading NIC must (ip6_output.c:966-981 leaves CSUM_*_IPV6 to a
    // driver that advertises it, extension headers or not), the transport is
    // found past the extension headers; the seed already in its checksum
    // field holds the final destination.
    Ip6 ip6;
    int off = 40, nxt = 0;
    if (!(fl & (kCsumTcpIpv6 | kCsumUdpIpv6)) || !parse_ip6(m, l3, &ip6) || ip6.plen == 0 ||
        ip6_walk(m, ip6, false, &off, &nxt) != 1) {
      p.st = UINET_TX_SKIP;
      return none;
    }
    p.st = UINET_TX_IPV6;
    p.udp = (fl & kCsumUdpIpv6) != 0;
    p.clear = kCsumTcpIpv6 | kCsumUdpIpv6;
    p.l4_store = l3 + off + pkthdr_of(m)->csum_data;
    p.l4_job = true;
    *l4 = Job{m, l3 + 40 + ip6.plen, l3 + off, 0u};
    return none;
  }
  Ip4 ip;
  if (ver != 4 || !(fl & (kCsumIp | kCsumTcp | kCsumUdp)) || !parse_ip4(m, l3, &ip)) {
    p.st = UINET_TX_SKIP;
    return none;
  }
  if ((fl & kCsumIp) && ip.l3 + 12 > m->m_len) {
    p.st = UINET_TX_SKIP;  // header not in the first mbuf: leave it to the stack
    return none;
  }
  if (fl & (kCsumTcp | kCsumUdp)) {  // in_delayed_cksum, ip_output.c:958-963
    p.udp = (fl & kCsumUdp) != 0;
    p.clear = kCsumTcp | kCsumUdp;
    p.l4_store = ip.l3 + ip.hl + pkthdr_of(m)->csum_data;
    p.l4_job = true;
    *l4 = Job{m, ip.l3 + ip.ip_len, ip.l3 + ip.hl, 0u};
  }
  if (fl & kCsumIp) {  // ip_output.c:665-667: ip_sum = 0, then in_cksum(m, hlen)
    m->m_data[ip.l3 + 10] = 0;
    m->m_data[ip.l3 + 11] = 0;
    p.ip_l3 = ip.l3;
    p.ip_job = true;
    return Job{m, ip.l3 + ip.hl, ip.l3, 0u};
  }
  return none;
}
Job tx_make(void* ctx, int i) {
  HookCtx& c = *static_cast<HookCtx*>(ctx);
  const int k = i >> 1;
  if (i & 1) return c.l4[k];
  // no data prefetch: a TX packet's headers sit in its first mbuf (m_pktdat),
  // which the walk's own prefetch brings in (measured 9 % slower with it, r04hk3)
  return tx_parse(reinterpret_cast<MbufHdr*>(c.mv[k]), c.l2len, static_cast<TxPlan*>(c.plan)[k],
                  &c.l4[k]);
}

}  // namespace
}  // namespace uinet

using namespace uinet;

extern "C" {

int uinet_cksum_rx_offload(struct mbuf* const* mv, int n, int l2len, uint8_t* status) {
  if (n < 0 || (n > 0 && !mv) || l2len < -1) return UINET_CKSUM_EINVAL;
  if (n == 0) return UINET_CKSUM_OK;
  CpuScope cpu(n);
  PhaseTrace tr("rx");
  std::vector<RxPlan>& plan = t_rx;
  std::vector<Job>& l4 = t_l4;
  plan.resize((size_t)n);
  l4.resize((size_t)n);
  HookCtx ctx{mv, n, l2len, plan.data(), l4.data()};
  tr.set_up();  // parsing runs inside the walk
  std::vector<uint16_t>& res = t_res;
  res.resize(2 * (size_t)n);
  const int rc = run_jobs_made(2 * n, rx_make, hook_first, &ctx, res.data());
  if (rc) return rc;
  tr.summed();
  for_chunks(n, [&](int i0, int i1) {
    for (int i = i0; i < i1; i++) {
      RxPlan& p = plan[(size_t)i];
      MbufHdr* m = reinterpret_cast<MbufHdr*>(mv[i]);
      const bool hdr = m && (m->m_flags & kMPktHdr);
      if (p.ip_job) {
        const bool ok = res[2 * (size_t)i] == 0;
        p.st |= ok ? UINET_RX_IP_OK : 0;
        if (hdr) pkthdr_of(m)->csum_flags |= kCsumIpChecked | (ok ? kCsumIpValid : 0);
      }
      if (p.l4_job) {
        const uint16_t r = res[2 * (size_t)i + 1];
        p.st |= UINET_RX_L4 | (r == 0 ? UINET_RX_L4_OK : 0);
        if (hdr) {
          PktHdr* ph = pkthdr_of(m);
          ph->csum_flags |= kCsumDataValid | kCsumPseudoHdr;
          ph->csum_data = r ^ 0xffff;
        }
      }
      if (status) status[i] = p.st;
    }
  });
  tr.done(n);
  return UINET_CKSUM_OK;
}

int uinet_cksum_tx_offload(struct mbuf* const* mv, int n, int l2len, uint8_t* status) {
  if (n < 0 || (n > 0 && !mv) || l2len < -1) return UINET_CKSUM_EINVAL;
  if (n == 0) return UINET_CKSUM_OK;
  CpuScope cpu(n);
  PhaseTrace tr("tx");
  std::vector<TxPlan>& plan = t_tx;
  std::vector<Job>& l4 = t_l4;
  plan.resize((size_t)n);
  l4.resize((size_t)n);
  HookCtx ctx{mv, n, l2len, plan.data(), l4.data()};
  tr.set_up();  // parsing runs inside the walk
  std::vector<uint16_t>& res = t_res;
  res.resize(2 * (size_t)n);
  const int rc = run_jobs_made(2 * n, tx_make, hook_first, &ctx, res.data());
  if (rc) return rc;
  tr.summed();
  for_chunks(n, [&](int i0, int i1) {
    for (int i = i0; i < i1; i++) {
      TxPlan& p = plan[(size_t)i];
      MbufHdr* m = reinterpret_cast<MbufHdr*>(mv[i]);
      if (p.l4_job) {
        uint16_t c = res[2 * (size_t)i + 1];
        if (p.udp && c == 0) c = 0xffff;  // ip_output.c:962-963, ip6_output.c:193-194
        if (p.l4_store + 2 > m->m_len) {
          p.st |= UINET_TX_L4_LOST;  // ip_output.c:966-974: the reference gives up too
        } else {
          memcpy(m->m_data + p.l4_store, &c, 2);
          p.st |= UINET_TX_L4;
        }
        pkthdr_of(m)->csum_flags &= ~p.clear;
      }
      if (p.ip_job) {
        const uint16_t c = res[2 * (size_t)i];
        memcpy(m->m_data + p.ip_l3 + 10, &c, 2);
        p.st |= UINET_TX_IP;
        pkthdr_of(m)->csum_flags &= ~kCsumIp;
      }
      if (status) status[i] = p.st;
    }
  });
  tr.done(n);
  return UINET_CKSUM_OK;
}

}  // extern "C"
