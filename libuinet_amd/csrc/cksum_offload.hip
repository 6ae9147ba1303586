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
#include "offload_hostview.h"
#include "offload_parse.h"

namespace uinet {
namespace {

using namespace hook;

inline Job job_of(const PJob& j) {
  return Job{reinterpret_cast<const MbufHdr*>(j.m), j.len, j.skip, j.seed};
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
  host_pool().run(nch, threads, [&](int j) { f(j * cs, j * cs + cs < n ? j * cs + cs : n); });
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

Job rx_make(void* ctx, int i) {
  HookCtx& c = *static_cast<HookCtx*>(ctx);
  const int k = i >> 1;
  if (i & 1) return c.l4[k];
  prefetch_headers(c, k);
  PJob l4;
  const HostView v{reinterpret_cast<MbufHdr*>(c.mv[k])};
  const PJob j = rx_parse(v, c.l2len, static_cast<RxPlan*>(c.plan)[k], &l4);
  c.l4[k] = job_of(l4);
  return job_of(j);
}

Job tx_make(void* ctx, int i) {
  HookCtx& c = *static_cast<HookCtx*>(ctx);
  const int k = i >> 1;
  if (i & 1) return c.l4[k];
  // no data prefetch: a TX packet's headers sit in its first mbuf (m_pktdat),
  // which the walk's own prefetch brings in (measured 9 % slower with it, r04hk3)
  PJob l4;
  HostView v{reinterpret_cast<MbufHdr*>(c.mv[k])};
  const PJob j = tx_parse(v, c.l2len, static_cast<TxPlan*>(c.plan)[k], &l4);
  c.l4[k] = job_of(l4);
  return job_of(j);
}

}  // namespace
}  // namespace uinet

using namespace uinet;

extern "C" {

int uinet_cksum_rx_offload(struct mbuf* const* mv, int n, int l2len, uint8_t* status) {
  if (n < 0 || (n > 0 && !mv) || l2len < -1) return UINET_CKSUM_EINVAL;
  if (n == 0) return UINET_CKSUM_OK;
  CpuScope cpu(n);
  // mbufs and frames in registered memory: the whole hook on the device
  // (cksum_hookdev.hip); otherwise, or when the device view cannot take the
  // batch, the host parses and walks below
  {
    const int drc = run_hook_device(true, mv, n, l2len, status);
    if (drc != 1) return drc;
  }
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
  {
    const int drc = run_hook_device(false, mv, n, l2len, status);
    if (drc != 1) return drc;
  }
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
