// The driver hooks' header parse (libuinet_amd/csrc/offload_parse.h) through
// the host hook's own view (offload_hostview.h), built with g++ as a small
// shared library for tests/test_parse_host.py: the CPU suite checks the jobs
// and plans it makes against the oracle's hooks, with the sums folded by the
// oracle, no GPU involved.
#include <stdint.h>

#include "offload_hostview.h"
#include "offload_parse.h"

using uinet::MbufHdr;
using namespace uinet::hook;

namespace {

void put_jobs(int k, const PJob& j0, const PJob& j1, uint64_t* jm, int32_t* jl, int32_t* js,
              uint32_t* jd) {
  jm[2 * k] = j0.m;
  jl[2 * k] = j0.len;
  js[2 * k] = j0.skip;
  jd[2 * k] = j0.seed;
  jm[2 * k + 1] = j1.m;
  jl[2 * k + 1] = j1.len;
  js[2 * k + 1] = j1.skip;
  jd[2 * k + 1] = j1.seed;
}

}  // namespace

extern "C" {

// Per frame k: jobs 2k (IP header) and 2k + 1 (transport), m == 0 for none;
// plan: ip_job, l4_job, status bits so far.
void parse_rx(const uint64_t* mv, int n, int l2len, uint64_t* jm, int32_t* jl, int32_t* js,
              uint32_t* jd, uint8_t* ip_job, uint8_t* l4_job, uint8_t* st) {
  for (int k = 0; k < n; k++) {
    const HostView v{reinterpret_cast<MbufHdr*>(mv[k])};
    RxPlan p;
    PJob j1;
    const PJob j0 = rx_parse(v, l2len, p, &j1);
    put_jobs(k, j0, j1, jm, jl, js, jd);
    ip_job[k] = p.ip_job;
    l4_job[k] = p.l4_job;
    st[k] = p.st;
  }
}

// TX: as parse_rx, plus where the sums go (chain offsets in the first mbuf)
// and which csum_flags bits the hook takes over.  Zeroes ip_sum in the frame
// as the host hook does (ip_output.c:665-667).
void parse_tx(const uint64_t* mv, int n, int l2len, uint64_t* jm, int32_t* jl, int32_t* js,
              uint32_t* jd, uint8_t* ip_job, uint8_t* l4_job, uint8_t* udp, int32_t* l4_store,
              int32_t* ip_l3, int32_t* clear, uint8_t* st) {
  for (int k = 0; k < n; k++) {
    HostView v{reinterpret_cast<MbufHdr*>(mv[k])};
    TxPlan p;
    PJob j1;
    const PJob j0 = tx_parse(v, l2len, p, &j1);
    put_jobs(k, j0, j1, jm, jl, js, jd);
    ip_job[k] = p.ip_job;
    l4_job[k] = p.l4_job;
    udp[k] = p.udp;
    l4_store[k] = p.l4_store;
    ip_l3[k] = p.ip_l3;
    clear[k] = p.clear;
    st[k] = p.st;
  }
}

}  // extern "C"
