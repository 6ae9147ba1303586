// Host-side mbuf view and the walked-batch entry point shared by the C ABI
// (cksum_api.hip) and the driver offload hooks (cksum_offload.hip).
// Internal; not part of the C ABI.
#pragma once

#include <stddef.h>
#include <stdint.h>

struct mbuf;  // the C ABI's opaque struct mbuf (include/uinet_cksum.h)

namespace uinet {

// struct m_hdr (sys/sys/mbuf.h:90-98) on amd64: M_HDR_PAD 6 (:82), 40 bytes.
struct MbufHdr {
  MbufHdr* m_next;
  void* m_nextpkt;
  uint8_t* m_data;
  int m_len;
  int m_flags;
  short m_type;
  uint8_t pad[6];
};
static_assert(offsetof(MbufHdr, m_next) == 0, "m_next offset");
static_assert(offsetof(MbufHdr, m_data) == 16, "m_data offset");
static_assert(offsetof(MbufHdr, m_len) == 24, "m_len offset");
static_assert(offsetof(MbufHdr, m_flags) == 28, "m_flags offset");
static_assert(sizeof(MbufHdr) == 40, "struct m_hdr size");

// struct pkthdr (sys/sys/mbuf.h:116-133), right after m_hdr when M_PKTHDR.
struct PktHdr {
  void* rcvif;
  void* header;
  int len;
  uint32_t flowid;
  int csum_flags;
  int csum_data;
  uint16_t tso_segsz;
  uint16_t vtag;
  void* tags;
};
static_assert(offsetof(PktHdr, csum_flags) == 24, "csum_flags at mbuf+64");
static_assert(offsetof(PktHdr, csum_data) == 28, "csum_data at mbuf+68");
static_assert(sizeof(MbufHdr) + sizeof(PktHdr) == 88, "m_pktdat at mbuf+88 (MHLEN 168)");

inline PktHdr* pkthdr_of(MbufHdr* m) {
  return reinterpret_cast<PktHdr*>(reinterpret_cast<uint8_t*>(m) + sizeof(MbufHdr));
}

// One in_cksum_skip(m, len, skip) with `seed` added to the sum before the
// complement (0 for plain in_cksum_skip).
struct Job {
  const MbufHdr* m;
  int len;
  int skip;
  uint32_t seed;
};

// Folds every job on the GPU in one batch (walk, zero-copy or staging, one
// launch).  Returns a UINET_CKSUM_* code.
int run_jobs(const Job* jobs, int n, uint16_t* out);

// The same for jobs made while the batch is walked: make(ctx, i) returns job
// i on the walking thread, just before its chain is walked, so a caller that
// derives jobs from packet headers reads each header once, while its lines
// are being fetched anyway.  Jobs 2k and 2k + 1 are made on one thread, in
// that order (a walk chunk never splits such a pair), and a job may be made
// more than once (a zero-copy batch that has to be staged is walked again):
// make must be idempotent.  first(ctx, i) is job i's first mbuf (prefetched
// a few jobs ahead), without making the job.
typedef Job (*JobMaker)(void* ctx, int i);
typedef const MbufHdr* (*JobFirst)(void* ctx, int i);
int run_jobs_made(int n, JobMaker make, JobFirst first, void* ctx, uint16_t* out);

// The RX (rx true) / TX hook of a batch whose mbufs and frames all lie in
// registered memory, done on the device: parse, walk, fold and the verdicts
// (cksum_hookdev.hip).  Returns 1 when it does not apply or the device view
// could not take the batch (nothing was written), else a UINET_CKSUM_* code.
int run_hook_device(bool rx, struct mbuf* const* mv, int n, int l2len, uint8_t* status);

// Host CPU accounting of the batch entry points (uinet_cksum_host_cpu): a
// CpuScope at each public host-batch entry adds the call's wall time, the
// calling thread's CPU time and the pool helpers' CPU time to the calling
// thread's counters.  Nested scopes (a hook's batch) count once.
struct CpuScope {
  explicit CpuScope(int packets);
  ~CpuScope();
  CpuScope(const CpuScope&) = delete;
  CpuScope& operator=(const CpuScope&) = delete;
  bool outer;
  int packets;
  uint64_t wall0, cpu0, helper0;
};
// The calling thread's batch was walked on the device (counted by the scope).
void note_device_walk();
// The calling thread's batch went down the single-mbuf span path, `dma`
// bytes of it copied to HBM by DMA.
void note_span_fast(uint64_t dma);

// The per-call ABI's host fold (cksum_percall.cpp): one chain on the calling
// thread, no device involved, no error path (like the reference).
uint16_t host_cksum_skip(const MbufHdr* m, long len, long skip, uint32_t seed);
uint16_t host_cksum_pseudo(const MbufHdr* m, int plen, int off0, uint32_t src, uint32_t dst,
                           uint8_t proto);
uint32_t host_cksum_hdr(const void* ip);

}  // namespace uinet
