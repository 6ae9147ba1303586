// Host side of the engine: the C ABI of include/uinet_cksum.h.
//
//  * Device-resident descriptor API: argument checks + one launch.
//  * Host-mbuf batch API: walks each chain exactly like the reference
//    (/root/reference/sys/amd64/amd64/in_cksum.c:193-232 for in_cksum_skip,
//    :241-276 for in_cksum_pseudo_header, :278-285 for in_cksum_hdr).  Over
//    registered memory it writes chain descriptors and the chain kernel folds
//    the bytes in place over PCIe, group by group while the host walks on.
//    Otherwise it packs the bytes each packet contributes into pinned staging
//    (one contiguous run per packet, logical order, 16-byte aligned starts),
//    ships staging to HBM, folds it with one launch of the span kernel and
//    copies the 16-bit results back.
//  * Per-call drop-in ABI: one chain folded on the calling thread
//    (cksum_percall.cpp); no device, no error path, like the reference.
//
// Threading: the reference checksum is fully reentrant; here
// every calling thread gets its own stream and staging buffers (thread_local),
// so concurrent RX/TX threads never share device state.  A large host-mbuf
// batch is walked and packed by the host pool (host_pool.h); a batch that
// finds the pool in use by another thread does that work itself.
#include <hip/hip_runtime.h>

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cxxabi.h>
#include <sys/prctl.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "cksum_internal.h"
#include "host_batch.h"
#include "host_pool.h"

namespace uinet {

static thread_local int t_last_hip = 0;

int record_hip(hipError_t e) {
  if (e == hipSuccess) return UINET_CKSUM_OK;
  t_last_hip = (int)e;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return UINET_CKSUM_ENODEV;
  if (e == hipErrorOutOfMemory) return UINET_CKSUM_ENOMEM;
  return UINET_CKSUM_EHIP;
}

int check_launch() { return record_hip(hipGetLastError()); }

thread_local const void* t_last_kernel = nullptr;
void note_kernel(const void* host_stub) { t_last_kernel = host_stub; }

// The live knob values.  uinet_cksum_set_tuning may run while other threads
// launch, so each knob is a relaxed atomic and a launch reads one snapshot
// (tuning()).  The environment seeds them through the same validation.
struct TuningLive {
  std::atomic<int> blocks_per_cu{0}, host_threads{8}, chains_long{128}, xcd_remap{1},
      multi_gather{0}, walk_device{1}, chains_wide{0}, span_fast{1};
};

static std::atomic<int>* tuning_field(TuningLive& t, const char* key, int value) {
  struct Knob {
    const char* key;
    std::atomic<int> TuningLive::*field;
    bool (*ok)(int);
  };
  static const Knob knobs[] = {
      {"blocks_per_cu", &TuningLive::blocks_per_cu, [](int v) { return v >= 0 && v <= 4096; }},
      {"chains_long", &TuningLive::chains_long,
       [](int v) { return v == 0 || (v >= 16 && v <= (1 << 24)); }},
      {"xcd_remap", &TuningLive::xcd_remap, [](int v) { return v == 0 || v == 1; }},
      {"host_threads", &TuningLive::host_threads, [](int v) { return v >= 1 && v <= 64; }},
      {"multi_gather", &TuningLive::multi_gather, [](int v) { return v == 0 || v == 1; }},
      {"walk_device", &TuningLive::walk_device, [](int v) { return v >= 0 && v <= 3; }},
      {"chains_wide", &TuningLive::chains_wide, [](int v) { return v >= 0 && v <= 2; }},
      {"span_fast", &TuningLive::span_fast, [](int v) { return v >= 0 && v <= 2; }},
  };
  for (const Knob& k : knobs)
    if (!strcmp(key, k.key)) return k.ok(value) ? &(t.*k.field) : nullptr;
  return nullptr;
}

static TuningLive& tuning_live() {
  static TuningLive* t = [] {
    auto* x = new TuningLive;  // never freed: launches may run during exit
    const unsigned hw = std::thread::hardware_concurrency();
    x->host_threads = (int)std::min(16u, hw ? hw : 1u);
    static const char* const env[][2] = {
        {"UINET_CKSUM_BLOCKS_PER_CU", "blocks_per_cu"}, {"UINET_CKSUM_CHAINS_LONG", "chains_long"},
        {"UINET_CKSUM_XCD_REMAP", "xcd_remap"},         {"UINET_CKSUM_HOST_THREADS", "host_threads"},
        {"UINET_CKSUM_MULTI_GATHER", "multi_gather"},   {"UINET_CKSUM_WALK_DEVICE", "walk_device"},
        {"UINET_CKSUM_CHAINS_WIDE", "chains_wide"},     {"UINET_CKSUM_SPAN_FAST", "span_fast"},
    };
    for (const auto& kv : env) {
      const char* e = getenv(kv[0]);
      if (!e || !*e) continue;
      int v = atoi(e);
      if (!strcmp(kv[1], "xcd_remap"))
        v = v ? 1 : 0;
      if (std::atomic<int>* f = tuning_field(*x, kv[1], v)) f->store(v, std::memory_order_relaxed);
    }
    return x;
  }();
  return *t;
}

Tuning tuning() {
  const TuningLive& t = tuning_live();
  const auto ld = [](const std::atomic<int>& a) { return a.load(std::memory_order_relaxed); };
  Tuning x;
  x.blocks_per_cu = ld(t.blocks_per_cu);
  x.host_threads = ld(t.host_threads);
  x.chains_long = ld(t.chains_long);
  x.xcd_remap = ld(t.xcd_remap);
  x.multi_gather = ld(t.multi_gather);
  x.walk_device = ld(t.walk_device);
  x.chains_wide = ld(t.chains_wide);
  x.span_fast = ld(t.span_fast);
  return x;
}

// ---- host CPU accounting (uinet_cksum_host_cpu) -----------------------------

namespace {
thread_local struct uinet_cksum_host_cpu t_cpu{};
thread_local int t_cpu_depth = 0;
uint64_t wall_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

CpuScope::CpuScope(int n) : outer(t_cpu_depth++ == 0), packets(n) {
  if (!outer) return;
  wall0 = wall_ns();
  cpu0 = thread_cpu_ns();
  helper0 = t_pool_helper_ns;
}

CpuScope::~CpuScope() {
  --t_cpu_depth;
  if (!outer) return;
  t_cpu.calls++;
  t_cpu.packets += packets > 0 ? (uint64_t)packets : 0u;
  t_cpu.wall_ns += wall_ns() - wall0;
  t_cpu.caller_cpu_ns += thread_cpu_ns() - cpu0;
  t_cpu.helper_cpu_ns += t_pool_helper_ns - helper0;
}

void note_device_walk() { t_cpu.device_walks++; }
void note_span_fast(uint64_t dma) {
  t_cpu.span_batches++;
  t_cpu.span_dma_bytes += dma;
}

namespace {

uint32_t fold16_host(uint64_t s) {
  while (s >> 16) s = (s & 0xffff) + (s >> 16);
  return (uint32_t)s;
}

uint16_t bswap16(uint16_t x) { return (uint16_t)((x << 8) | (x >> 8)); }

// ---- per-thread engine context --------------------------------------------

struct Ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* h_buf = nullptr;  // pinned: descriptors, then packet bytes
  size_t h_cap = 0;
  uint8_t* d_buf = nullptr;  // device mirror of h_buf
  size_t d_cap = 0;
  uint16_t* h_out = nullptr;  // pinned results
  uint16_t* d_out = nullptr;
  size_t out_cap = 0;
  hipEvent_t done = nullptr;  // recorded after a batch; ctx_wait sleeps until it completes
  hipStream_t side = nullptr;  // device walk: the second stream of the walk/fold pipeline
  hipEvent_t fork = nullptr, join = nullptr;
  uint32_t walk_k = 0;        // device walk: segment slots per packet last needed
  uint8_t* d_stage = nullptr;  // span path: HBM copy of a group's packet range
  size_t stage_cap = 0;
  std::vector<hipEvent_t> gev;  // span walk: one event per group
};

// One context per (thread, device): a thread that serves several devices --
// the multi-device batch workers (cksum_multi.hip), or a caller that switches
// with hipSetDevice -- keeps every device's stream and staging instead of
// dropping and rebuilding them.  Staging is intentionally not released at
// thread exit: HIP may already be torn down when the main thread's
// thread_local destructors run.
constexpr int kMaxDevices = 64;
thread_local Ctx t_ctx[kMaxDevices];

// The calling thread's context for its current device, stream created.
int ctx_current(Ctx** out) {
  int dev = 0;
  int rc = record_hip(hipGetDevice(&dev));
  if (rc) return rc;
  if (dev < 0 || dev >= kMaxDevices) return UINET_CKSUM_ENODEV;
  Ctx& c = t_ctx[dev];
  if (!c.stream) {
    rc = record_hip(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    if (rc) return rc;
    c.device = dev;
  }
  if (!c.done) {
    rc = record_hip(
        hipEventCreateWithFlags(&c.done, hipEventDisableTiming));
    if (rc) return rc;
  }
  *out = &c;
  return UINET_CKSUM_OK;
}

// Waits for everything queued on the context's stream without burning the
// calling core.  hipEventSynchronize / hipStreamSynchronize poll the
// completion signal on this thread for the whole wait, even with
// hipEventBlockingSync (round 5, profiles/r05/r05a2/: a device-walked
// config-3 batch cost 11.5 ms of CPU in an 11.6-ms call).  Here the thread
// polls the event for the first kSpinUs (a small batch's whole fold: no
// added latency), then sleeps between polls for 1/32 of the time waited so
// far (10 us to 1 ms; at most ~3 % added to a long wait), with the timer slack
// at 1 us meanwhile so a short sleep is not stretched to the default 50 us.
// The lab build -DUINET_WAIT_SPIN waits in hipEventSynchronize instead (the
// CPU-time A/B in DESIGN.md).
constexpr long kSpinUs = 50;
// `min_us`: a lower bound on the time the queued work still takes (0 =
// unknown): the thread sleeps that long in one nap before it starts polling,
// instead of the ~150 polls -- each a wakeup -- the geometric schedule below
// spends over a 30-ms batch.
int ctx_wait(Ctx& c, long min_us = 0) {
  int rc = record_hip(hipEventRecord(c.done, c.stream));
  if (rc) return rc;
#ifdef UINET_WAIT_SPIN
  return record_hip(hipEventSynchronize(c.done));
#else
  using clk = std::chrono::steady_clock;
  const clk::time_point t0 = clk::now();
  int slack = -1;  // the thread's timer slack, restored on return
  if (min_us > kSpinUs) {
    const timespec ts{min_us / 1000000, (min_us % 1000000) * 1000};
    nanosleep(&ts, nullptr);
  }
  for (;;) {
    const hipError_t e = hipEventQuery(c.done);
    if (e != hipErrorNotReady) {
      if (slack >= 0) prctl(PR_SET_TIMERSLACK, (unsigned long)slack, 0, 0, 0);
      return record_hip(e);
    }
    const long us = (long)std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - t0)
                        .count();
    if (us < kSpinUs) continue;
    if (slack < 0) {
      slack = (int)prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
      prctl(PR_SET_TIMERSLACK, 1ul, 0, 0, 0);
    }
    const long nap = std::min(1000l, std::max(10l, us / 32));
    const timespec ts{0, nap * 1000};
    nanosleep(&ts, nullptr);
  }
#endif
}

// Grows the pinned staging to `bytes`, its HBM mirror to `dbytes` (default:
// `bytes`; the zero-copy path reads pinned memory in place and passes 0) and
// the result buffers to `nout` entries.
int ctx_reserve(Ctx& c, size_t bytes, size_t nout, size_t dbytes = ~size_t(0)) {
  if (dbytes == ~size_t(0)) dbytes = bytes;
  const bool device = dbytes > 0;
  const auto grow = [](size_t cap, size_t want) {
    cap = cap ? cap : (1u << 20);
    while (cap < want) cap *= 2;
    return cap;
  };
  if (bytes > c.h_cap) {
    const size_t cap = grow(c.h_cap, bytes);
    if (c.h_buf) (void)hipHostFree(c.h_buf);
    c.h_buf = nullptr;
    c.h_cap = 0;
    int rc = record_hip(hipHostMalloc((void**)&c.h_buf, cap, hipHostMallocMapped));
    if (rc) return rc;
    c.h_cap = cap;
  }
  if (device && dbytes > c.d_cap) {
    const size_t cap = grow(c.d_cap, dbytes);
    if (c.d_buf) (void)hipFree(c.d_buf);
    c.d_buf = nullptr;
    c.d_cap = 0;
    int rc = record_hip(hipMalloc((void**)&c.d_buf, cap));
    if (rc) return rc;
    c.d_cap = cap;
  }
  if (nout > c.out_cap) {
    size_t cap = c.out_cap ? c.out_cap : 4096;
    while (cap < nout) cap *= 2;
    if (c.h_out) (void)hipHostFree(c.h_out);
    if (c.d_out) (void)hipFree(c.d_out);
    c.h_out = nullptr;
    c.d_out = nullptr;
    c.out_cap = 0;
    int rc = record_hip(hipHostMalloc((void**)&c.h_out, cap * 2, hipHostMallocMapped));
    if (rc) return rc;
    rc = record_hip(hipMalloc((void**)&c.d_out, cap * 2));
    if (rc) return rc;
    c.out_cap = cap;
  }
  return UINET_CKSUM_OK;
}

// The batch's results from the mapped result buffer into the caller's array:
// one bulk copy for u16 results (per-element reads of the pinned buffer cost
// ~1 ms per million packets).
void deliver(const Ctx& c, int n, uint16_t* out16, unsigned* out32) {
  if (out16) memcpy(out16, c.h_out, 2 * (size_t)n);
  if (out32)
    for (int i = 0; i < n; i++) out32[i] = c.h_out[i];
}

// ---- the reference chain walk, emitting the bytes each packet sums --------

struct Piece {
  const uint8_t* p;
  uint32_t n;
};

// One packet as the reference walks it: the in-order pieces whose bytes are
// summed, the logical parity of the first summed byte, and the seed.
struct PacketWalk {
  std::vector<Piece>* out = nullptr;  // pieces are appended here
  uint64_t bytes = 0;
  long clen = 0;    // logical bytes consumed (may go negative, see below)
  long remain = 0;  // bytes still wanted
  long first_clen = 0;
  bool have_first = false;
  bool long_piece = false;  // a piece over 65535 B since the owner last cleared it

  void reset(long want) {
    bytes = 0;
    clen = 0;
    remain = want;
    have_first = false;
    first_clen = 0;
  }
  // The `skip_start:` block (in_cksum.c:219-228, :263-272).  A negative
  // mlen (len < skip, or m_len < off0) is outside the reference's contract:
  // it then indexes in_masks[] negatively for unaligned addresses; for
  // aligned ones it sums nothing, which is what happens here, while the
  // length/parity bookkeeping follows the reference.
  void take(const uint8_t* addr, long mlen) {
    if (remain < mlen) mlen = remain;
    if (mlen > 0) {
      if (!have_first) {
        have_first = true;
        first_clen = clen;
      }
      out->push_back({addr, (uint32_t)mlen});
      long_piece |= mlen > 0xffff;
      bytes += (uint64_t)mlen;
    }
    clen += mlen;
    remain -= mlen;
  }
  void take_rest(const MbufHdr* m) {  // in_cksum.c:214-229
    for (; m && remain; m = m->m_next) {
      if (m->m_len == 0) continue;
      take(m->m_data, m->m_len);
    }
  }
  void walk_skip(const MbufHdr* m, int len, int skip) {  // in_cksum.c:193-232
    reset((long)len - skip);
    while (skip && m) {
      if (m->m_len > skip) {
        take(m->m_data + skip, (long)m->m_len - skip);
        m = m->m_next;
        skip = 0;
        break;
      }
      skip -= m->m_len;
      m = m->m_next;
    }
    if (skip == 0) take_rest(m);
  }
  void walk_pseudo(const MbufHdr* m, int plen, int off0) {  // in_cksum.c:241-276
    reset(plen);
    take(m->m_data + off0, (long)m->m_len - off0);
    take_rest(m->m_next);
  }
};

// Staging image: [off u64 x n][len u32 x n][seed u32 x n][parity u8 x n] pad16
// then the packed packet bytes.
struct Layout {
  size_t off_o, len_o, seed_o, par_o, data_o;
};

Layout layout_for(size_t n) {
  Layout L;
  L.off_o = 0;
  L.len_o = L.off_o + 8 * n;
  L.seed_o = L.len_o + 4 * n;
  L.par_o = L.seed_o + 4 * n;
  L.data_o = (L.par_o + n + 15) & ~size_t(15);
  return L;
}

// ---- registered host regions (zero-copy) ------------------------------------
//
// Memory registered with uinet_cksum_register_host (netmap rings, UMA slabs)
// is mapped into the GPU's address space; a batch whose pieces all lie in
// registered regions is folded in place over PCIe -- the host only walks the
// chains and writes 12-byte descriptors, it never copies packet bytes.

struct Region {
  uintptr_t base, end;
  intptr_t delta;  // device address - host address
  bool owned;      // registered by us (unregister on removal)
};

// Batches hold it shared for as long as the GPU may read registered memory;
// register/unregister hold it exclusive, so a region is never unmapped under
// a running batch and concurrent batches do not serialise.
std::shared_mutex g_reg_mu;
std::vector<Region> g_regions;  // sorted by base, non-overlapping

// Device address of [p, p + n) if it lies inside one registered region.
bool device_addr(const std::vector<Region>& regs, const uint8_t* p, uint32_t n,
                 uint64_t* dev) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  size_t lo = 0, hi = regs.size();
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (regs[mid].base <= a) lo = mid + 1; else hi = mid;
  }
  if (lo == 0) return false;
  const Region& r = regs[lo - 1];
  if (a < r.base || a + n > r.end) return false;
  *dev = (uint64_t)(a + r.delta);
  return true;
}

// ---- walked batches -------------------------------------------------------------
//
// A batch runs in three phases.  (1) Every packet is walked like the reference
// walks it; packets are split into chunks of consecutive packets that the host
// pool walks in parallel, each chunk into its own piece list.  (2) A serial
// prefix over the chunks places them.  (3) The chunks, again in parallel,
// either write chain descriptors that point into registered memory (zero-copy:
// the kernel folds the bytes in place over PCIe; pipelined group by group
// with the walk) or pack the bytes into pinned
// staging for one H2D copy and one span launch.

struct Chunk {
  std::vector<Piece> pieces;
  PacketWalk w;
  int i0 = 0, i1 = 0;          // packets [i0, i1)
  uint64_t total = 0, packed = 0;
  uint32_t first_piece = 0;    // global index of pieces[0]
  uint64_t pack_base = 0;      // staging offset of packet i0
  bool odd = false, too_big = false, unmapped = false;
  bool long_piece = false;     // a piece over 65535 B: its group takes wide descriptors
};

// Per-thread scratch, reused across calls.
struct Batch {
  std::vector<Chunk> chunks;
  std::vector<uint32_t> pk_first, seed, bytes;  // pk_first is chunk-local
  std::vector<uint8_t> par;
};
thread_local Batch t_batch;

constexpr int kChunkMin = 1024;  // packets; below this one thread walks
// Host-mbuf batches of at most this many jobs are staged even over registered
// memory (run_host_batch; the hooks apply their own frame threshold).
constexpr int kStageBelowJobs = 128;
constexpr int kHookDeviceMin = 2048;  // frames; smaller hook batches take the host hook
// Staged batches up to this many bytes (descriptors + packed packet bytes) are
// folded in place from mapped pinned memory instead of being copied to HBM.
constexpr size_t kMappedStagingMax = 64 << 10;
// Staged batches of at least this many packet bytes overlap packing and copying.
constexpr uint64_t kStreamCopyMin = 32ull << 20;

// Device address of [p, p + n) with a one-entry cache of the last region hit
// (consecutive pieces almost always share a region).
inline bool device_addr_cached(const std::vector<Region>& regs, const uint8_t* p, uint32_t n,
                               const Region*& last, uint64_t* dev) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  if (last && a >= last->base && a + n <= last->end) {
    *dev = (uint64_t)(a + last->delta);
    return true;
  }
  if (!device_addr(regs, p, n, dev)) return false;
  last = &*(std::upper_bound(regs.begin(), regs.end(), a,
                             [](uintptr_t x, const Region& r) { return x < r.base; }) -
            1);
  return true;
}

// zero_copy_batch's "take the staging path instead" (not a UINET_CKSUM_* code).
constexpr int kFallback = 1;

// The zero-copy batch, pipelined by groups of `threads` chunks: walk the
// group (pool), place its chunks (serial prefix), write its chain descriptors
// into the pinned ring (pool), launch; then the next group is walked while
// the GPU folds this one.  Per group, in pinned memory read over PCIe:
//   seg_off u64[np_g] | seg_len u32[np_g] | pkt_seg u32[n_g + 1] | seed u32[n_g]
// Results land in the mapped c.h_out.  Called with g_reg_mu held (shared) and at
// least one region registered; returns kFallback (stream drained) when a
// group has an odd-parity start, an oversized packet or an unregistered piece.
template <typename WalkChunk>
int zero_copy_batch(Ctx& c, Batch& B, HostPool& pool, int threads, int nch, int n,
                    uint32_t flags, const WalkChunk& walk_chunk, bool trace) {
  using clk = std::chrono::steady_clock;
  const clk::time_point t0 = trace ? clk::now() : clk::time_point();
  double t_walk = 0, t_desc = 0;
  int rc = ctx_reserve(c, std::max<size_t>(c.h_cap, 1u << 20), (size_t)n, 0);
  if (rc) return rc;
  uint64_t lo_addr = ~0ull, hi_addr = 0;
  for (const Region& r : g_regions) {
    lo_addr = std::min(lo_addr, (uint64_t)(r.base + r.delta));
    hi_addr = std::max(hi_addr, (uint64_t)(r.end + r.delta));
  }
  // Packed 6-B descriptors (u32 offset, u16 length: launch_chains32) when every
  // registered byte lies within 4 GiB of the lowest and no piece is longer than
  // 65535 B, else the 12-B wide ones.  The kernel reads them over PCIe, where a
  // byte costs ~140x what it does in HBM.  A group holding a longer piece is
  // written wide (its chunks flag it).
#ifdef UINET_HOST_WIDE_DESC  // lab A/B build only (profiles/r04/scripts/r04_hostdesc.sh)
  const bool span32 = false;
#else
  const bool span32 = hi_addr - lo_addr <= 0x100000000ull;
#endif
  void* dout = nullptr;
  rc = record_hip(hipHostGetDevicePointer(&dout, c.h_out, 0));
  if (rc) return rc;
  void* dbuf = nullptr;
  rc = record_hip(hipHostGetDevicePointer(&dbuf, c.h_buf, 0));
  if (rc) return rc;
  const std::vector<Region>& regs = g_regions;
  const auto a16 = [](size_t b) { return (b + 15) & ~size_t(15); };
  const auto drain = [&]() { return ctx_wait(c); };
  // chunks per pipeline group: one per thread (one pool pass each; 2-64 per
  // thread lost in every A/B, profiles/r04/pruned/knobs.diff)
  const int group = std::max(1, threads);
  size_t ring = 0;  // next free byte of the descriptor ring in c.h_buf
  uint64_t total = 0;
  size_t np_all = 0;
  for (int g0 = 0; g0 < nch; g0 += group) {
    const int g1 = std::min(nch, g0 + group);
    clk::time_point ta = trace ? clk::now() : clk::time_point();
    pool.run(g1 - g0, threads, [&](int jj) { walk_chunk(g0 + jj); });
    clk::time_point tb = trace ? clk::now() : clk::time_point();
    if (trace) t_walk += std::chrono::duration<double, std::milli>(tb - ta).count();

    // place the group's chunks
    uint64_t np64 = 0, tot_g = 0;
    bool bad = false;
    for (int j = g0; j < g1; j++) {
      Chunk& C = B.chunks[(size_t)j];
      bad |= C.odd || C.too_big;
      C.first_piece = (uint32_t)np64;
      np64 += C.pieces.size();
      tot_g += C.total;
    }
    if (bad || np64 > 0xffffffffull) {
      rc = drain();
      return rc ? rc : kFallback;
    }
    const size_t np = (size_t)np64;
    const int i0 = B.chunks[(size_t)g0].i0;
    const int ng = B.chunks[(size_t)g1 - 1].i1 - i0;
    bool packed = span32;
    for (int j = g0; j < g1 && packed; j++) packed = !B.chunks[(size_t)j].long_piece;
    const size_t o_len = a16((packed ? 4 : 8) * np), o_ps = o_len + a16((packed ? 2 : 4) * np);
    const size_t o_sd = o_ps + a16(4 * ((size_t)ng + 1)), need = o_sd + a16(4 * (size_t)ng);
    if (ring + need > c.h_cap) {
      // the ring is full: wait for the launched groups, then reuse it from
      // the start (grown to hold every remaining group at this group's size)
      rc = drain();
      if (rc) return rc;
      ring = 0;
      if (need > c.h_cap) {
        rc = ctx_reserve(c, need * (size_t)((nch - g0 + group - 1) / group), (size_t)n, 0);
        if (rc) return rc;
        rc = record_hip(hipHostGetDevicePointer(&dbuf, c.h_buf, 0));
        if (rc) return rc;
      }
    }
    uint8_t* h = c.h_buf + ring;
    uint64_t* so = reinterpret_cast<uint64_t*>(h);
    uint32_t* sl = reinterpret_cast<uint32_t*>(h + o_len);
    uint32_t* so32 = reinterpret_cast<uint32_t*>(h);
    uint16_t* sl16 = reinterpret_cast<uint16_t*>(h + o_len);
    uint32_t* ps = reinterpret_cast<uint32_t*>(h + o_ps);
    uint32_t* sd = reinterpret_cast<uint32_t*>(h + o_sd);
    pool.run(g1 - g0, threads, [&](int jj) {
      Chunk& C = B.chunks[(size_t)(g0 + jj)];
      const Region* last = nullptr;
      const size_t k0 = C.first_piece;
      for (size_t k = 0; k < C.pieces.size(); k++) {
        uint64_t dev;
        if (!device_addr_cached(regs, C.pieces[k].p, C.pieces[k].n, last, &dev)) {
          C.unmapped = true;
          return;
        }
        if (packed) {
          so32[k0 + k] = (uint32_t)(dev - lo_addr);
          sl16[k0 + k] = (uint16_t)C.pieces[k].n;
        } else {
          so[k0 + k] = dev - lo_addr;
          sl[k0 + k] = C.pieces[k].n;
        }
      }
      for (int i = C.i0; i < C.i1; i++) {
        ps[i - i0] = C.first_piece + B.pk_first[(size_t)i];
        sd[i - i0] = B.seed[(size_t)i];
      }
    });
    ps[ng] = (uint32_t)np;
    for (int j = g0; j < g1; j++) bad |= B.chunks[(size_t)j].unmapped;
    if (trace) t_desc += std::chrono::duration<double, std::milli>(clk::now() - tb).count();
    if (bad) {
      rc = drain();
      return rc ? rc : kFallback;
    }
    uint8_t* d = static_cast<uint8_t*>(dbuf) + ring;
    if (packed)
      rc = launch_chains32(reinterpret_cast<const void*>(lo_addr),
                           reinterpret_cast<const uint32_t*>(d),
                           reinterpret_cast<const uint16_t*>(d + o_len),
                           reinterpret_cast<const uint32_t*>(d + o_ps), nullptr, nullptr,
                           reinterpret_cast<const uint32_t*>(d + o_sd),
                           static_cast<uint16_t*>(dout) + i0, (uint32_t)ng, flags,
                           np ? (uint32_t)(tot_g / np) : 1u, c.stream);
    else
      rc = launch_chains(reinterpret_cast<const void*>(lo_addr),
                         reinterpret_cast<const uint64_t*>(d),
                         reinterpret_cast<const uint32_t*>(d + o_len),
                         reinterpret_cast<const uint32_t*>(d + o_ps), nullptr, nullptr,
                         reinterpret_cast<const uint32_t*>(d + o_sd),
                         static_cast<uint16_t*>(dout) + i0, (uint32_t)ng, flags,
                         np ? (uint32_t)(tot_g / np) : 1u, c.stream);
    if (rc) {
      (void)drain();
      return rc;
    }
    ring += need;
    total += tot_g;
    np_all += np;
  }
  const clk::time_point tw = trace ? clk::now() : clk::time_point();
  rc = drain();
  if (rc) return rc;
  if (trace)
    fprintf(stderr,
            "uinet_cksum host batch: n=%d pieces=%zu bytes=%llu zero-copy threads=%d groups=%d "
            "| walk %.3f descriptors %.3f (overlapped with the GPU) wait %.3f total %.3f ms\n",
            n, np_all, (unsigned long long)total, threads, (nch + group - 1) / group, t_walk,
            t_desc, std::chrono::duration<double, std::milli>(clk::now() - tw).count(),
            std::chrono::duration<double, std::milli>(clk::now() - t0).count());
  return UINET_CKSUM_OK;
}

// ---- device walk (cksum_walk.hip) -------------------------------------------
//
// Registered memory and a chain-walking batch: the host writes only the jobs
// (head, len, skip, seed: 20 B per packet) into pinned memory; the GPU walks
// the chains (k_walk_mbufs) into a K-slot segment list in HBM and folds it with
// the chain kernel, reading mbuf headers and packet bytes in place over PCIe.
// The host thread sleeps in ctx_wait meanwhile.

enum WalkKind { kWalkNone = 0, kWalkSkip = 1, kWalkPseudo = 2 };
constexpr int kWalkGroupMin = 16384;  // packets per walk/fold pipeline group, at least

// The HBM work area of a walk + fold of N jobs at K segment slots per job:
// seg_off u64[N K] | seg_len u32[N K] | pkt_seg u32[N + 1] | len | skip | seed.
struct WalkWork {
  size_t sl, ps, ln, sk, sd, end;
};
WalkWork walk_work(size_t N, uint32_t K) {
  const auto a16 = [](size_t b) { return (b + 15) & ~size_t(15); };
  WalkWork w;
  w.sl = a16(8 * N * K);
  w.ps = w.sl + a16(4 * N * K);
  w.ln = w.ps + a16(4 * (N + 1));
  w.sk = w.ln + a16(4 * N);
  w.sd = w.sk + a16(4 * N);
  w.end = w.sd + a16(4 * N);
  return w;
}

// The context's side stream and its fork / join events, created on first use.
int ctx_side(Ctx& c) {
  int rc = UINET_CKSUM_OK;
  if (!c.side) rc = record_hip(hipStreamCreateWithFlags(&c.side, hipStreamNonBlocking));
  if (!rc && !c.fork) rc = record_hip(hipEventCreateWithFlags(&c.fork, hipEventDisableTiming));
  if (!rc && !c.join) rc = record_hip(hipEventCreateWithFlags(&c.join, hipEventDisableTiming));
  return rc;
}

// Enqueues the walk (k_walk_mbufs) and the fold (k_chains_pipe) of N jobs --
// device-readable arrays jm / jl / js / jd (jd may be NULL) -- over the work
// area at `wa` (HBM), results into `out`, status bits into `dstatus` (zeroed
// by the caller, on c.stream, before this).  Groups of consecutive jobs
// alternate between the context's stream and a side stream, each group's walk
// then its fold: group g + 1's walk (a chase of dependent PCIe reads) runs
// while group g's fold streams its bytes.  Everything ends on c.stream; on an
// error nothing is left running.
int launch_walk_fold(Ctx& c, const uint64_t* jm, const int32_t* jl, const int32_t* js,
                     const uint32_t* jd, const WalkRegionHost* regs, int nreg, uint64_t lo,
                     size_t N, uint32_t K, bool pseudo, uint8_t* wa, uint32_t* dstatus,
                     uint16_t* out, uint32_t flags) {
#ifndef UINET_WALK_GROUPS  // lab A/B: -DUINET_WALK_GROUPS=1 walks the batch in one group
#define UINET_WALK_GROUPS 8
#endif
  const int n = (int)N;
  const int groups = n >= 2 * kWalkGroupMin ? std::min(UINET_WALK_GROUPS, n / kWalkGroupMin) : 1;
  int rc = groups > 1 ? ctx_side(c) : UINET_CKSUM_OK;
  if (rc) return rc;
  const WalkWork W = walk_work(N, K);
  if (groups > 1) rc = record_hip(hipEventRecord(c.fork, c.stream));
  if (!rc && groups > 1) rc = record_hip(hipStreamWaitEvent(c.side, c.fork, 0));
  for (int g = 0; g < groups && !rc; g++) {
    const size_t i0 = N * (size_t)g / (size_t)groups, i1 = N * (size_t)(g + 1) / (size_t)groups;
    const uint32_t ng = (uint32_t)(i1 - i0);
    hipStream_t sg = (g & 1) ? c.side : c.stream;
    rc = launch_walk_mbufs(jm + i0, jl + i0, js + i0, jd ? jd + i0 : nullptr, regs, nreg, ng, K,
                           (uint32_t)(i0 * K), lo, pseudo,
                           reinterpret_cast<uint64_t*>(wa) + i0 * K,
                           reinterpret_cast<uint32_t*>(wa + W.sl) + i0 * K,
                           reinterpret_cast<uint32_t*>(wa + W.ps) + i0,
                           reinterpret_cast<uint32_t*>(wa + W.ln) + i0,
                           reinterpret_cast<uint32_t*>(wa + W.sk) + i0,
                           reinterpret_cast<uint32_t*>(wa + W.sd) + i0, dstatus, sg);
    // the group's rows are indexed from the list's row 0 (pkt_seg holds
    // global row numbers)
    if (!rc)
      rc = launch_chains(reinterpret_cast<const void*>(lo), reinterpret_cast<const uint64_t*>(wa),
                         reinterpret_cast<const uint32_t*>(wa + W.sl),
                         reinterpret_cast<const uint32_t*>(wa + W.ps) + i0,
                         reinterpret_cast<const uint32_t*>(wa + W.ln) + i0,
                         reinterpret_cast<const uint32_t*>(wa + W.sk) + i0,
                         jd ? reinterpret_cast<const uint32_t*>(wa + W.sd) + i0 : nullptr,
                         out + i0, ng, flags, 0, sg);
  }
  if (!rc && groups > 1) rc = record_hip(hipEventRecord(c.join, c.side));
  if (!rc && groups > 1) rc = record_hip(hipStreamWaitEvent(c.stream, c.join, 0));
  if (rc && groups > 1) (void)hipStreamSynchronize(c.side);  // nothing left running
  return rc;
}

// The region table in the form the device walk reads, and the lowest device
// address of a registered byte (the chain kernel's base).  0 regions or more
// than the walk takes: false.  Called with g_reg_mu held.
bool walk_regions(WalkRegionHost* R, size_t cap, size_t* nreg, uint64_t* lo) {
  const size_t n = g_regions.size();
  if (n == 0 || n > (size_t)kWalkRegionsMax || n > cap) return false;
  uint64_t l = ~0ull;
  for (size_t k = 0; k < n; k++) {
    const Region& r = g_regions[k];
    R[k] = WalkRegionHost{r.base, r.end, (int64_t)r.delta};
    l = std::min(l, (uint64_t)(r.base + r.delta));
  }
  *nreg = n;
  *lo = l;
  return true;
}

// Next row size from the longest chain seen (the next batch on this thread
// starts from it).
uint32_t walk_k_for(uint32_t longest) {
  uint32_t k = 4;
  while (k < longest) k *= 2;
  return k;
}

// Whether the first, middle and last chains of a batch start in registered
// memory.  When only the packet bytes are registered (the zero-copy setup),
// the device paths would launch their kernels only to find every mbuf
// unmapped and hand the batch back; this sends it to the host walk first.
// (A batch that passes and still holds an unregistered mbuf is caught by the
// kernels' status word as before.)  Called with g_reg_mu held.
template <typename HeadAt>
bool heads_registered(int n, const HeadAt& head_at) {
  const int idx[3] = {0, n / 2, n - 1};
  for (int i : idx) {
    const uint8_t* m = reinterpret_cast<const uint8_t*>(head_at(i));
    uint64_t dev;
    if (m && !device_addr(g_regions, m, 32, &dev)) return false;
  }
  return true;
}

// job(i) -> Job (the in_cksum_skip form; len and skip as the caller gave
// them).  Returns kFallback (nothing delivered) when the batch must take the
// host walk.  Called with g_reg_mu held (shared) and at least one region.
template <typename HeadFn, typename JobFn>
int device_walk_batch(Ctx& c, HostPool& pool, int threads, int cs, int n, uint32_t flags,
                      WalkKind kind, bool seeded, const HeadFn& head, const JobFn& job,
                      uint16_t* out16, unsigned* out32, bool trace) {
  using clk = std::chrono::steady_clock;
  const clk::time_point t0 = trace ? clk::now() : clk::time_point();
  const size_t nreg_all = g_regions.size();
  if (nreg_all == 0 || nreg_all > (size_t)kWalkRegionsMax) return kFallback;
  // head(i) is side-effect free (job(i) of a hook parses the frame)
  if (!heads_registered(n, [&](int i) { return head(i).m; })) return kFallback;
  // the chain batches walk into a segment list by default: over PCIe a
  // fused wave waits out each hop's round trip between its folds, the walk
  // kernel keeps a hop per lane in flight (config 3: 9.6 ms against 16.0,
  // profiles/r06/host_cpu_r06b.md)
  const bool fused = tuning().walk_device == 3;
  uint32_t K = c.walk_k ? c.walk_k : 4;
  const auto a16 = [](size_t b) { return (b + 15) & ~size_t(15); };
  const size_t N = (size_t)n;
  if ((uint64_t)N * K > 0xffffffffull) return kFallback;  // rows indexed by u32
  // pinned: heads u64 | len i32 | skip i32 | seed u32 | regions | status u32[2]
  const size_t h_len = a16(8 * N), h_skip = h_len + a16(4 * N), h_seed = h_skip + a16(4 * N);
  const size_t h_reg = h_seed + (seeded ? a16(4 * N) : 0);
  const size_t h_st = h_reg + a16(sizeof(WalkRegionHost) * nreg_all), h_end = h_st + 16;
  // HBM: status u32[4] | the two-pass walk's work area
  int rc = ctx_reserve(c, h_end, N, fused ? 16 : 16 + walk_work(N, K).end);
  if (rc) return rc;
  uint8_t* h = c.h_buf;
  uint64_t* heads = reinterpret_cast<uint64_t*>(h);
  int32_t* jl = reinterpret_cast<int32_t*>(h + h_len);
  int32_t* js = reinterpret_cast<int32_t*>(h + h_skip);
  uint32_t* jd = reinterpret_cast<uint32_t*>(h + h_seed);
  // the jobs, in chunks of consecutive packets on the host pool (a hook's
  // jobs are made -- its headers parsed -- here)
  const int nch = (n + cs - 1) / cs;
  pool.run(nch, threads, [&](int j) {
    const int i1 = std::min(n, (j + 1) * cs);
    for (int i = j * cs; i < i1; i++) {
      const Job J = job(i);
      heads[i] = reinterpret_cast<uint64_t>(J.m);
      jl[i] = J.len;
      js[i] = J.skip;
      if (seeded) jd[i] = J.seed;
    }
  });
  size_t nreg = 0;
  uint64_t lo_addr = 0;
  (void)walk_regions(reinterpret_cast<WalkRegionHost*>(h + h_reg), nreg_all, &nreg, &lo_addr);
  const clk::time_point t1 = trace ? clk::now() : clk::time_point();
  void* dh = nullptr;
  rc = record_hip(hipHostGetDevicePointer(&dh, c.h_buf, 0));
  if (rc) return rc;
  void* dout = nullptr;
  rc = record_hip(hipHostGetDevicePointer(&dout, c.h_out, 0));
  if (rc) return rc;
  const uint8_t* dj = static_cast<const uint8_t*>(dh);
  volatile uint32_t* st = reinterpret_cast<volatile uint32_t*>(h + h_st);
  if (fused) {
    // one launch walks the chains and folds their bytes (cksum_mbufs.hip),
    // reading jobs, mbuf headers and packet bytes in place over PCIe
    uint32_t* dstatus = reinterpret_cast<uint32_t*>(c.d_buf);
    rc = record_hip(hipMemsetAsync(dstatus, 0, 8, c.stream));
    if (!rc)
      rc = launch_mbufs_xlate(reinterpret_cast<const uint64_t*>(dj),
                              reinterpret_cast<const int32_t*>(dj + h_len),
                              reinterpret_cast<const int32_t*>(dj + h_skip),
                              seeded ? reinterpret_cast<const uint32_t*>(dj + h_seed) : nullptr,
                              reinterpret_cast<const WalkRegionHost*>(dj + h_reg), (int)nreg,
                              kind == kWalkPseudo, static_cast<uint16_t*>(dout), (uint32_t)N,
                              flags, dstatus, c.stream);
    if (!rc)
      rc = record_hip(hipMemcpyAsync(h + h_st, dstatus, 8, hipMemcpyDeviceToHost, c.stream));
    const int wrc = ctx_wait(c);
    if (rc) return rc;
    if (wrc) return wrc;
    if (st[0]) return kFallback;  // a job the host walk must take
    deliver(c, n, out16, out32);
    note_device_walk();
    if (trace)
      fprintf(stderr,
              "uinet_cksum host batch: n=%d device walk (fused) | jobs %.3f fold %.3f total "
              "%.3f ms\n",
              n, std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(clk::now() - t1).count(),
              std::chrono::duration<double, std::milli>(clk::now() - t0).count());
    return UINET_CKSUM_OK;
  }
  for (int attempt = 0; attempt < 2; attempt++) {
    rc = ctx_reserve(c, h_end, N, 16 + walk_work(N, K).end);
    if (rc) return rc;
    uint8_t* d = c.d_buf;
    uint32_t* dstatus = reinterpret_cast<uint32_t*>(d);
    rc = record_hip(hipMemsetAsync(dstatus, 0, 8, c.stream));
    if (!rc)
      rc = launch_walk_fold(c, reinterpret_cast<const uint64_t*>(dj),
                            reinterpret_cast<const int32_t*>(dj + h_len),
                            reinterpret_cast<const int32_t*>(dj + h_skip),
                            seeded ? reinterpret_cast<const uint32_t*>(dj + h_seed) : nullptr,
                            reinterpret_cast<const WalkRegionHost*>(dj + h_reg), (int)nreg,
                            lo_addr, N, K, kind == kWalkPseudo, d + 16, dstatus,
                            static_cast<uint16_t*>(dout), flags);
    if (!rc)
      rc = record_hip(hipMemcpyAsync(h + h_st, dstatus, 8, hipMemcpyDeviceToHost, c.stream));
    const int wrc = ctx_wait(c);
    if (rc) return rc;
    if (wrc) return wrc;
    if (st[0]) return kFallback;  // a job the host walk must take
    const uint32_t longest = st[1];
    const uint32_t k2 = walk_k_for(longest);
    c.walk_k = k2;
    if (longest <= K) {
      deliver(c, n, out16, out32);
      note_device_walk();
      if (trace)
        fprintf(stderr,
                "uinet_cksum host batch: n=%d device walk K=%u longest=%u | jobs %.3f fold "
                "%.3f total %.3f ms\n",
                n, K, longest, std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(clk::now() - t1).count(),
                std::chrono::duration<double, std::milli>(clk::now() - t0).count());
      return UINET_CKSUM_OK;
    }
    if (k2 > kWalkKMax || (uint64_t)N * k2 > 0xffffffffull) return kFallback;
    K = k2;  // a chain longer than K: walk again with room for it
  }
  return kFallback;
}

// ---- single-mbuf spans (host-resident batches whose sums lie in one mbuf) ---
//
// The netmap RX shape (uinet_if_netmap.c:1472-1523: one mbuf per received
// frame) and any batch whose summed bytes all lie in each packet's first
// mbuf: the host reads each head mbuf's m_next / m_data / m_len (one line it
// would read to walk anyway), writes a packed span descriptor (u32 offset,
// u16 length: 6 B) into pinned memory, and the span kernel folds the bytes
// in place over PCIe.  No mbuf line crosses the link (the device walk moves a
// 128-B line per mbuf for 32 useful bytes), so the link carries the packet
// bytes and 6 B per packet.  Pipelined by groups: the host writes group g + 1
// while the GPU folds group g.  Returns kFallback (stream drained) at the
// first packet whose sum needs a second mbuf, whose bytes lie outside the
// registered regions, or that is outside the reference's contract; the
// caller then takes the general paths.  Called with g_reg_mu held (shared)
// and at least one region registered.
// Packets per pipeline group (16 K: 7 % slower; 256 K: the same;
// profiles/r06/r06sab/).
constexpr int kSpanGroup = 1 << 16;
// Head mbufs are requested this many packets ahead.  One host thread spends
// ~3 ns per packet and a head mbuf (a DRAM line, often on a page not touched
// yet) takes ~100-300 ns to arrive, so the distance must cover ~100 packets:
// config 2, one thread, host CPU per 1,000 packets at distance 8 / 32 / 64 /
// 128 / 192: 6.3-6.8 / 4.4 / 3.4 / 2.8 / 2.8 us (profiles/r06/r06pf*/).
constexpr int kSpanPrefetch = 128;
// Groups summing fewer bytes are folded in place (a copy's fixed cost).
constexpr uint64_t kSpanDmaMin = 1u << 20;

// The span path's common packet (span_fast_batch, once a group has its
// origin): the sum lies in the head mbuf, inside one region and the packed
// window [lo, hi) of host addresses; offsets are from hb.  Writes packets
// [i, e) until the first that is not such a packet and returns its index (e
// for none).  Out of line and with its own copies of the accessors (captured
// by value), so the loop no longer reloads its arrays through the captures:
// ~40 instructions per packet, every branch predictable, ~2 ns per packet on
// config 2 where the general loop spent ~3 whether the heads were in cache or
// in DRAM (instructions, reloads and spills, not misses: profiles/r06/r06pass/,
// r06fp*/).
struct SpanRun {
  uintptr_t hb, lo, hi;
  uint64_t add = 0;   // summed bytes written
  uintptr_t top = 0;  // highest host address + 1 written, 0 for none
};
template <typename HeadFn, typename JobFn>
__attribute__((noinline)) int span_run(HeadFn head, JobFn job, int i, const int e, uint32_t* so,
                                       uint16_t* sl, uint32_t* sd, SpanRun& R) {
  const uintptr_t hb = R.hb, lo = R.lo, hi = R.hi;
  uint64_t add = 0;
  uintptr_t top = 0;
  const auto one = [&](int k) -> bool {
    const Job J = job(k);
    const MbufHdr* m = J.m;
    if (!m) return false;
    const long ml = m->m_len, S = J.skip, L = J.len;
    const uintptr_t a = reinterpret_cast<uintptr_t>(m->m_data) + (uintptr_t)S;
    const long span = std::min(L, ml) - S;
    // 0 <= S < ml, S < L, [S, L) ends in this mbuf or nothing follows it
    // (in_cksum.c:203-229), a packed length, inside [lo, hi)
    const bool ok = (S >= 0) & (S < ml) & (L > S) & ((L <= ml) | (m->m_next == nullptr)) &
                    (span <= 0xffffL) & (a >= lo) & (a + (uintptr_t)span <= hi);
    if (!ok) return false;
    so[k] = (uint32_t)(a - hb);
    sl[k] = (uint16_t)span;
    if (sd) sd[k] = J.seed;
    add += (uint64_t)span;
    top = std::max(top, a + (uintptr_t)span);
    return true;
  };
  // (a prefetch of a null head is dropped by the core: no test)
  const int e1 = std::max(i, e - kSpanPrefetch);
  for (; i < e1; i++) {
    __builtin_prefetch(head(i + kSpanPrefetch).m, 0, 3);
    if (!one(i)) break;
  }
  if (i >= e1)
    for (; i < e; i++)
      if (!one(i)) break;
  R.add = add;
  R.top = top;
  return i;
}
template <typename HeadFn, typename JobFn>
int span_fast_batch(Ctx& c, int n, uint32_t flags, WalkKind kind, bool seeded, const HeadFn& head,
                    const JobFn& job, uint16_t* out16, unsigned* out32) {
  uint64_t lo_addr = ~0ull, hi_addr = 0, big_base = 0, big_len = 0;
  for (const Region& r : g_regions) {
    lo_addr = std::min(lo_addr, (uint64_t)(r.base + r.delta));
    hi_addr = std::max(hi_addr, (uint64_t)(r.end + r.delta));
    if (r.end - r.base > big_len) {
      big_len = r.end - r.base;
      big_base = (uint64_t)(r.base + r.delta);
    }
  }
  // Packed descriptors (u32 offset, u16 length) from a base every summed
  // byte lies within 4 GiB of: the lowest registered byte when all regions
  // fit that window, else the largest region's start (the packet arena, with
  // the mbufs registered elsewhere); a span outside it sends the batch round
  // once more with wide descriptors (u64, u32).
  const bool all_packed = hi_addr - lo_addr <= 0x100000000ull;
  for (int attempt = 0; attempt < 2; attempt++) {
    const bool packed = attempt == 0;
    const uint64_t base = packed && !all_packed ? big_base : lo_addr;
    bool outside = false;  // packed: a span outside [base, base + 4 GiB)
    const uint32_t max_span = packed ? 0xffffu : 0x7fffffffu;
    const auto a16 = [](size_t b) { return (b + 15) & ~size_t(15); };
    const int G = std::min(n, kSpanGroup);
    const size_t o_len = a16((packed ? 4 : 8) * (size_t)G);
    const size_t o_sd = o_len + a16((packed ? 2 : 4) * (size_t)G);
    const size_t need = o_sd + (seeded ? a16(4 * (size_t)G) : 0);
    const int groups = (n + G - 1) / G;
    // every group's descriptors in pinned memory, and their copy in HBM: the
    // span kernel reads descriptors with scalar loads, each a round trip that
    // over PCIe its two-step prefetch does not cover (read in place the fold
    // ran at 47 GB/s); one DMA per group puts them in HBM first
    int rc = ctx_reserve(c, need * (size_t)groups, (size_t)n, need * (size_t)groups);
    if (rc) return rc;
    void* dout = nullptr;
    rc = record_hip(hipHostGetDevicePointer(&dout, c.h_out, 0));
    if (rc) return rc;
    const std::vector<Region>& regs = g_regions;
    bool bad = false;
    uint64_t dma_bytes = 0, link_bytes = 0;  // link_bytes: what crosses PCIe, at least
    std::chrono::steady_clock::time_point t_first;  // the first group's launch
    // UINET_CKSUM_TRACE_HOST=1: where the calling thread's time goes (tools)
    static const bool trace = getenv("UINET_CKSUM_TRACE_HOST") != nullptr;
    using tclk = std::chrono::steady_clock;
    const tclk::time_point t_in = trace ? tclk::now() : tclk::time_point();
    double pass_us = 0;
    for (int g = 0; g < groups && !bad && !outside; g++) {
      const int i0 = g * G, ng = std::min(G, n - i0);
      uint8_t* h = c.h_buf + need * (size_t)g;
      uint32_t* so = reinterpret_cast<uint32_t*>(h);
      uint16_t* sl = reinterpret_cast<uint16_t*>(h + o_len);
      uint64_t* wo = reinterpret_cast<uint64_t*>(h);
      uint32_t* wl = reinterpret_cast<uint32_t*>(h + o_len);
      uint32_t* sd = reinterpret_cast<uint32_t*>(h + o_sd);
      // One thread, the caller: a head mbuf line per packet is all the host
      // reads, and the GPU's fold of a group takes longer than the host's
      // pass over it, so helpers would only add CPU time.
      uint64_t gb = 0;  // the group's summed bytes: its mean span picks the geometry
      const tclk::time_point t_g = trace ? tclk::now() : tclk::time_point();
      const Region* last = nullptr;
      // Offsets are relative to the group's origin `gbase` (its first span's
      // address, 256-B aligned within its region), so that a dense group can
      // be copied to HBM as one run with its descriptors as they are; a span
      // before the origin sends the group's offsets back to the batch's base.
      // The span kernel may read its base itself (an empty pair's offset is
      // 0), and gbase is registered memory, as is base.
      const uint64_t window = packed ? 0x100000000ull : ~0ull;
      uint64_t gbase = 0, g_hi = 0;
      bool local = false, has_gbase = false;
      const Region* g_reg = nullptr;  // gbase's region
      bool one_reg = true;
      const int e = i0 + ng;
      for (int i = i0; i < e; i++) {
        if (packed && local) {
          // The common packet, once the group has its origin (span_run); any
          // other packet leaves to the general code below, which decides it
          // exactly as before.
          SpanRun R;
          R.hb = (uintptr_t)((intptr_t)gbase - g_reg->delta);
          R.lo = std::max(g_reg->base, R.hb);
          R.hi = std::min(g_reg->end, R.hb + (uintptr_t)window);
          i = span_run(head, job, i, e, so - i0, sl - i0, seeded ? sd - i0 : nullptr, R);
          gb += R.add;
          if (R.top) g_hi = std::max(g_hi, (uint64_t)((intptr_t)R.top + g_reg->delta));
          if (i >= e) break;
        }
        if (i + kSpanPrefetch < e) {  // (the locality hint makes no difference, r06pfab/)
          const auto r = head(i + kSpanPrefetch);
          if (r.m) __builtin_prefetch(r.m, 0, 3);
        }
        const Job J = job(i);
        const MbufHdr* m = J.m;
        uint64_t off = 0;
        uint32_t len = 0;
        if (J.skip < 0) {
          bad = true;
          break;
        }
        if (m && J.len > J.skip) {
          // in_cksum.c:203-229 (and :254-272, off0 = skip): the sum stays in
          // this mbuf when [skip, len) ends in it, or when nothing follows it
          const long ml = m->m_len, S = J.skip, L = J.len;
          const bool more = m->m_next != nullptr;
          const bool second = S < ml ? (L > ml && more)
                                     : (more || (kind == kWalkPseudo && S > ml));
          if (ml < 0 || second) {
            bad = true;  // the sum needs a second mbuf
            break;
          }
          if (S < ml) {
            const long span = std::min(L, ml) - S;
            uint64_t dev;
            if (span > 0x7fffffffL ||
                !device_addr_cached(regs, m->m_data + S, (uint32_t)span, last, &dev)) {
              bad = true;
              break;
            }
            if (span > (long)max_span) {
              outside = true;  // packed only: wide descriptors take it
              break;
            }
            if (!has_gbase) {
              has_gbase = local = true;
              g_reg = last;
              gbase = std::max(dev & ~uint64_t(255), (uint64_t)(last->base + last->delta));
            }
            if (local && (dev < gbase || dev - gbase + (uint64_t)span > window)) {
              // back to the batch's base: the group's earlier offsets move
              if (gbase < base) {
                outside = true;
                break;
              }
              const uint64_t sh = gbase - base;
              for (int k = i0; k < i; k++) {
                const bool nz = packed ? sl[k - i0] != 0 : wl[k - i0] != 0;
                if (!nz) continue;
                const uint64_t o = (packed ? (uint64_t)so[k - i0] : wo[k - i0]) + sh;
                const uint64_t l = packed ? (uint64_t)sl[k - i0] : (uint64_t)wl[k - i0];
                if (o + l > window) {
                  outside = true;
                  break;
                }
                if (packed) so[k - i0] = (uint32_t)o;
                else wo[k - i0] = o;
              }
              if (outside) break;
              local = false;
            }
            if (local) {
              off = dev - gbase;
            } else {
              if (dev < base || dev - base + (uint64_t)span > window) {
                outside = true;
                break;
              }
              off = dev - base;
            }
            len = (uint32_t)span;
            g_hi = std::max(g_hi, dev + (uint64_t)span);
            one_reg &= last == g_reg;
          }
        }
        if (packed) {
          so[i - i0] = (uint32_t)off;
          sl[i - i0] = (uint16_t)len;
        } else {
          wo[i - i0] = off;
          wl[i - i0] = len;
        }
        if (seeded) sd[i - i0] = J.seed;
        gb += len;
      }
      if (bad || outside) break;
      if (trace)
        pass_us += std::chrono::duration<double, std::micro>(tclk::now() - t_g).count();
      // A dense group (its bytes one run of a region, at most 1/16 of it
      // between packets: config 2, netmap rings of full frames) goes to HBM by
      // one DMA copy and is folded there: the copy engines move 57.6 GB/s
      // over the link where the span kernel's own reads of host memory get
      // 48-52 (profiles/r06/).  The copy keeps every byte's address mod 256,
      // so chunks and parities are the same; the kernel's base moves so that
      // the descriptors written above address the copy.
      uint64_t kbase = local ? gbase : base;
      uint32_t fl = flags | kFlagHostBytes;  // read over PCIe: temporal loads
      if (local && one_reg && gb >= kSpanDmaMin) {
        const uint64_t lo_copy = gbase;
        const uint64_t range = g_hi - lo_copy;
        if (range <= gb + gb / 16 + 4096) {
          // 256 B of headroom: a span's first chunk may start up to 15 B
          // before the copy's first byte (masked, but loaded)
          const size_t want = (size_t)range + 1024;
          if (want > c.stage_cap) {  // grown between groups: drain what may read it
            rc = ctx_wait(c);
            if (rc) return rc;
            if (c.d_stage) (void)hipFree(c.d_stage);
            c.d_stage = nullptr;
            c.stage_cap = 0;
            size_t cap = std::max<size_t>(want, size_t(64) << 20);
            rc = record_hip(hipMalloc((void**)&c.d_stage, cap));
            if (rc) return rc;
            c.stage_cap = cap;
          }
          uint8_t* dst = c.d_stage + 256 + (lo_copy & 255);
          // (from the device alias as a device-to-device or default-kind
          // copy: the same time and host CPU, profiles/r06/r06dma/)
          rc = record_hip(hipMemcpyAsync(dst, reinterpret_cast<const void*>(lo_copy - g_reg->delta),
                                         (size_t)range, hipMemcpyHostToDevice, c.stream));
          if (rc) {
            (void)ctx_wait(c);
            return rc;
          }
          // the offsets (from gbase) now address the copy
          kbase = reinterpret_cast<uint64_t>(dst);
          fl = flags;  // HBM: non-temporal loads
          dma_bytes += range;
          link_bytes += range - gb;  // gb is added below
        }
      }
      uint8_t* d = c.d_buf + need * (size_t)g;
      rc = record_hip(hipMemcpyAsync(d, h, need, hipMemcpyHostToDevice, c.stream));
      if (rc) {
        (void)ctx_wait(c);
        return rc;
      }
      const uint32_t* dsd = seeded ? reinterpret_cast<const uint32_t*>(d + o_sd) : nullptr;
      const uint32_t hint = ng ? (uint32_t)(gb / (uint64_t)ng) : 0u;
      if (packed)
        rc = launch_spans32(reinterpret_cast<const void*>(kbase),
                            reinterpret_cast<const uint32_t*>(d),
                            reinterpret_cast<const uint16_t*>(d + o_len), dsd, nullptr,
                            static_cast<uint16_t*>(dout) + i0, (uint32_t)ng, fl, hint, c.stream);
      else
        rc = launch_spans(reinterpret_cast<const void*>(kbase),
                          reinterpret_cast<const uint64_t*>(d),
                          reinterpret_cast<const uint32_t*>(d + o_len), dsd, nullptr,
                          static_cast<uint16_t*>(dout) + i0, (uint32_t)ng, fl, hint, c.stream);
      if (rc) {
        (void)ctx_wait(c);
        return rc;
      }
      link_bytes += gb;
      if (g == 0) t_first = std::chrono::steady_clock::now();
    }
    // The GPU cannot have moved the bytes over the link faster than 64 GB/s
    // (PCIe 5.0 x16; the copy engines reach 57.6 here) since the first launch:
    // that lower bound is slept in one nap.
    long min_us = 0;
    if (!bad && !outside && link_bytes > 0) {
      const long since = (long)std::chrono::duration_cast<std::chrono::microseconds>(
                             std::chrono::steady_clock::now() - t_first)
                             .count();
      min_us = std::max(0l, (long)(link_bytes / 64000u) - since);
    }
    const tclk::time_point t_w = trace ? tclk::now() : tclk::time_point();
    rc = ctx_wait(c, min_us);  // the groups launched so far (their buffers are reused)
    if (rc) return rc;
    if (bad) return kFallback;
    if (outside) continue;
    const tclk::time_point t_d = trace ? tclk::now() : tclk::time_point();
    deliver(c, n, out16, out32);
    note_span_fast(dma_bytes);
    if (trace) {
      const auto us = [](tclk::time_point a, tclk::time_point b) {
        return std::chrono::duration<double, std::micro>(b - a).count();
      };
      fprintf(stderr,
              "uinet_cksum spans: n=%d groups=%d dma %.1f MB | pass %.0f us, calls %.0f us, "
              "wait %.0f us (slept %ld), deliver %.0f us, total %.0f us\n",
              n, groups, dma_bytes / 1e6, pass_us, us(t_in, t_w) - pass_us, us(t_w, t_d), min_us,
              us(t_d, tclk::now()), us(t_in, tclk::now()));
    }
    return UINET_CKSUM_OK;
  }
  return kFallback;
}

// ---- single-mbuf spans, heads read by the GPU ------------------------------
//
// The span path above with the mbufs registered too: instead of the calling
// thread reading every head mbuf (one DRAM line per packet, 2.7-3.9 us of CPU
// per 1,000 packets by host), it copies the jobs (20 B per packet, sequential)
// and the GPU reads the heads over PCIe (k_span_walk: one 128-B link line per
// packet).  Per group of kSpanGroup packets, on the side stream: the walk, then
// its stats to pinned memory; the calling thread waits for each group's stats
// and then, on the main stream, copies a dense group to HBM as one run (as the
// host span path does) or folds it in place, after rebasing its offsets.  The
// walks run ahead on their stream while the copies of earlier groups use the
// copy engines.  Returns kFallback (everything drained) when any packet is
// not the shape; the caller then takes the other paths.  Called with
// g_reg_mu held (shared).
template <typename HeadFn, typename JobFn>
int span_walk_batch(Ctx& c, int n, uint32_t flags, WalkKind kind, bool seeded, const HeadFn& head,
                    const JobFn& job, uint16_t* out16, unsigned* out32) {
  const size_t nreg_all = g_regions.size();
  if (nreg_all == 0 || nreg_all > (size_t)kWalkRegionsMax) return kFallback;
  if (!heads_registered(n, [&](int i) { return head(i).m; })) return kFallback;
  // a quick look at three heads: a chain whose sum needs its second mbuf
  // means the batch is not this shape (config 3), before anything is queued
  {
    const int idx[3] = {0, n / 2, n - 1};
    for (int i : idx) {
      const auto r = head(i);
      if (r.m && r.m->m_next && r.limit > r.m->m_len) return kFallback;
    }
  }
  using clk = std::chrono::steady_clock;
  static const bool trace = getenv("UINET_CKSUM_TRACE_HOST") != nullptr;
  const clk::time_point t_in = trace ? clk::now() : clk::time_point();
  const auto a16 = [](size_t b) { return (b + 15) & ~size_t(15); };
  const size_t N = (size_t)n;
  const int G = std::min(n, kSpanGroup);
  const int groups = (n + G - 1) / G;
  // pinned: heads u64 | len i32 | skip i32 | seed u32 | regions | stats u64[6] x groups
  //         | the stats' initial value u64[6]
  const size_t h_len = a16(8 * N), h_skip = h_len + a16(4 * N), h_seed = h_skip + a16(4 * N);
  const size_t h_reg = h_seed + (seeded ? a16(4 * N) : 0);
  const size_t h_st = h_reg + a16(sizeof(WalkRegionHost) * nreg_all);
  const size_t h_init = h_st + 48 * (size_t)groups, h_end = h_init + 48;
  // HBM: off u64 | len u32 | seed u32 | stats u64[6] x groups
  const size_t d_len = a16(8 * N), d_seed = d_len + a16(4 * N);
  const size_t d_st = d_seed + (seeded ? a16(4 * N) : 0), d_end = d_st + 48 * (size_t)groups;
  int rc = ctx_reserve(c, h_end, N, d_end);
  if (rc) return rc;
  rc = ctx_side(c);
  if (rc) return rc;
  while ((int)c.gev.size() < groups) {
    hipEvent_t e;
    rc = record_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (rc) return rc;
    c.gev.push_back(e);
  }
  uint8_t* h = c.h_buf;
  uint64_t* heads = reinterpret_cast<uint64_t*>(h);
  int32_t* jl = reinterpret_cast<int32_t*>(h + h_len);
  int32_t* js = reinterpret_cast<int32_t*>(h + h_skip);
  uint32_t* jd = reinterpret_cast<uint32_t*>(h + h_seed);
  for (int i = 0; i < n; i++) {  // the calling thread: 20 B per packet, in order
    const Job J = job(i);
    heads[i] = reinterpret_cast<uint64_t>(J.m);
    jl[i] = J.len;
    js[i] = J.skip;
    if (seeded) jd[i] = J.seed;
  }
  size_t nreg = 0;
  uint64_t lo_addr = 0;
  (void)walk_regions(reinterpret_cast<WalkRegionHost*>(h + h_reg), nreg_all, &nreg, &lo_addr);
  const WalkRegionHost* RH = reinterpret_cast<const WalkRegionHost*>(h + h_reg);
  uint64_t* init = reinterpret_cast<uint64_t*>(h + h_init);
  init[0] = ~0ull;
  init[1] = init[2] = init[3] = 0;
  init[4] = ~0ull;
  init[5] = 0;
  void* dh = nullptr;
  rc = record_hip(hipHostGetDevicePointer(&dh, c.h_buf, 0));
  if (rc) return rc;
  void* dout = nullptr;
  rc = record_hip(hipHostGetDevicePointer(&dout, c.h_out, 0));
  if (rc) return rc;
  const uint8_t* dj = static_cast<const uint8_t*>(dh);
  uint8_t* d = c.d_buf;
  uint64_t* doff = reinterpret_cast<uint64_t*>(d);
  uint32_t* dlen = reinterpret_cast<uint32_t*>(d + d_len);
  uint32_t* dsd = seeded ? reinterpret_cast<uint32_t*>(d + d_seed) : nullptr;
  unsigned long long* dst_st = reinterpret_cast<unsigned long long*>(d + d_st);
  volatile uint64_t* hst = reinterpret_cast<volatile uint64_t*>(h + h_st);
  // the walks, all of them, on the side stream (after what c.stream holds)
  rc = record_hip(hipEventRecord(c.gev[0], c.stream));
  if (!rc) rc = record_hip(hipStreamWaitEvent(c.side, c.gev[0], 0));
  for (int g = 0; g < groups && !rc; g++) {
    const int i0 = g * G, ng = std::min(G, n - i0);
    rc = record_hip(hipMemcpyAsync(dst_st + 6 * g, init, 48, hipMemcpyHostToDevice, c.side));
    if (!rc)
      rc = launch_span_walk(reinterpret_cast<const uint64_t*>(dj) + i0,
                            reinterpret_cast<const int32_t*>(dj + h_len) + i0,
                            reinterpret_cast<const int32_t*>(dj + h_skip) + i0,
                            seeded ? reinterpret_cast<const uint32_t*>(dj + h_seed) + i0 : nullptr,
                            reinterpret_cast<const WalkRegionHost*>(dj + h_reg), (int)nreg,
                            (uint32_t)ng, kind == kWalkPseudo, doff + i0, dlen + i0,
                            dsd ? dsd + i0 : nullptr, dst_st + 6 * g, c.side);
    if (!rc)
      rc = record_hip(hipMemcpyAsync(const_cast<uint64_t*>(hst) + 6 * g, dst_st + 6 * g, 48,
                                     hipMemcpyDeviceToHost, c.side));
    if (!rc) rc = record_hip(hipEventRecord(c.gev[g], c.side));
  }
  const auto drain = [&]() {
    (void)hipStreamSynchronize(c.side);
    (void)ctx_wait(c);
  };
  if (rc) {
    drain();
    return rc;
  }
  uint64_t dma_bytes = 0, link_bytes = 0;
  clk::time_point t_first;
  double wait_us = 0;
  for (int g = 0; g < groups; g++) {
    const int i0 = g * G, ng = std::min(G, n - i0);
    // this group's walk: sleep-poll its event (a walk takes a few hundred us)
    const clk::time_point tw = clk::now();
    for (;;) {
      const hipError_t e = hipEventQuery(c.gev[g]);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) {
        drain();
        return record_hip(e);
      }
      const long us = (long)std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - tw)
                          .count();
      const long nap = std::min(500l, std::max(20l, us / 8));
      const timespec ts{0, nap * 1000};
      nanosleep(&ts, nullptr);
    }
    if (trace) wait_us += std::chrono::duration<double, std::micro>(clk::now() - tw).count();
    const uint64_t lo = hst[6 * g], hi = hst[6 * g + 1], gb = hst[6 * g + 2];
    const uint64_t bad = hst[6 * g + 3], rmin = hst[6 * g + 4], rmax = hst[6 * g + 5];
    if (bad) {  // not the shape (or outside the regions): the other paths
      drain();
      return kFallback;
    }
    // the group's origin: its lowest span's 256-B line within its region
    // when one region holds it, else the lowest registered byte
    uint64_t gbase = lo_addr;
    const bool one = gb && rmin == rmax && rmin < nreg;
    if (one) {
      const uint64_t r_lo = RH[rmin].base + (uint64_t)RH[rmin].delta;
      gbase = std::max(lo & ~uint64_t(255), r_lo);
    }
    rc = record_hip(hipStreamWaitEvent(c.stream, c.gev[g], 0));
    uint64_t kbase = gbase;
    uint32_t fl = flags | kFlagHostBytes;
    if (!rc && one && gb >= kSpanDmaMin && hi - gbase <= gb + gb / 16 + 4096) {
      const uint64_t range = hi - gbase;
      const size_t want = (size_t)range + 1024;
      if (want > c.stage_cap) {  // grown between groups: drain what may read it
        rc = ctx_wait(c);
        if (!rc) {
          if (c.d_stage) (void)hipFree(c.d_stage);
          c.d_stage = nullptr;
          c.stage_cap = 0;
          const size_t cap = std::max<size_t>(want, size_t(64) << 20);
          rc = record_hip(hipMalloc((void**)&c.d_stage, cap));
          if (!rc) c.stage_cap = cap;
        }
      }
      if (!rc) {
        uint8_t* dstp = c.d_stage + 256 + (gbase & 255);
        rc = record_hip(hipMemcpyAsync(dstp, reinterpret_cast<const void*>(gbase - (uint64_t)RH[rmin].delta),
                                       (size_t)range, hipMemcpyHostToDevice, c.stream));
        kbase = reinterpret_cast<uint64_t>(dstp);
        fl = flags;
        dma_bytes += range;
        link_bytes += range - gb;
      }
    }
    if (!rc) rc = launch_span_rebase(doff + i0, dlen + i0, (uint32_t)ng, gbase, c.stream);
    if (!rc)
      rc = launch_spans(reinterpret_cast<const void*>(kbase), doff + i0, dlen + i0,
                        dsd ? dsd + i0 : nullptr, nullptr, static_cast<uint16_t*>(dout) + i0,
                        (uint32_t)ng, fl, ng ? (uint32_t)(gb / (uint64_t)ng) : 0u, c.stream);
    if (rc) {
      drain();
      return rc;
    }
    link_bytes += gb;
    if (g == 0) t_first = clk::now();
  }
  long min_us = 0;
  if (link_bytes) {
    const long since =
        (long)std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - t_first).count();
    min_us = std::max(0l, (long)(link_bytes / 64000u) - since);
  }
  const clk::time_point t_w = trace ? clk::now() : clk::time_point();
  rc = ctx_wait(c, min_us);
  if (rc) {
    (void)hipStreamSynchronize(c.side);
    return rc;
  }
  deliver(c, n, out16, out32);
  note_span_fast(dma_bytes);
  note_device_walk();
  if (trace)
    fprintf(stderr,
            "uinet_cksum spans (GPU-read heads): n=%d groups=%d dma %.1f MB | group waits %.0f "
            "us, final wait %.0f us (slept %ld), total %.0f us\n",
            n, groups, dma_bytes / 1e6, wait_us,
            std::chrono::duration<double, std::micro>(clk::now() - t_w).count(), min_us,
            std::chrono::duration<double, std::micro>(clk::now() - t_in).count());
  return UINET_CKSUM_OK;
}

struct ChainRef {
  const MbufHdr* m;  // first mbuf, nullptr = nothing to chase
  long limit;        // bytes from the chain start the walk consumes
};

// Walk prefetch.  The walk is bound by misses on mbuf headers
// (m_next/m_data/m_len share the first line), each dependent on the previous
// one, so walking one chain after another keeps about one miss in flight per
// thread.  prefetch_ahead requests headers a few packets ahead (the knob that
// turned it off went in round 6, profiles/r06/pruned/).  A lockstep chase of
// 16 chains (equal on config 3, 3-12 % slower on the offload hooks,
// profiles/r01/ab/walk_pf/) was removed in round 4 (profiles/r04/pruned/).
// Plain software prefetch ahead: packet i+16's head, i+8's second mbuf,
// i+4's third (each read from a line an earlier step requested).
inline void prefetch_ahead(const ChainRef& r, int depth) {
  const MbufHdr* h = r.limit > 0 ? r.m : nullptr;
  long rem = r.limit;
  for (int d = 0; h && d < depth; d++) {
    rem -= h->m_len;
    h = rem > 0 ? h->m_next : nullptr;
  }
  if (h) __builtin_prefetch(h, 0, 3);
}

// Walk every packet (`walk(i, pw)` fills pw and returns the packet's seed;
// `head(i)` is the ChainRef the walk will follow, {nullptr, 0} for none),
// then fold the pieces in place (all registered, even start parity; pipelined
// with the walk) or pack them into pinned staging.
// `job(i)` is packet i in the in_cksum_skip form (head, len, skip, seed) for
// the device walk; `kind` kWalkNone keeps the batch on the host walk.
// Batches of at most `stage_below` jobs are staged even over registered memory;
// `hooks` (run_jobs_made) keeps the walk's plain prefetch.
template <typename WalkFn, typename HeadFn, typename JobFn>
int run_host_batch(int n, uint32_t flags, uint16_t* out16, unsigned* out32, WalkFn walk,
                   HeadFn head, WalkKind kind, bool seeded, JobFn job,
                   int stage_below = kStageBelowJobs, bool hooks = false) {
  if (n < 0) return UINET_CKSUM_EINVAL;
  if (n == 0) return UINET_CKSUM_OK;
  Ctx* cp = nullptr;
  int rc = ctx_current(&cp);
  if (rc) return rc;
  Ctx& c = *cp;

  const int threads = tuning().host_threads;
  // ~16 chunks per thread: the staging path packs and ships them in groups
  // of `threads`, so packing group g+1 overlaps the copy of group g
  int cs = (n + threads * 16 - 1) / (threads * 16);
  if (cs < kChunkMin) cs = kChunkMin;
  cs = (cs + 1) & ~1;  // even: no chunk splits a job pair 2k, 2k + 1 (run_jobs_made)
  const int nch = (n + cs - 1) / cs;
  Batch& B = t_batch;
  if ((int)B.chunks.size() < nch) B.chunks.resize((size_t)nch);
  B.pk_first.resize((size_t)n + 1);
  B.seed.resize((size_t)n);
  B.bytes.resize((size_t)n);
  B.par.resize((size_t)n);
  HostPool& pool = host_pool();

  // UINET_CKSUM_TRACE_HOST=1: per-batch phase times on stderr (tools only)
  static const bool trace = getenv("UINET_CKSUM_TRACE_HOST") != nullptr;
  using clk = std::chrono::steady_clock;
  const clk::time_point t_start = trace ? clk::now() : clk::time_point();
  clk::time_point t_walk, t_place, t_fill, t_launch;

  // Walk chunk j: every packet as the reference walks it, into the chunk's
  // piece list (pk_first chunk-local).
  // The walk's prefetch (chain batches walked by one thread): one cursor per
  // upcoming packet, advanced one mbuf every kCurG packets from the line it
  // requested then, so that mbufs several deep are in cache when the walk
  // reaches them without a chained step stalling on a late line.  Config 3,
  // one thread: 140-156 -> 114-122 us of host CPU per 1,000 packets (zero
  // copy), 191-197 -> 157-165 (staged); with 16 threads, and for the hooks
  // (whose head() parses the frame), no gain or a loss, so they keep the
  // three plain steps (profiles/r06/r06cursor/, r06walkab*/).
  const bool cursor = !hooks && threads == 1;
  auto walk_chunk = [&](int j) {
    Chunk& C = B.chunks[(size_t)j];
    C.i0 = j * cs;
    C.i1 = std::min(n, C.i0 + cs);
    C.pieces.clear();
    C.w.out = &C.pieces;
    C.total = C.packed = 0;
    C.odd = C.too_big = C.unmapped = false;
    C.w.long_piece = false;
    // cursor prefetch: mbuf k of packet p is requested at iteration
    // p - kCurD + k * kCurG, from the line requested kCurG iterations before
    constexpr int kCurD = 48, kCurG = 8, kCurL = kCurD / kCurG;
    struct Cur {
      const MbufHdr* m;
      long rem;
    };
    Cur ring[64];
    if (cursor)
      for (int p = C.i0; p < std::min(C.i1, C.i0 + kCurD); p++) {
        const ChainRef r = head(p);
        ring[p & 63] = {r.limit > 0 ? r.m : nullptr, r.limit};
        if (ring[p & 63].m) __builtin_prefetch(ring[p & 63].m, 0, 3);
      }
    for (int i = C.i0; i < C.i1; i++) {
      if (cursor) {
        if (i + kCurD < C.i1) {
          const ChainRef r = head(i + kCurD);
          Cur& q = ring[(i + kCurD) & 63];
          q = {r.limit > 0 ? r.m : nullptr, r.limit};
          if (q.m) __builtin_prefetch(q.m, 0, 3);
        }
        for (int k = 1; k < kCurL; k++) {
          const int p = i + kCurD - k * kCurG;
          if (p >= C.i1 || p < C.i0) continue;
          Cur& q = ring[p & 63];
          if (!q.m) continue;
          q.rem -= q.m->m_len;
          q.m = q.rem > 0 ? q.m->m_next : nullptr;
          if (q.m) __builtin_prefetch(q.m, 0, 3);
        }
      } else {  // headers a few packets ahead
        if (i + 16 < C.i1) prefetch_ahead(head(i + 16), 0);
        if (i + 8 < C.i1) prefetch_ahead(head(i + 8), 1);
        if (i + 4 < C.i1) prefetch_ahead(head(i + 4), 2);
      }
      B.pk_first[(size_t)i] = (uint32_t)C.pieces.size();
      B.seed[(size_t)i] = walk(i, C.w);
      const uint64_t nb = C.w.bytes;
      C.too_big |= nb > 0xffffffffull;
      B.bytes[(size_t)i] = (uint32_t)nb;
      B.par[(size_t)i] = (uint8_t)(C.w.first_clen & 1);
      C.odd |= B.par[(size_t)i] != 0;
      C.total += nb;
      C.packed += (nb + 15) & ~uint64_t(15);
    }
    C.long_piece = C.w.long_piece;
  };

  // (Z) Registered memory: zero-copy, pipelined.  Groups of `threads` chunks
  // are walked, described (6-B or 12-B chain descriptors in pinned memory, packet
  // bytes read in place over PCIe) and launched one after another, so the
  // host walks group g+1 while the GPU folds group g.  A group whose pieces
  // are not all registered (or that starts at an odd logical parity: the
  // chain kernel counts parity from each packet's first byte) sends the
  // whole batch down the staging path below.
  // Small batches skip both: staging them (one launch out of mapped pinned
  // memory below 64 KiB) answers sooner than the zero-copy launch reading
  // over PCIe or the device walk's four launches and round trips
  // (profiles/r05/r05k/: 1 packet 23 us staged, 46 zero-copy, 34 device walk;
  // 64 packets 36 / 58 / 42; from 256 packets the device walk leads).
  if (n > stage_below) {
    std::shared_lock<std::shared_mutex> g(g_reg_mu);
    // Single-mbuf sums as spans first (no mbuf line crosses the link: config
    // 2 at 0.87 of it for ~3 us of host CPU per 1,000 packets), then the
    // device walk when the mbufs are registered too, then the host walk
    // (profiles/r06/NOTES.md)
    if (!g_regions.empty() && kind != kWalkNone && tuning().span_fast) {
      // span_fast 2: the GPU reads the head mbufs when they are registered
      // (1.4 us of host CPU per 1,000 packets instead of ~3.4, but 0.81 of the
      // link instead of 0.91: each head crosses it as a 128-B line,
      // profiles/r06/r06q/)
      if (tuning().span_fast == 2) {
        rc = span_walk_batch(c, n, flags, kind, seeded, head, job, out16, out32);
        if (rc != kFallback) return rc;
      }
      rc = span_fast_batch(c, n, flags, kind, seeded, head, job, out16, out32);
      if (rc != kFallback) return rc;
    }
    if (!g_regions.empty() && kind != kWalkNone && tuning().walk_device) {
      rc = device_walk_batch(c, pool, threads, cs, n, flags, kind, seeded, head, job, out16,
                             out32, trace);
      if (rc != kFallback) return rc;
    }
    if (!g_regions.empty()) {
      rc = zero_copy_batch(c, B, pool, threads, nch, n, flags, walk_chunk, trace);
      if (rc != kFallback) {
        if (rc) return rc;
        deliver(c, n, out16, out32);
        return UINET_CKSUM_OK;
      }
    }
  }

  // (1) walk
  pool.run(nch, threads, walk_chunk);

  if (trace) t_walk = clk::now();
  // (2) place the chunks
  uint64_t total = 0, packed = 0, np64 = 0;
  for (int j = 0; j < nch; j++) {
    Chunk& C = B.chunks[(size_t)j];
    if (C.too_big) return UINET_CKSUM_EINVAL;
    C.first_piece = (uint32_t)np64;
    C.pack_base = packed;
    np64 += C.pieces.size();
    total += C.total;
    packed += C.packed;
  }
  if (np64 > 0xffffffffull) return UINET_CKSUM_EINVAL;
  const size_t np = (size_t)np64;
  const uint32_t mean = (uint32_t)(total / (uint64_t)n);

  if (trace) t_place = clk::now();
  if (trace) t_fill = clk::now();
  {
    // (3) staging
    const Layout L = layout_for((size_t)n);
    rc = ctx_reserve(c, L.data_o + packed + 16, (size_t)n);
    if (rc) return rc;
    uint64_t* off = reinterpret_cast<uint64_t*>(c.h_buf + L.off_o);
    uint32_t* len = reinterpret_cast<uint32_t*>(c.h_buf + L.len_o);
    uint32_t* seed = reinterpret_cast<uint32_t*>(c.h_buf + L.seed_o);
    uint8_t* par = c.h_buf + L.par_o;
    uint8_t* data = c.h_buf + L.data_o;
    const bool mapped = L.data_o + packed <= kMappedStagingMax;
    // A large batch is packed in groups of chunks, each group's bytes
    // shipped to HBM (async DMA) while the pool packs the next group.
    const bool stream_copy = !mapped && packed >= kStreamCopyMin;
    const int group = stream_copy ? std::max(1, threads) : nch;
    for (int g0 = 0; g0 < nch; g0 += group) {
      const int g1 = std::min(nch, g0 + group);
      pool.run(g1 - g0, threads, [&](int jj) {
        const Chunk& C = B.chunks[(size_t)(g0 + jj)];
        uint64_t cur = C.pack_base;
        uint32_t k = 0;
        for (int i = C.i0; i < C.i1; i++) {
          off[i] = cur;
          seed[i] = B.seed[(size_t)i];
          par[i] = B.par[(size_t)i];
          len[i] = B.bytes[(size_t)i];
          const uint32_t k1 =
              i + 1 < C.i1 ? B.pk_first[(size_t)i + 1] : (uint32_t)C.pieces.size();
          uint8_t* dst = data + cur;
          for (; k < k1; k++) {
            memcpy(dst, C.pieces[k].p, C.pieces[k].n);
            dst += C.pieces[k].n;
          }
          cur += ((uint64_t)B.bytes[(size_t)i] + 15) & ~uint64_t(15);
        }
      });
      if (stream_copy) {
        const uint64_t b0 = B.chunks[(size_t)g0].pack_base;
        const uint64_t b1 = g1 < nch ? B.chunks[(size_t)g1].pack_base : packed;
        rc = record_hip(hipMemcpyAsync(c.d_buf + L.data_o + b0, data + b0, b1 - b0,
                                       hipMemcpyHostToDevice, c.stream));
        if (rc) return rc;
      }
    }
    // A small batch (the per-call ABI is a batch of one) is folded straight
    // out of the mapped staging and its results written straight back: one
    // launch instead of copy + launch + copy, the two copies being most of
    // its latency.  Large batches copy to HBM first (PCIe reads by the
    // kernel are slower than one bulk DMA).
    uint8_t* src = c.d_buf;
    uint16_t* dout = c.d_out;
    if (mapped) {
      void* dd = nullptr;
      void* dst = nullptr;
      rc = record_hip(hipHostGetDevicePointer(&dd, c.h_buf, 0));
      if (rc) return rc;
      rc = record_hip(hipHostGetDevicePointer(&dst, c.h_out, 0));
      if (rc) return rc;
      src = static_cast<uint8_t*>(dd);
      dout = static_cast<uint16_t*>(dst);
    } else {
      rc = record_hip(hipMemcpyAsync(c.d_buf, c.h_buf, stream_copy ? L.data_o : L.data_o + packed,
                                     hipMemcpyHostToDevice, c.stream));
      if (rc) return rc;
    }
    rc = launch_spans(src + L.data_o, reinterpret_cast<const uint64_t*>(src + L.off_o),
                      reinterpret_cast<const uint32_t*>(src + L.len_o),
                      reinterpret_cast<const uint32_t*>(src + L.seed_o), src + L.par_o, dout,
                      (uint32_t)n, flags, mean ? mean : 1, c.stream);
    if (rc) return rc;
    if (!mapped) {
      rc = record_hip(hipMemcpyAsync(c.h_out, c.d_out, (size_t)n * 2, hipMemcpyDeviceToHost,
                                     c.stream));
      if (rc) return rc;
    }
  }
  if (trace) t_launch = clk::now();
  rc = ctx_wait(c);
  if (rc) return rc;
  if (trace) {
    const auto ms = [](clk::time_point a, clk::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const clk::time_point t_end = clk::now();
    fprintf(stderr,
            "uinet_cksum host batch: n=%d pieces=%zu bytes=%llu staged threads=%d | walk %.3f "
            "place %.3f descriptors %.3f pack+launch %.3f wait %.3f ms\n",
            n, np, (unsigned long long)total, threads,
            ms(t_start, t_walk), ms(t_walk, t_place), ms(t_place, t_fill), ms(t_fill, t_launch),
            ms(t_launch, t_end));
  }
  deliver(c, n, out16, out32);
  return UINET_CKSUM_OK;
}

}  // namespace

int run_jobs(const Job* jobs, int n, uint16_t* out) {
  if (n > 0 && (!jobs || !out)) return UINET_CKSUM_EINVAL;
  return run_host_batch(n, 0, out, nullptr, [&](int i, PacketWalk& w) -> uint32_t {
    w.walk_skip(jobs[i].m, jobs[i].len, jobs[i].skip);
    return jobs[i].seed;
  }, [=](int i) { return ChainRef{jobs[i].m, (long)jobs[i].len}; }, kWalkSkip, true,
     [=](int i) { return jobs[i]; });
}

int run_jobs_made(int n, JobMaker make, JobFirst first, void* ctx, uint16_t* out) {
  if (n > 0 && (!make || !first || !out)) return UINET_CKSUM_EINVAL;
  // the hooks: 2 jobs per frame; a batch that did not go to the device
  // (run_hook_device) below kHookDeviceMin frames is staged
  return run_host_batch(n, 0, out, nullptr, [&](int i, PacketWalk& w) -> uint32_t {
    const Job j = make(ctx, i);
    w.walk_skip(j.m, j.len, j.skip);
    return j.seed;
  }, [&](int i) { return ChainRef{first(ctx, i), 0x7fffffffL}; },  // chased like a whole chain
     kWalkSkip, true, [&](int i) { return make(ctx, i); }, 2 * kHookDeviceMin - 1, true);
}

int run_hook_device(bool rx, struct mbuf* const* mv, int n, int l2len, uint8_t* status) {
  // Below kHookDeviceMin frames the host hook answers sooner (its batch is
  // staged; profiles/r05/r05k/, RX: 256 frames 45 us on the host against 100
  // on the device, 1,024: 101 against 124, 4,096: 372 against 215)
  if (n < kHookDeviceMin || !tuning().walk_device) return kFallback;
  std::shared_lock<std::shared_mutex> g(g_reg_mu);
  const size_t nreg_all = g_regions.size();
  if (nreg_all == 0 || nreg_all > (size_t)kWalkRegionsMax) return kFallback;
  if (!heads_registered(n, [&](int i) { return mv[i]; })) return kFallback;
  Ctx* cp = nullptr;
  int rc = ctx_current(&cp);
  if (rc) return rc;
  Ctx& c = *cp;
  static const bool trace = getenv("UINET_CKSUM_TRACE_HOST") != nullptr;
  using clk = std::chrono::steady_clock;
  const clk::time_point t0 = trace ? clk::now() : clk::time_point();
  const auto a16 = [](size_t b) { return (b + 15) & ~size_t(15); };
  const size_t N = (size_t)n, J = 2 * N;  // frames, jobs
  // pinned: mbuf pointers u64[n] | regions | status u32[4] | verdicts u8[n]
  const size_t h_reg = a16(8 * N), h_st = h_reg + a16(sizeof(WalkRegionHost) * nreg_all);
  const size_t h_v = h_st + 16, h_end = h_v + a16(N);
  // HBM: status | jobs (m u64, len i32, skip i32, seed u32) x 2n | plans | frames |
  //      results u16[2n] | the walk's work area
  const size_t d_jm = 16, d_jl = d_jm + a16(8 * J), d_js = d_jl + a16(4 * J);
  const size_t d_jd = d_js + a16(4 * J), d_pl = d_jd + a16(4 * J);
  const size_t d_fr = d_pl + a16(hook_plan_bytes(rx) * N), d_res = d_fr + a16(hook_frame_bytes() * N);
  const size_t d_wa = d_res + a16(2 * J);
  // the hooks fold in the walking launch by default: their chains are one to
  // three mbufs, and one launch fewer is worth more (profiles/r06/)
  const bool fused = tuning().walk_device != 2;
  uint32_t K = fused ? 0u : c.walk_k ? c.walk_k : 4;
  if ((uint64_t)J * K > 0xffffffffull) return kFallback;  // rows indexed by u32
  rc = ctx_reserve(c, h_end, N, d_wa + (fused ? 0 : walk_work(J, K).end));
  if (rc) return rc;
  uint8_t* h = c.h_buf;
  memcpy(h, mv, 8 * N);
  size_t nreg = 0;
  uint64_t lo = 0;
  (void)walk_regions(reinterpret_cast<WalkRegionHost*>(h + h_reg), nreg_all, &nreg, &lo);
  void* dhv = nullptr;
  rc = record_hip(hipHostGetDevicePointer(&dhv, c.h_buf, 0));
  if (rc) return rc;
  const uint8_t* dh = static_cast<const uint8_t*>(dhv);
  const WalkRegionHost* dregs = reinterpret_cast<const WalkRegionHost*>(dh + h_reg);
  volatile uint32_t* st = reinterpret_cast<volatile uint32_t*>(h + h_st);
  bool parsed = false;
  for (int attempt = 0; attempt < (fused ? 1 : 2); attempt++) {
    rc = ctx_reserve(c, h_end, N, d_wa + (fused ? 0 : walk_work(J, K).end));
    if (rc) return rc;
    uint8_t* d = c.d_buf;
    uint32_t* dstatus = reinterpret_cast<uint32_t*>(d);
    uint64_t* jm = reinterpret_cast<uint64_t*>(d + d_jm);
    int32_t* jl = reinterpret_cast<int32_t*>(d + d_jl);
    int32_t* js = reinterpret_cast<int32_t*>(d + d_js);
    uint32_t* jd = reinterpret_cast<uint32_t*>(d + d_jd);
    rc = record_hip(hipMemsetAsync(dstatus, 0, 8, c.stream));
    // the parse runs once; a second attempt (rows too short) walks its jobs again
    // (ctx_reserve keeps the buffer's contents only when it does not grow it)
    if (!rc && !parsed)
      rc = launch_hook_parse(rx, reinterpret_cast<const uint64_t*>(dh), (uint32_t)n, l2len,
                             dregs, (int)nreg, jm, jl, js, jd, d + d_pl, d + d_fr, dstatus,
                             c.stream);
    if (!rc && fused)  // the jobs' chains walked and folded in one launch
      rc = launch_mbufs_xlate(jm, jl, js, jd, dregs, (int)nreg, false,
                              reinterpret_cast<uint16_t*>(d + d_res), (uint32_t)J, 0, dstatus,
                              c.stream);
    else if (!rc)
      rc = launch_walk_fold(c, jm, jl, js, jd, dregs, (int)nreg, lo, J, K, false, d + d_wa,
                            dstatus, reinterpret_cast<uint16_t*>(d + d_res), 0);
    if (!rc)
      rc = launch_hook_apply(rx, d + d_pl, d + d_fr, reinterpret_cast<uint16_t*>(d + d_res),
                             (uint32_t)n, K, dstatus, const_cast<uint8_t*>(dh) + h_v, c.stream);
    if (!rc) rc = record_hip(hipMemcpyAsync(h + h_st, dstatus, 8, hipMemcpyDeviceToHost, c.stream));
    const int wrc = ctx_wait(c);
    if (rc) return rc;
    if (wrc) return wrc;
    if (st[0]) return kFallback;  // the device view could not take a frame
    const uint32_t longest = st[1];  // 0 after the fused walk
    const uint32_t k2 = walk_k_for(longest);
    if (!fused) c.walk_k = k2;
    if (longest <= K) {  // the apply step ran
      if (status) memcpy(status, h + h_v, N);
      note_device_walk();
      if (trace)
        fprintf(stderr, "uinet_cksum offload %s: n=%d on the device, K=%u | total %.3f ms\n",
                rx ? "rx" : "tx", n, K,
                std::chrono::duration<double, std::milli>(clk::now() - t0).count());
      return UINET_CKSUM_OK;
    }
    if (k2 > kWalkKMax || (uint64_t)J * k2 > 0xffffffffull) return kFallback;
    // the rows must grow: the device buffer is reallocated, so parse again
    if (walk_work(J, k2).end + d_wa > c.d_cap) parsed = false; else parsed = true;
    K = k2;
  }
  return kFallback;
}

namespace {

// ---- IPv6 pseudo header (sys/netinet6/in6_cksum.c:86-126) -------------------

// The zone index KAME embeds in word 1 of link-local unicast and link- /
// interface-local multicast addresses is left out of the sum
// (in6_cksum.c:110-124, scope6.c:502-509, netinet6/in6.h:294-356).
uint64_t in6_scope_word(const uint8_t* a) {
  const bool ll = a[0] == 0xfe && (a[1] & 0xc0) == 0x80;
  const bool mc = a[0] == 0xff && ((a[1] & 0x0f) == 0x02 || (a[1] & 0x0f) == 0x01);
  return (ll || mc) ? (uint64_t)(a[2] | a[3] << 8) : 0;
}

// htonl(len), three zero bytes, nxt, then the source and destination
// addresses, all as little-endian 16-bit words; folded.
uint32_t in6_pseudo_fold(const uint8_t* ip6, uint32_t len, uint8_t nxt) {
  uint64_t s = ((len >> 24) & 0xff) | ((len >> 16) & 0xff) << 8;
  s += ((len >> 8) & 0xff) | (len & 0xff) << 8;
  s += (uint64_t)nxt << 8;
  for (int i = 0; i < 32; i += 2) s += (uint64_t)(ip6[8 + i] | ip6[8 + i + 1] << 8);
  return fold16_host(s - in6_scope_word(ip6 + 8) - in6_scope_word(ip6 + 24));
}

}  // namespace
}  // namespace uinet

using namespace uinet;

extern "C" {

const char* uinet_cksum_version(void) { return "libuinet_cksum 0.1 (gfx950)"; }

const char* uinet_cksum_last_kernel(void) {
  thread_local std::string name;
  name.clear();
  if (!t_last_kernel) return "";
  const char* m = hipKernelNameRefByPtr(t_last_kernel, nullptr);
  if (!m) return "";
  int st = 0;
  char* d = abi::__cxa_demangle(m, nullptr, nullptr, &st);
  name = (st == 0 && d) ? d : m;
  free(d);
  return name.c_str();
}

const char* uinet_cksum_strerror(int code) {
  switch (code) {
    case UINET_CKSUM_OK: return "ok";
    case UINET_CKSUM_EINVAL: return "invalid argument";
    case UINET_CKSUM_ENODEV: return "no usable gfx950 device";
    case UINET_CKSUM_ENOMEM: return "out of memory";
    case UINET_CKSUM_EHIP: return "HIP runtime error";
    default: return "unknown error";
  }
}

int uinet_cksum_last_hip_error(void) { return t_last_hip; }

int uinet_cksum_register_host(void* base, size_t len) {
  if (!base || len == 0) return UINET_CKSUM_EINVAL;
  const uintptr_t b = reinterpret_cast<uintptr_t>(base), e = b + len;
  std::unique_lock<std::shared_mutex> g(g_reg_mu);
  for (const Region& r : g_regions)
    if (b < r.end && r.base < e) return UINET_CKSUM_EINVAL;  // overlaps
  bool owned = true;
  hipError_t he = hipHostRegister(base, len, hipHostRegisterMapped | hipHostRegisterPortable);
  if (he == hipErrorHostMemoryAlreadyRegistered) {  // e.g. hipHostMalloc'd / torch-pinned
    (void)hipGetLastError();
    owned = false;
  } else if (he != hipSuccess) {
    return record_hip(he);
  }
  void* dev = nullptr;
  int rc = record_hip(hipHostGetDevicePointer(&dev, base, 0));
  if (rc) {
    if (owned) (void)hipHostUnregister(base);
    return rc;
  }
  Region r{b, e, (intptr_t)(reinterpret_cast<uintptr_t>(dev) - b), owned};
  g_regions.insert(std::upper_bound(g_regions.begin(), g_regions.end(), r,
                                    [](const Region& x, const Region& y) { return x.base < y.base; }),
                   r);
  return UINET_CKSUM_OK;
}

int uinet_cksum_unregister_host(void* base) {
  const uintptr_t b = reinterpret_cast<uintptr_t>(base);
  std::unique_lock<std::shared_mutex> g(g_reg_mu);
  for (size_t i = 0; i < g_regions.size(); i++) {
    if (g_regions[i].base == b) {
      const bool owned = g_regions[i].owned;
      g_regions.erase(g_regions.begin() + (long)i);
      return owned ? record_hip(hipHostUnregister(base)) : UINET_CKSUM_OK;
    }
  }
  return UINET_CKSUM_EINVAL;
}

int uinet_cksum_host_cpu(struct uinet_cksum_host_cpu* st, int reset) {
  if (st) *st = t_cpu;
  if (reset) t_cpu = {};
  return UINET_CKSUM_OK;
}

int uinet_cksum_set_tuning(const char* key, int value) {
  if (!key) return UINET_CKSUM_EINVAL;
  std::atomic<int>* f = tuning_field(tuning_live(), key, value);
  if (!f) return UINET_CKSUM_EINVAL;
  f->store(value, std::memory_order_relaxed);
  return UINET_CKSUM_OK;
}

int uinet_cksum_device_ok(void) {
  int dev = 0, count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

// ---- device-resident API ----------------------------------------------------

int uinet_cksum_spans(const void* base, const uint64_t* off, const uint32_t* len,
                      const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                      uint32_t flags, uint32_t len_hint, void* stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (n > UINET_CKSUM_MAX_PACKETS) return UINET_CKSUM_EINVAL;
  if (!base || !off || !len || !out) return UINET_CKSUM_EINVAL;
  return launch_spans(base, off, len, seed, parity, out, n, flags & ~kFlagHostBytes, len_hint,
                      static_cast<hipStream_t>(stream));
}

int uinet_cksum_spans32(const void* base, const uint32_t* off, const uint16_t* len,
                        const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                        uint32_t flags, uint32_t len_hint, void* stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (n > UINET_CKSUM_MAX_PACKETS) return UINET_CKSUM_EINVAL;
  if (!base || !off || !len || !out) return UINET_CKSUM_EINVAL;
  return launch_spans32(base, off, len, seed, parity, out, n, flags & ~kFlagHostBytes, len_hint,
                        static_cast<hipStream_t>(stream));
}

int uinet_cksum_strided(const void* base, uint64_t stride, uint32_t len, const uint32_t* seed,
                        uint16_t* out, uint32_t n, uint32_t flags, void* stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (n > UINET_CKSUM_MAX_PACKETS || len >= UINET_CKSUM_MAX_SPAN) return UINET_CKSUM_EINVAL;
  if (!base || !out) return UINET_CKSUM_EINVAL;
  return launch_strided(base, stride, len, seed, out, n, flags,
                        static_cast<hipStream_t>(stream));
}

int uinet_cksum_chains(const void* base, const uint64_t* seg_off, const uint32_t* seg_len,
                       const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                       const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                       uint32_t len_hint, void* stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (n > UINET_CKSUM_MAX_PACKETS) return UINET_CKSUM_EINVAL;
  if (!base || !seg_off || !seg_len || !pkt_seg || !out) return UINET_CKSUM_EINVAL;
  return launch_chains(base, seg_off, seg_len, pkt_seg, len, skip, seed, out, n, flags,
                       len_hint, static_cast<hipStream_t>(stream));
}

int uinet_cksum_chains32(const void* base, const uint32_t* seg_off, const uint16_t* seg_len,
                         const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                         const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                         uint32_t len_hint, void* stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (n > UINET_CKSUM_MAX_PACKETS) return UINET_CKSUM_EINVAL;
  if (!base || !seg_off || !seg_len || !pkt_seg || !out) return UINET_CKSUM_EINVAL;
  return launch_chains32(base, seg_off, seg_len, pkt_seg, len, skip, seed, out, n, flags,
                         len_hint, static_cast<hipStream_t>(stream));
}

int uinet_cksum_mbufs(const struct mbuf* const* heads, const int32_t* len, const int32_t* skip,
                      const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                      uint32_t seg_hint, uint32_t* status, void* stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (n > UINET_CKSUM_MAX_PACKETS) return UINET_CKSUM_EINVAL;
  if (!heads || !out) return UINET_CKSUM_EINVAL;
  return launch_mbufs(reinterpret_cast<const uint64_t*>(heads), len, skip, seed, out, n, flags,
                      seg_hint, status, static_cast<hipStream_t>(stream));
}

// ---- host-mbuf batch API ------------------------------------------------------

int in_cksum_skip_batch(struct mbuf* const* m, const int* len, const int* skip,
                        unsigned short* out, int n) {
  if (n > 0 && (!m || !len || !skip || !out)) return UINET_CKSUM_EINVAL;
  CpuScope cpu(n);
  return run_host_batch(n, 0, out, nullptr, [&](int i, PacketWalk& w) -> uint32_t {
    w.walk_skip(reinterpret_cast<const MbufHdr*>(m[i]), len[i], skip[i]);
    return 0u;
  }, [=](int i) { return ChainRef{reinterpret_cast<const MbufHdr*>(m[i]), (long)len[i]}; },
     kWalkSkip, false,
     [=](int i) { return Job{reinterpret_cast<const MbufHdr*>(m[i]), len[i], skip[i], 0u}; });
}

int in_cksum_pseudo_header_batch(struct mbuf* const* m, const int* plen, const int* off0,
                                 const uint32_t* src, const uint32_t* dst,
                                 const uint8_t* protonum, uint16_t* out, int n) {
  if (n > 0 && (!m || !plen || !off0 || !src || !dst || !protonum || !out))
    return UINET_CKSUM_EINVAL;
  CpuScope cpu(n);
  return run_host_batch(n, 0, out, nullptr, [&](int i, PacketWalk& w) -> uint32_t {
    w.walk_pseudo(reinterpret_cast<const MbufHdr*>(m[i]), plen[i], off0[i]);
    // in_cksum.c:252-253; folded on the host so it fits the u32 seed slot
    // (folding keeps both the value mod 65535 and "is zero").
    const uint64_t s = (uint64_t)src[i] + dst[i] + bswap16(protonum[i]) +
                       bswap16((uint16_t)plen[i]);
    return fold16_host(s);
  }, [=](int i) {
    return ChainRef{reinterpret_cast<const MbufHdr*>(m[i]), (long)off0[i] + plen[i]};
  }, kWalkPseudo, true, [=](int i) {
    // in_cksum_skip(m, off0 + plen, off0) when off0 lies in the first mbuf
    // (the walk checks that); an off0 + plen past INT_MAX takes the host walk
    // (a negative skip is the walk's "host" mark)
    const long e = (long)off0[i] + plen[i];
    const uint64_t s = (uint64_t)src[i] + dst[i] + bswap16(protonum[i]) +
                       bswap16((uint16_t)plen[i]);
    return Job{reinterpret_cast<const MbufHdr*>(m[i]), e > 0x7fffffffL ? 0 : (int)e,
               e > 0x7fffffffL ? -1 : off0[i], fold16_host(s)};
  });
}

int in6_cksum_batch(struct mbuf* const* m, const uint8_t* nxt, const uint32_t* off,
                    const uint32_t* len, uint16_t* out, int n) {
  if (n > 0 && (!m || !nxt || !off || !len || !out)) return UINET_CKSUM_EINVAL;
  for (int i = 0; i < n; i++)  // the header is read on the host; off + len fits an int
    if (!m[i] || (uint64_t)off[i] + len[i] > 0x7fffffffull) return UINET_CKSUM_EINVAL;
  CpuScope cpu(n);
  return run_host_batch(n, 0, out, nullptr, [&](int i, PacketWalk& w) -> uint32_t {
    // in6_cksum.c:208-350: off counts from the chain start, then len bytes
    const MbufHdr* mm = reinterpret_cast<const MbufHdr*>(m[i]);
    w.walk_skip(mm, (int)(off[i] + len[i]), (int)off[i]);
    return in6_pseudo_fold(mm->m_data, len[i], nxt[i]);  // "contiguous IP6 header"
  }, [=](int i) {
    return ChainRef{reinterpret_cast<const MbufHdr*>(m[i]), (long)off[i] + (long)len[i]};
  }, kWalkSkip, true, [=](int i) {
    const MbufHdr* mm = reinterpret_cast<const MbufHdr*>(m[i]);
    return Job{mm, (int)(off[i] + len[i]), (int)off[i], in6_pseudo_fold(mm->m_data, len[i], nxt[i])};
  });
}

int in_cksum_hdr_batch(const struct ip* const* ip, unsigned int* out, int n) {
  if (n > 0 && (!ip || !out)) return UINET_CKSUM_EINVAL;
  CpuScope cpu(n);
  return run_host_batch(n, 0, nullptr, out, [&](int i, PacketWalk& w) -> uint32_t {
    // in_cksum.c:278-285: in_cksumdata(ip, 20) weights by ADDRESS parity and
    // never re-aligns, so the header's logical start parity is its address
    // parity.
    w.reset(20);
    w.clen = (long)(reinterpret_cast<uintptr_t>(ip[i]) & 1);
    w.take(reinterpret_cast<const uint8_t*>(ip[i]), 20);
    return 0u;
  }, [](int) { return ChainRef{nullptr, 0}; }, kWalkNone, false,
     [](int) { return Job{nullptr, 0, 0, 0u}; });
}

// ---- drop-in per-call ABI (sys/amd64/include/in_cksum.h:76-83) --------------
//
// One chain per call, folded on the calling thread (cksum_percall.cpp): a
// synchronous GPU round trip per packet is ~30x slower than the fold, and
// the reference has no error channel, so these never touch the device and
// never fail.  Batches of packets go to the GPU (sections 2b-2d of the header).

unsigned short in_cksum_skip(struct mbuf* m, int len, int skip) {
  return host_cksum_skip(reinterpret_cast<const MbufHdr*>(m), len, skip, 0u);
}

uint16_t in_cksum_pseudo_header(struct mbuf* m, int plen, int off0, uint32_t src, uint32_t dst,
                                uint8_t protonum) {
  return host_cksum_pseudo(reinterpret_cast<const MbufHdr*>(m), plen, off0, src, dst, protonum);
}

unsigned int in_cksum_hdr(const struct ip* ip) { return host_cksum_hdr(ip); }

// sys/netinet6/in6.h:638, in6_cksum.c:150-357 (off counts from the chain
// start, m_data at a contiguous IPv6 header).
int in6_cksum(struct mbuf* m, uint8_t nxt, uint32_t off, uint32_t len) {
  const MbufHdr* mm = reinterpret_cast<const MbufHdr*>(m);
  return host_cksum_skip(mm, (long)off + (long)len, (long)off,
                         in6_pseudo_fold(mm->m_data, len, nxt));
}

// in6.h:637, in6_cksum.c:129-140: 36 header bytes, no payload -- a host fold.
int in6_cksum_pseudo(struct ip6_hdr* ip6, uint32_t len, uint8_t nxt, uint16_t csum) {
  const uint8_t* a = reinterpret_cast<const uint8_t*>(ip6);
  uint64_t s = (uint64_t)in6_pseudo_fold(a, len, nxt) + csum;
  return (int)fold16_host(s);
}

// in_pseudo / in_addword fold three or two register values -- no packet
// bytes, O(1): they stay scalar (in_cksum.c:172-191).
unsigned short in_pseudo(unsigned int a, unsigned int b, unsigned int c) {
  return (unsigned short)fold16_host((uint64_t)a + b + c);
}

unsigned short in_addword(unsigned short a, unsigned short b) {
  return (unsigned short)fold16_host((uint64_t)a + b);
}

}  // extern "C"
