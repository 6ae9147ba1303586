// MI355X (gfx950) mbuf-chain kernel: in_cksum_skip(m, len, skip) over
// struct mbuf chains that lie where the GPU reads them -- in HBM (the
// device-resident uinet_cksum_mbufs) or, through the region table of
// uinet_cksum_register_host, in registered host memory (the host-mbuf batch
// API's device walk).  One kernel walks AND folds: no segment list is
// written or read back.
//
// What it computes is the reference walk
// (/root/reference/sys/amd64/amd64/in_cksum.c:193-232): the chain bytes
// [skip, len) -- len counts from the chain start -- found by following
// m_next / m_data / m_len (struct m_hdr offsets 0 / 16 / 24,
// /root/reference/sys/sys/mbuf.h:90-98); a zero-length mbuf contributes
// nothing, a chain shorter than len sums what it has, and each byte is
// weighted by its logical parity counted from `skip` (the "<< 8" of
// :222-225).  The walk stops where the reference's does: after the mbuf
// that holds byte len - 1, or at m_next == NULL.
//
// Shape.  A wave owns 64 chains at a time, one per lane, and advances all of
// them by one mbuf per round:
//   * each lane has its current mbuf's header (issued the round before),
//     clips the mbuf's bytes to [skip, len) at its chain offset, and -- before
//     anything waits -- issues the NEXT mbuf's header load, so the dependent
//     m_next chase of round r + 1 is in flight while round r's bytes stream;
//   * the round's 64 segments are folded by the whole wave as one dense list
//     of 16-byte chunks (the k_chains_pipe chunk list, cksum_chains.hip:
//     segment lookup by LDS start markers + a DPP max-scan, 17x17 LDS mask
//     table, telescoping DPP prefix sums into LDS bins), binned per
//     (lane, logical parity); the round's segments of 2 KiB or more are
//     streamed by the whole wave, one after another, the next one's loads
//     issued before this one's are summed;
//   * a lane whose chain ends writes its result and takes the next packet of
//     the wave's range at once (its job -- head, len, skip, seed -- was
//     prefetched when it took the previous one), so every lane stays busy
//     until the range runs dry: the rounds a wave runs are the range's mbufs
//     / 64, not the longest chain times the packets per lane.  The range is
//     handed out longest packet first (per window of 64 packets, by len), so
//     the last rounds are short chains.
// Every m_next hop costs one round trip, but 64 chains per wave and every
// wave of the chip in flight keep ~100 K hops outstanding: the walk runs at
// the rate HBM delivers the header lines and packet bytes.
//
// Bounds (the reference trusts its chains; a GPU must still finish): a chain
// is followed for at most kHopsMax mbufs (UINET_CKSUM_MBUF_TRUNC); a negative
// m_len, outside the reference's contract, ends the chain there
// (UINET_CKSUM_MBUF_BADLEN), and so does a negative skip (the whole packet
// then sums nothing, UINET_CKSUM_MBUF_BADARG).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "cksum_device.h"
#include "walk_xlate.h"

namespace uinet {
namespace {

constexpr int kWaves = kBlock / 64;
constexpr uint32_t kNone = 0xffffffffu;
constexpr int kPass = 2;                    // 64-chunk passes per pipelined batch
constexpr int kWin = 64 * kPass;            // chunks per batch
// Segments of 2 KiB and more are streamed by the whole wave, pipelined across
// the round's long segments; shorter ones go through the chunk list.  (A first
// build streamed each long segment on its own, one latency per 4-KiB round:
// 5tso's mbuf form 0.342 ms; all segments up to 16 KiB through the chunk
// list, whose per-chunk lookup then runs over 9-KB payloads: 0.388 ms.)
constexpr uint32_t kLongCh = 128;           // segments of >= 2 KiB stream wave-wide
constexpr int kLongU = 2;                   // chunks per lane per streamed item
constexpr uint32_t kHopsMax = UINET_CKSUM_MBUF_HOPS_MAX;  // mbufs followed per chain, at most
constexpr uint32_t kRing = 128;             // jobs a wave holds in LDS

// A wave's queue of jobs (uinet_cksum_mbufs arguments of one packet each).
struct JobRing {
  uint64_t head[kRing];
  int32_t len[kRing], skip[kRing];
  uint32_t seed[kRing], pkt[kRing];
};
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short us16x2 __attribute__((ext_vector_type(2)));

// 16-B raw buffer load, non-temporal, from a resource spanning 4 GiB (as in
// cksum_chains.hip): one VGPR of offset instead of a 64-bit address per chunk.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mb_window_rsrc(uint64_t sbase) {
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(sbase), 0, (int)0xffffffffu,
                                           0x00020000);
}
// kTemporal: an ordinary (temporal) load, else non-temporal (aux bit 1).
template <bool kTemporal>
__device__ __forceinline__ u32x4 mb_load_chunk_buf(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kTemporal ? 0 : 2);
}

// Loads from an address held as an integer, in the global address space: a
// generic pointer made from an integer compiles to a flat load, which counts
// in lgkmcnt too, so the next LDS wait would also wait for it (the first build
// exposed every header load's latency at the fold's first LDS read that way).
typedef __attribute__((address_space(1))) const uint64_t GlobalU64;
typedef __attribute__((address_space(1))) const int32_t GlobalI32;
typedef __attribute__((address_space(1))) const u32x4 GlobalChunk;
__device__ __forceinline__ uint64_t gload_u64(uint64_t a) {
  return *reinterpret_cast<GlobalU64*>(a);
}
__device__ __forceinline__ int32_t gload_i32(uint64_t a) {
  return *reinterpret_cast<GlobalI32*>(a);
}
template <bool kTemporal = false>
__device__ __forceinline__ u32x4 gload_chunk(uint64_t a) {
  if constexpr (kTemporal) return *reinterpret_cast<GlobalChunk*>(a);
  return __builtin_nontemporal_load(reinterpret_cast<GlobalChunk*>(a));
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

#ifdef UINET_MBUFS_WAVES  // build-time occupancy A/B
#define UINET_MBUFS_OCC __attribute__((amdgpu_waves_per_eu(UINET_MBUFS_WAVES)))
#else
#define UINET_MBUFS_OCC __attribute__((amdgpu_waves_per_eu(5)))
#endif

// kXlate: mbuf and data addresses are host addresses inside the registered
// regions (read through their device aliases; anything outside, or -- with
// `pseudo`, the in_cksum_pseudo_header form -- a first mbuf shorter than
// skip, is reported in status[0] as kWalkUnmapped / kWalkFallback and the
// host redoes the batch).  Without it they are device addresses used as is.
// kTemporal: the packet-byte loads are ordinary (temporal) loads, else
// non-temporal.  Short mbufs (config 3's 1-256-B m_fragment pieces) gain from
// temporal loads -- a chain's next piece, read by the same lane a round later,
// usually starts in the line this one ends in, still in L2: config 3 0.434 ->
// 0.375 ms -- and long ones lose (3tx's page slices +8 %, whether chosen per
// round or per piece inside one kernel; profiles/r06/r06ab_temporal*/).  The
// caller's seg_hint (mean bytes per mbuf) picks the instantiation.
template <bool kXlate, bool kTemporal>
__global__ __launch_bounds__(kBlock) UINET_MBUFS_OCC void k_mbufs(
    const uint64_t* __restrict__ heads, const int32_t* __restrict__ plen,
    const int32_t* __restrict__ pskip, const uint32_t* __restrict__ seed,
    uint16_t* __restrict__ out, uint32_t n, uint32_t per_wave, uint32_t flags,
    const WalkRegionHost* __restrict__ regions, int nreg, int pseudo,
    uint32_t* __restrict__ status) {
  __shared__ MaskLut lut;
  __shared__ unsigned long long lds_acc[kWaves][128];  // (lane, parity) bins
  // segment-start markers per batch, (lane + 1) << 8 | meta, and one spare
  // slot per lane that lanes without a start in the batch write
  __shared__ uint16_t lds_mark[kWaves][kWin + 64];
  __shared__ WalkRegionHost R[kXlate ? kWalkRegionsMax : 1];
  __shared__ JobRing lds_ring[kWaves];
  if constexpr (kXlate)
    for (int k = (int)threadIdx.x; k < nreg; k += (int)blockDim.x) R[k] = regions[k];
  for (int i = threadIdx.x; i < kWaves * 128; i += blockDim.x) (&lds_acc[0][0])[i] = 0;
  for (int i = threadIdx.x; i < kWaves * (kWin + 64); i += blockDim.x) (&lds_mark[0][0])[i] = 0;
  lut.init();  // ends in __syncthreads
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned long long* acc = lds_acc[wid];
  uint16_t* mark = lds_mark[wid];
  s16x2 lane16[kPass];
#pragma unroll
  for (int q = 0; q < kPass; ++q) {
    const short x = (short)(16 * (q * 64 + lane));
    lane16[q] = s16x2{x, x};
  }

  // The wave's packets [wq, qe) reach the lanes through a ring of jobs in LDS
  // (head, len, skip, seed, packet index), refilled at the end of a round
  // with the next 64 packets, longest first (by len[], a counting sort on
  // eight length classes): a lane whose chain ends takes the ring's next job
  // at once, so the short packets of a window run while the long ones finish
  // and the wave's last rounds are short chains, not a 1500-B packet started
  // late.  The jobs live in LDS, not in registers, so the kernel keeps its
  // occupancy.
  const uint64_t w0 = (uint64_t)(blockIdx.x * kWaves + wid) * per_wave;
  uint32_t wq = (uint32_t)min(w0, (uint64_t)n);
  const uint32_t qe = (uint32_t)min(w0 + per_wave, (uint64_t)n);
  const bool has_len = plen != nullptr;
  uint32_t st = 0;  // this lane's status bits
  JobRing& ring = lds_ring[wid];
  uint32_t rhd = 0, rtl = 0;  // ring head (next job to take) and tail (wave-uniform)
  auto fill = [&]() {  // wave-uniform: 64 more jobs when the ring runs below 64
    if (wq >= qe || rtl - rhd > 64u) return;
    const uint32_t cnt = min(64u, qe - wq);
    const uint32_t i = wq + (uint32_t)lane;
    const bool v = (uint32_t)lane < cnt;
    uint64_t h = 0;
    int32_t l = 0, k = 0;
    uint32_t d = 0;
    if (v) {
      h = heads[i];
      l = has_len ? plen[i] : 0x7fffffff;
      k = pskip ? pskip[i] : 0;
      d = seed ? seed[i] : 0u;
    }
    const int32_t lc = l < 128 ? 127 : l;
    const uint32_t b = v ? (uint32_t)min(7, 25 - __builtin_clz((uint32_t)lc)) : 8u;  // 0: < 256 B
    uint32_t pos = 0, cursor = 0;
    for (int c = 7; c >= 0; --c) {
      const uint64_t bm = __ballot(b == (uint32_t)c);
      if (b == (uint32_t)c) pos = cursor + lane_rank(bm);
      cursor += (uint32_t)__builtin_popcountll(bm);
    }
    if (v) {
      const uint32_t slot = (rtl + pos) & (kRing - 1);
      ring.head[slot] = h;
      ring.len[slot] = l;
      ring.skip[slot] = k;
      ring.seed[slot] = d;
      ring.pkt[slot] = i;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    rtl += cnt;
    wq += cnt;
  };
  // the current chain
  uint32_t p = kNone, L = 0, S = 0, sd = 0, pos = 0, hops = 0;
  uint64_t m = 0, hn = 0, hd = 0;
  int32_t hl = 0;
  auto hdr_issue = [&](uint64_t mm) {
    uint64_t a = mm;
    if constexpr (kXlate) {
      uint64_t d;
      if (!walk_xlate(R, nreg, mm, 32, &d)) {
        st |= kWalkUnmapped;
        m = 0;
        return;
      }
      a = d;
    }
    hn = gload_u64(a);        // m_next
    hd = gload_u64(a + 16);   // m_data
    hl = gload_i32(a + 24);   // m_len
  };
  // Every lane with `want` takes the ring's next job (wave-uniform call): its
  // first mbuf's header load goes out at once.
  auto take_job = [&](bool want) {
    const uint64_t tm = __ballot(want);
    if (!tm) return;
    const uint32_t r = lane_rank(tm), avail = rtl - rhd;
    if (want) {
      p = kNone;
      m = 0;
      if (r < avail) {
        const uint32_t slot = (rhd + r) & (kRing - 1);
        p = ring.pkt[slot];
        int32_t l = ring.len[slot], k = ring.skip[slot];
        L = has_len ? (uint32_t)(l < 0 ? 0 : l) : 0xffffffffu;
        if (k < 0) {  // outside the contract (the device walk's host mark)
          st |= kXlate ? kWalkFallback : (uint32_t)UINET_CKSUM_MBUF_BADARG;
          L = 0;
          k = 0;
        }
        S = (uint32_t)k;
        sd = ring.seed[slot];
        pos = 0;
        hops = 0;
        const uint64_t h = ring.head[slot];
        if (L > S && h) {  // nothing to read when nothing is summed
          m = h;
          hdr_issue(m);
        }
      }
    }
    rhd += min((uint32_t)__builtin_popcountll(tm), avail);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  };
  // start: two windows in the ring, every lane takes its first job
  fill();
  fill();
  take_job(true);

  // Chunk-list fold of one round's segments (see cksum_chains.hip,
  // k_chains_pipe, for the addressing and pipelining details).
  u32x4 va[kPass], vb[kPass];
  uint32_t ka[kPass], kb[kPass];
  auto consume = [&](const u32x4 (&v)[kPass], const uint32_t (&key)[kPass]) {
    uint32_t P[kPass], sl[kPass], nx[kPass];
#pragma unroll
    for (int k = 0; k < kPass; ++k) P[k] = lut.sum_oc_idx(v[k], key[k] & 0xffffu);  // < 2^19
#pragma unroll
    for (int k = 0; k < kPass; ++k) {
      sl[k] = key[k] >> 16;
      nx[k] = wave_shl1(sl[k]);
    }
    wave_scan_add_n<kPass>(P);  // < 2^26
#pragma unroll
    for (int k = 0; k < kPass; ++k) {
      if (lane == 63 || nx[k] != sl[k]) {
        atomicAdd(&acc[sl[k]], (unsigned long long)P[k]);
        if (lane != 63) __atomic_fetch_sub(&acc[nx[k]], (unsigned long long)P[k], __ATOMIC_RELAXED);
      }
    }
  };

  for (;;) {
    if (__ballot(p != kNone) == 0) break;
    // --- this round's mbuf, one per lane ---------------------------------
    const bool has = p != kNone && m != 0;
    uint64_t nx = has ? hn : 0ull;
    const uint64_t da = has ? hd : 0ull;
    int32_t mli = has ? hl : 0;
    if (mli < 0) {
      st |= kXlate ? kWalkFallback : (uint32_t)UINET_CKSUM_MBUF_BADLEN;
      mli = 0;
      nx = 0;
    }
    const uint32_t ml = (uint32_t)mli;
    if (kXlate && pseudo && has && hops == 0 && ml < S) st |= kWalkFallback;
    const uint32_t lo = S > pos ? min(S - pos, ml) : 0u;
    const uint32_t hi = L > pos ? min(L - pos, ml) : 0u;
    uint32_t eff = hi > lo ? hi - lo : 0u;
    uint64_t ao = da + lo;
    if constexpr (kXlate) {
      if (ml > 0) {
        uint64_t dd;
        if (walk_xlate(R, nreg, da, ml, &dd)) {
          ao = dd + lo;
        } else {
          st |= kWalkUnmapped;
          eff = 0;
          nx = 0;
        }
      }
    }
    const uint32_t head = eff ? (uint32_t)(ao & 15u) : 0u;
    const uint32_t nch = eff ? (eff >> 4) + ((head + (eff & 15u) + 15u) >> 4) : 0u;
    const uint64_t c0 = ao - head;
    const uint32_t rot = ((pos + lo - S) ^ (uint32_t)ao) & 1u;
    const uint32_t meta = ((uint32_t)lane << 1) | rot;

    // --- advance: next header out before anything waits on this round ----
    const uint32_t pos1 = pos + ml;
    const bool more = has && nx != 0 && pos1 < L;
    const bool capped = more && hops + 1 >= kHopsMax;
    if (capped) st |= kXlate ? kWalkFallback : (uint32_t)UINET_CKSUM_MBUF_TRUNC;
    const bool cont = more && !capped;
    const bool fin = p != kNone && !cont;
    const uint32_t pf = fin ? p : kNone, sf = sd;
    if (cont) {
      m = nx;
      pos = pos1;
      hops++;
      hdr_issue(m);
    }
    take_job(fin);

    // --- long segments (>= 2 KiB): one wave-wide stream over all of them -
    // Items of kLongU chunks per lane, the round's long segments one after
    // another, item i + 1's loads issued before item i is summed (ping-pong
    // register sets: a copy of loads in flight would wait for them).
    const bool is_long = nch >= kLongCh;
    if (uint64_t lm = __ballot(is_long)) {
      const uint32_t c0_lo = (uint32_t)c0, c0_hi = (uint32_t)(c0 >> 32);
      struct LongSeg {
        uint64_t cb;
        uint32_t h, nc, last_end, mts;
      };
      auto seg_at = [&](int sl) {
        LongSeg g;
        g.h = __builtin_amdgcn_readlane(head, sl);
        const uint32_t el = __builtin_amdgcn_readlane(eff, sl);
        g.mts = __builtin_amdgcn_readlane(meta, sl);
        g.cb = readlane_u64(c0_lo, c0_hi, sl);
        g.nc = __builtin_amdgcn_readlane(nch, sl);
        g.last_end = ((g.h + (el & 15u) + 15u) & 15u) + 1u;
        return g;
      };
      auto load = [&](const LongSeg& g, uint32_t k0, u32x4 (&v)[kLongU]) {
#pragma unroll
        for (int u = 0; u < kLongU; ++u)
          if (u == 0 || k0 + 64u * u < g.nc)
            v[u] = gload_chunk(g.cb + 16ull * min(k0 + (uint32_t)(u * 64 + lane), g.nc - 1));
        asm volatile("" ::: "memory");  // keep the loads here, ahead of the sums
      };
      auto sum = [&](const LongSeg& g, uint32_t k0, const u32x4 (&v)[kLongU]) {
        uint32_t part = 0;  // < kLongU * 2^19
#pragma unroll
        for (int u = 0; u < kLongU; ++u) {
          if (u == 0 || k0 + 64u * u < g.nc) {
            const uint32_t k = k0 + (uint32_t)(u * 64 + lane);
            const int lo_b = k == 0 ? (int)g.h : (k < g.nc ? 0 : 16);
            const int hi_b = k + 1 < g.nc ? 16 : (k + 1 == g.nc ? (int)g.last_end : 0);
            part += lut.sum_oc(v[u], lo_b, hi_b);
          }
        }
        return part;
      };
      int sl = (int)__builtin_ctzll(lm);
      lm &= lm - 1;
      LongSeg g = seg_at(sl);
      uint32_t k0 = 0;
      uint64_t tot = 0;
      u32x4 la[kLongU], lb[kLongU];
      load(g, 0, la);
      auto step = [&](const u32x4 (&cur)[kLongU], u32x4 (&nxt)[kLongU]) {
        LongSeg g2 = g;
        uint32_t k2 = k0 + 64u * kLongU;
        bool more = true, next_seg = false;
        if (k2 >= g.nc) {
          if (lm) {
            sl = (int)__builtin_ctzll(lm);
            lm &= lm - 1;
            g2 = seg_at(sl);
            k2 = 0;
            next_seg = true;
          } else {
            more = false;
          }
        }
        if (more) load(g2, k2, nxt);
        tot += sum(g, k0, cur);
        if (!more || next_seg) {  // the segment's sum into its (lane, parity) bin
          const uint32_t x = __builtin_amdgcn_readlane(wave_scan<0, false>(fold16(tot), 0u), 63);
          if (lane == 0) atomicAdd(&acc[g.mts], (unsigned long long)x);
          tot = 0;
        }
        g = g2;
        k0 = k2;
        return more;
      };
      while (step(la, lb) && step(lb, la)) {
      }
    }

    // --- the round's chunk list ------------------------------------------
    const uint32_t nch_l = is_long ? 0u : nch;
    const uint32_t ci = wave_scan<0, false>(nch_l, 0u);
    const uint32_t cst = ci - nch_l;
    const uint32_t C = __builtin_amdgcn_readlane(ci, 63);  // < 64 * kLongCh
    const uint64_t lm_list = __ballot(nch_l != 0);
    if (lm_list != 0) {
      const uint32_t c0_lo = (uint32_t)c0, c0_hi = (uint32_t)(c0 >> 32);
      const int lf = (int)__builtin_ctzll(lm_list);
      const uint64_t R0 = readlane_u64(c0_lo, c0_hi, lf);
      const uint64_t rel = c0 - R0 + (1ull << 31);  // R0 - 2 GiB .. R0 + 2 GiB
      const bool window = __ballot(nch_l != 0 && rel >= (1ull << 32) - (1ull << 16)) == 0;
      // the segment's kept bytes [q0, q0 + eff) in list bytes, as a pair of
      // 16-bit halves, computed modulo 2^16: a chunk's bounds relative to its
      // own segment stay within +-2 KiB, exact in 16 bits
      const uint32_t q0 = head + 16u * cst;
      const uint32_t r16 = (q0 & 0xffffu) | ((q0 + eff) << 16);
      const uint16_t mval = (uint16_t)(((uint32_t)lane + 1u) << 8 | meta);
      const uint64_t dk = c0 - 16ull * cst;
      const uint32_t dkr = (uint32_t)rel - 16u * cst;  // mod 2^32; + 16 c lands in range
      const __amdgpu_buffer_rsrc_t rsrc = mb_window_rsrc(R0 - (1ull << 31));
      uint32_t carry_seg1 = 0;  // segment + 1 of the chunk before the batch
      auto issue = [&](uint32_t b, u32x4 (&v)[kPass], uint32_t (&key)[kPass], auto kWindow) {
        const bool mk = nch_l != 0 && cst >= b && cst < b + kWin;
        const uint32_t mslot = mk ? cst - b : (uint32_t)(kWin + lane);
        mark[mslot] = mval;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        uint32_t sc1[kPass];
#pragma unroll
        for (int k = 0; k < kPass; ++k) sc1[k] = mark[k * 64 + lane];
#pragma unroll
        for (int k = 0; k < kPass; ++k) sc1[k] = wave_scan<1, false>(sc1[k], 0u);
#pragma unroll
        for (int k = 0; k < kPass; ++k) {
          const uint32_t last = __builtin_amdgcn_readlane(sc1[k], 63);
          sc1[k] = max(sc1[k], carry_seg1);
          carry_seg1 = max(carry_seg1, last);
        }
        const short b16 = (short)(16u * b);
        const s16x2 rb = __builtin_bit_cast(s16x2, r16) - s16x2{b16, b16};
        const uint32_t rbw = __builtin_bit_cast(uint32_t, rb);
#pragma unroll
        for (int k = 0; k < kPass; ++k) {
          const uint32_t c = b + (uint32_t)(k * 64 + lane);
          const uint32_t cc = min(c, C - 1);  // past the end: the last chunk, masked
          // the segment's lane (mark >> 8, minus 1) as a ds_bpermute byte address
          const int src = (int)((sc1[k] >> 8) << 2) - 4;
          const s16x2 pr =
              __builtin_bit_cast(s16x2, (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)rbw)) -
              lane16[k];
          const s16x2 cl = __builtin_elementwise_min(__builtin_elementwise_max(pr, s16x2{0, 0}),
                                                     s16x2{16, 16});
          // mask index lo * 17 + hi, and meta (byte 0 of the mark) in byte 2
          key[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(us16x2, cl), us16x2{17, 1},
                                          __builtin_amdgcn_perm(0u, sc1[k], 0x0c000c0cu), false);
          if constexpr (decltype(kWindow)::value) {
            const uint32_t d = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)dkr);
            v[k] = mb_load_chunk_buf<kTemporal>(rsrc, d + 16u * cc);
          } else {
            const uint32_t lo32 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)dk);
            const uint32_t hi32 =
                (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(dk >> 32));
            v[k] = gload_chunk<kTemporal>((((uint64_t)hi32 << 32) | lo32) + 16ull * cc);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        mark[mslot] = 0;
      };
      auto run = [&](auto kWindow) {
        uint32_t pend = 0;
        for (uint32_t b = 0; b < C; b += kWin) {
          issue(b, vb, kb, kWindow);
          if (pend) consume(va, ka);
#pragma unroll
          for (int k = 0; k < kPass; ++k) {
            va[k] = vb[k];
            ka[k] = kb[k];
          }
          pend = 1;
        }
        if (pend) consume(va, ka);
      };
      if (window)
        run(std::true_type());
      else
        run(std::false_type());
    }

    // --- results of the chains that ended this round ---------------------
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (pf != kNone) {
      const uint32_t odd = fold16(acc[2 * lane + 1]);
      out[pf] = finish(acc[2 * lane] + rot8(odd) + sf, flags);
      acc[2 * lane] = 0;
      acc[2 * lane + 1] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // --- the next 64 jobs into the ring (here, where the round's registers
    // are dead; the loads wait, once per 64 packets)
    fill();
  }
  // one atomic per wave, only when something was flagged
  for (int d = 32; d; d >>= 1) st |= (uint32_t)__shfl_xor((int)st, d);
  if (status && lane == 0 && st) atomicOr(status, st);
}

template <bool kXlate, bool kTemporal>
int launch_mbufs_t(const uint64_t* heads, const int32_t* len, const int32_t* skip,
                   const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                   const WalkRegionHost* regions, int nreg, bool pseudo, uint32_t* status,
                   hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  // persistent: 5 blocks of 4 waves per CU (the kernel's occupancy), each
  // wave a contiguous range of packets; batches too small to give every wave
  // 16 packets get fewer waves.  (At 128 packets per wave, 5tso's 131 K
  // packets ran on 1,024 waves, one per SIMD: the few lanes of a wave that
  // hold a packet still stream its long payload wave-wide, so it is the
  // waves in flight that count.)
  const uint64_t cap = 256ull * (uint64_t)blocks_per_cu(5) * kWaves;
  uint64_t waves = ((uint64_t)n + 15) / 16;
  waves = waves < cap ? waves : cap;
  waves = (waves + kWaves - 1) / kWaves * kWaves;
  const uint32_t per_wave = (uint32_t)(((uint64_t)n + waves - 1) / waves);
  const int blocks = (int)(waves / kWaves);
  UINET_LAUNCH((k_mbufs<kXlate, kTemporal>), dim3(blocks), dim3(kBlock), 0, stream, heads, len,
               skip, seed,
               out, n, per_wave, flags, regions, nreg, pseudo ? 1 : 0, status);
  return check_launch();
}

}  // namespace

// Mean mbuf lengths below this take temporal packet-byte loads (k_mbufs).
constexpr uint32_t kTemporalSegMax = 256;

int launch_mbufs(const uint64_t* heads, const int32_t* len, const int32_t* skip,
                 const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                 uint32_t seg_hint, uint32_t* status, hipStream_t stream) {
  if (seg_hint != 0 && seg_hint < kTemporalSegMax)
    return launch_mbufs_t<false, true>(heads, len, skip, seed, out, n, flags, nullptr, 0, false,
                                       status, stream);
  return launch_mbufs_t<false, false>(heads, len, skip, seed, out, n, flags, nullptr, 0, false,
                                      status, stream);
}

int launch_mbufs_xlate(const uint64_t* heads, const int32_t* len, const int32_t* skip,
                       const uint32_t* seed, const WalkRegionHost* regions, int nreg, bool pseudo,
                       uint16_t* out, uint32_t n, uint32_t flags, uint32_t* status,
                       hipStream_t stream) {
  if (nreg < 1 || nreg > kWalkRegionsMax) return UINET_CKSUM_EINVAL;
  // non-temporal: temporal loads measured 0-4 % slower on the hooks
  // (profiles/r06/r06hostt/)
  return launch_mbufs_t<true, false>(heads, len, skip, seed, out, n, flags, regions, nreg,
                                     pseudo, status, stream);
}

}  // namespace uinet
