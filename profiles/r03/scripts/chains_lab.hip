// Chain-kernel lab (measurement tool, not product): config-3-shaped chains
// built on the host, every kernel variant timed interleaved in one process
// and checked bit-identical against the shipped k_chains_pipe.
//
//   tools/chains_lab [packets] [rounds]
//
// Includes the shipped kernels (cksum_chains.hip) and adds candidates that
// are not (yet) part of the library.  Prints one JSON object.
#include "../libuinet_amd/csrc/cksum_chains.hip"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <random>
#include <string>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

namespace uinet {
// the library's host-side pieces the included kernels' launchers reference
Tuning tuning() {
  Tuning t{};
  t.chains_pass = 2;
  t.chains_long = 128;
  return t;
}
int blocks_per_cu(int d) { return d; }
int record_hip(hipError_t e) { return e == hipSuccess ? 0 : -1; }
int check_launch() { return record_hip(hipGetLastError()); }

namespace lab {

// kN independent inclusive add-scans over the wave, step by step side by side
// so the DPP read-after-write waits of one chain fill with the others' work.
template <int kN>
__device__ __forceinline__ void wave_scan_n(uint32_t (&x)[kN]) {
#define LAB_STEP(CTRL, RMASK)                                                                 \
  _Pragma("unroll") for (int i = 0; i < kN; ++i) x[i] +=                                     \
      (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x[i], CTRL, RMASK, 0xf, true);
  LAB_STEP(0x111, 0xf)
  LAB_STEP(0x112, 0xf)
  LAB_STEP(0x114, 0xf)
  LAB_STEP(0x118, 0xf)
  LAB_STEP(0x142, 0xa)
  LAB_STEP(0x143, 0xc)
#undef LAB_STEP
}

// ---------------------------------------------------------------------------
// k_lps: one lane per segment.  The descriptor round is k_chains_pipe's; then
// each lane streams its own segment's chunks, kU per step, double-buffered,
// with no chunk list, no per-chunk segment lookup and one binning scan per
// round instead of one per pass.
template <int kU, int kTile>
__global__ __launch_bounds__(kBlock) void k_lps(const uint8_t* __restrict__ base,
                                               const uint64_t* __restrict__ seg_off,
                                               const uint32_t* __restrict__ seg_len,
                                               const uint32_t* __restrict__ pkt_seg,
                                               const uint32_t* __restrict__ plen,
                                               const uint32_t* __restrict__ pskip,
                                               const uint32_t* __restrict__ seed,
                                               uint16_t* __restrict__ out, uint32_t n,
                                               uint32_t flags, uint32_t long_ch) {
  __shared__ MaskLut lut;
  __shared__ uint32_t lds_acc[kWaves][64];
  __shared__ uint32_t lds_pkmark[kWaves][64];
  lut.init();
  for (int i = threadIdx.x; i < kWaves * 64; i += blockDim.x) (&lds_pkmark[0][0])[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  uint32_t* acc = lds_acc[wid];
  uint32_t* pkmark = lds_pkmark[wid];
  const uint32_t tiles = (n + kTile - 1) / kTile;
  const uint32_t wstride = gridDim.x * kWaves;
  for (uint32_t t = blockIdx.x * kWaves + wid; t < tiles; t += wstride) {
    const uint32_t P0 = t * kTile;
    const int np = (int)min((uint32_t)kTile, n - P0);
    const uint32_t ps = pkt_seg[P0 + (uint32_t)min(lane, np)];
    const uint32_t k_skip = (lane < np && pskip) ? pskip[P0 + lane] : 0u;
    const uint32_t k_len = (lane < np) ? (plen ? plen[P0 + lane] : 0xffffffffu) : 0u;
    const uint32_t S0 = __builtin_amdgcn_readfirstlane(ps);
    const uint32_t S1 = __builtin_amdgcn_readlane(ps, np);
    acc[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t carry_slot1 = 0, carry_pos = 0;
    uint64_t so_next = 0;
    uint32_t l_next = 0;
    auto fetch = [&](uint32_t r) {
      const uint32_t s = r + (uint32_t)lane;
      const uint32_t sc = s < S1 ? s : S1 - 1;
      so_next = seg_off[sc];
      l_next = s < S1 ? seg_len[sc] : 0u;
    };
    if (S0 < S1) fetch(S0);
    for (uint32_t r0 = S0; r0 < S1; r0 += 64) {
      const uint64_t so = so_next;
      const uint32_t l = l_next;
      if (r0 + 64 < S1) fetch(r0 + 64);
      const bool pk_in = lane < np && ps >= r0 && ps < r0 + 64;
      if (pk_in) atomicMax(&pkmark[ps - r0], (uint32_t)lane + 1);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const uint32_t pk = pkmark[lane];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (pk_in) pkmark[ps - r0] = 0;
      const uint32_t slot1 = max(wave_scan<1, false>(pk, 0u), carry_slot1);
      const uint32_t slot = slot1 - 1;
      const uint32_t T = carry_pos + wave_scan<0, false>(l, 0u) - l;
      const uint32_t pos = T - wave_scan<1, false>(pk ? T : 0u, 0u);
      carry_slot1 = __builtin_amdgcn_readlane(slot1, 63);
      carry_pos = __builtin_amdgcn_readlane(pos + l, 63);
      const uint32_t sk = __shfl(k_skip, (int)slot);
      const uint32_t ln = __shfl(k_len, (int)slot);
      const uint32_t lo = sk > pos ? min(sk - pos, l) : 0u;
      const uint32_t hi = ln > pos ? min(ln - pos, l) : 0u;
      const uint32_t eff = hi > lo ? hi - lo : 0u;
      const uint8_t* a = base + so + lo;
      const uint32_t head = eff ? (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15) : 0u;
      const uint32_t nch = eff ? (eff >> 4) + ((head + (eff & 15u) + 15u) >> 4) : 0u;
      const uint8_t* cp = a - head;
      const uint32_t rot = ((pos + lo - sk) ^ (uint32_t)reinterpret_cast<uintptr_t>(a)) & 1u;
      uint32_t x = 0;
      // long segments: the whole wave streams each one
      const bool is_long = long_ch != 0 && nch >= long_ch;
      for (uint64_t lm = __ballot(is_long); lm; lm &= lm - 1) {
        const int s = (int)__builtin_ctzll(lm);
        const uint32_t h = __builtin_amdgcn_readlane(head, s);
        const uint32_t el = __builtin_amdgcn_readlane(eff, s);
        const uint8_t* cb = (const uint8_t*)(((uint64_t)__builtin_amdgcn_readlane(
                                                  (uint32_t)((uintptr_t)cp >> 32), s)
                                              << 32) |
                                             __builtin_amdgcn_readlane((uint32_t)(uintptr_t)cp, s));
        const uint32_t nc = __builtin_amdgcn_readlane(nch, s);
        const uint32_t last_end = ((h + (el & 15u) + 15u) & 15u) + 1u;
        uint64_t lsum = 0;
        for (uint32_t k0 = 0; k0 < nc; k0 += 64 * 4) {
          u32x4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (u == 0 || k0 + 64u * u < nc)
              v[u] = load_chunk(cb + 16ull * min(k0 + (uint32_t)(u * 64 + lane), nc - 1));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (u == 0 || k0 + 64u * u < nc) {
              const uint32_t k = k0 + (uint32_t)(u * 64 + lane);
              const int lo_b = k == 0 ? (int)h : (k < nc ? 0 : 16);
              const int hi_b = k + 1 < nc ? 16 : (k + 1 == nc ? (int)last_end : 0);
              lsum += lut.sum(v[u], lo_b, hi_b);
            }
          }
        }
        const uint32_t w = __builtin_amdgcn_readlane(wave_scan<0, false>(fold16(lsum), 0u), 63);
        if (lane == s) x = w;
      }
      const uint32_t nl = is_long ? 0u : nch;
      const uint32_t maxn = __builtin_amdgcn_readlane(wave_scan<1, false>(nl, 0u), 63);
      const int e = (int)(head + eff);
      uint32_t sacc = 0;
      u32x4 va[kU], vb[kU];
      auto issue = [&](uint32_t j0, u32x4(&v)[kU]) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const uint32_t k = j0 + (uint32_t)u;
          if (k < nl) v[u] = load_chunk(cp + 16u * k);
        }
      };
      auto sum = [&](uint32_t j0, const u32x4(&v)[kU]) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const uint32_t k = j0 + (uint32_t)u;
          const uint32_t idx = k < nl ? MaskLut::index((int)head - 16 * (int)k, e - 16 * (int)k) : 0u;
          sacc += lut.sum_oc_idx(v[u], idx);
        }
      };
      if (maxn) issue(0, va);
      for (uint32_t j0 = 0; j0 < maxn; j0 += 2 * kU) {
        if (j0 + kU < maxn) issue(j0 + kU, vb);
        sum(j0, va);
        if (j0 + kU >= maxn) break;
        if (j0 + 2 * kU < maxn) issue(j0 + 2 * kU, va);
        sum(j0 + kU, vb);
      }
      if (nl) x = fold16_32(sacc);
      if (rot) x = rot8(x);
      // per-packet sums: telescoping prefix over the round's lanes (slots
      // never decrease along the lanes)
      const uint32_t P = wave_scan<0, false>(x, 0u);
      const uint32_t nx = wave_shl1(slot);
      if (lane == 63 || nx != slot) {
        atomicAdd(&acc[slot], P);
        if (lane != 63) atomicAdd(&acc[nx], 0u - P);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane < np) {
      const uint32_t p = P0 + (uint32_t)lane;
      out[p] = finish((uint64_t)acc[lane] + (seed ? seed[p] : 0u), flags);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}


// ---------------------------------------------------------------------------
// k_grp: G lanes per segment.  The descriptor round is k_chains_pipe's; the
// round's short segments then go G lanes at a time (64 / G segments per step),
// each lane loading U chunks of its group's segment, with no chunk list and
// no per-chunk segment lookup: one 16-B LDS record per segment, a DPP group
// sum, one LDS atomic per segment into its packet's bin (rotated first).
template <int G, int U, int kTile>
__global__ __launch_bounds__(kBlock) void k_grp(const uint8_t* __restrict__ base,
                                               const uint64_t* __restrict__ seg_off,
                                               const uint32_t* __restrict__ seg_len,
                                               const uint32_t* __restrict__ pkt_seg,
                                               const uint32_t* __restrict__ plen,
                                               const uint32_t* __restrict__ pskip,
                                               const uint32_t* __restrict__ seed,
                                               uint16_t* __restrict__ out, uint32_t n,
                                               uint32_t flags, uint32_t long_ch) {
  static_assert(G == 4 || G == 8 || G == 16, "group sums stay inside a 16-lane DPP row");
  constexpr int S = 64 / G;  // segments per step
  __shared__ MaskLut lut;
  __shared__ unsigned long long lds_acc[kWaves][kTile];
  __shared__ uint32_t lds_pkmark[kWaves][64];
  __shared__ u32x4 lds_rec[kWaves][64];
  lut.init();
  for (int i = threadIdx.x; i < kWaves * 64; i += blockDim.x) (&lds_pkmark[0][0])[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int gl = lane & (G - 1), gi = lane / G;
  unsigned long long* acc = lds_acc[wid];
  uint32_t* pkmark = lds_pkmark[wid];
  u32x4* rec = lds_rec[wid];
  const uint32_t tiles = (n + kTile - 1) / kTile;
  const uint32_t wstride = gridDim.x * kWaves;
  for (uint32_t t = blockIdx.x * kWaves + wid; t < tiles; t += wstride) {
    const uint32_t P0 = t * kTile;
    const int np = (int)min((uint32_t)kTile, n - P0);
    const uint32_t ps = pkt_seg[P0 + (uint32_t)min(lane, np)];
    const uint32_t k_skip = (lane < np && pskip) ? pskip[P0 + lane] : 0u;
    const uint32_t k_len = (lane < np) ? (plen ? plen[P0 + lane] : 0xffffffffu) : 0u;
    const uint32_t S0 = __builtin_amdgcn_readfirstlane(ps);
    const uint32_t S1 = __builtin_amdgcn_readlane(ps, np);
    if (lane < kTile) acc[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t carry_slot1 = 0, carry_pos = 0;
    uint64_t so_next = 0;
    uint32_t l_next = 0;
    auto fetch = [&](uint32_t r) {
      const uint32_t s = r + (uint32_t)lane;
      const uint32_t sc = s < S1 ? s : S1 - 1;
      so_next = seg_off[sc];
      l_next = s < S1 ? seg_len[sc] : 0u;
    };
    if (S0 < S1) fetch(S0);
    for (uint32_t r0 = S0; r0 < S1; r0 += 64) {
      const uint64_t so = so_next;
      const uint32_t l = l_next;
      if (r0 + 64 < S1) fetch(r0 + 64);
      const bool pk_in = lane < np && ps >= r0 && ps < r0 + 64;
      if (pk_in) atomicMax(&pkmark[ps - r0], (uint32_t)lane + 1);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const uint32_t pk = pkmark[lane];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (pk_in) pkmark[ps - r0] = 0;
      const uint32_t slot1 = max(wave_scan<1, false>(pk, 0u), carry_slot1);
      const uint32_t slot = slot1 - 1;
      const uint32_t T = carry_pos + wave_scan<0, false>(l, 0u) - l;
      const uint32_t pos = T - wave_scan<1, false>(pk ? T : 0u, 0u);
      carry_slot1 = __builtin_amdgcn_readlane(slot1, 63);
      carry_pos = __builtin_amdgcn_readlane(pos + l, 63);
      const uint32_t sk = __shfl(k_skip, (int)slot);
      const uint32_t ln = __shfl(k_len, (int)slot);
      const uint32_t lo = sk > pos ? min(sk - pos, l) : 0u;
      const uint32_t hi = ln > pos ? min(ln - pos, l) : 0u;
      const uint32_t eff = hi > lo ? hi - lo : 0u;
      const uint8_t* a = base + so + lo;
      const uint32_t head = eff ? (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15) : 0u;
      const uint32_t nch = eff ? (eff >> 4) + ((head + (eff & 15u) + 15u) >> 4) : 0u;
      const uint8_t* cp = a - head;
      const uint32_t rot = ((pos + lo - sk) ^ (uint32_t)reinterpret_cast<uintptr_t>(a)) & 1u;
      const bool is_long = nch >= kListMax || (long_ch != 0 && nch >= long_ch);
      for (uint64_t lm = __ballot(is_long); lm; lm &= lm - 1) {
        const int s = (int)__builtin_ctzll(lm);
        const uint32_t h = __builtin_amdgcn_readlane(head, s);
        const uint32_t el = __builtin_amdgcn_readlane(eff, s);
        const uint8_t* cb = (const uint8_t*)(((uint64_t)__builtin_amdgcn_readlane(
                                                  (uint32_t)((uintptr_t)cp >> 32), s)
                                              << 32) |
                                             __builtin_amdgcn_readlane((uint32_t)(uintptr_t)cp, s));
        const uint32_t nc = __builtin_amdgcn_readlane(nch, s);
        const uint32_t last_end = ((h + (el & 15u) + 15u) & 15u) + 1u;
        uint64_t lsum = 0;
        for (uint32_t k0 = 0; k0 < nc; k0 += 64 * 4) {
          u32x4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (u == 0 || k0 + 64u * u < nc)
              v[u] = load_chunk(cb + 16ull * min(k0 + (uint32_t)(u * 64 + lane), nc - 1));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (u == 0 || k0 + 64u * u < nc) {
              const uint32_t k = k0 + (uint32_t)(u * 64 + lane);
              const int lo_b = k == 0 ? (int)h : (k < nc ? 0 : 16);
              const int hi_b = k + 1 < nc ? 16 : (k + 1 == nc ? (int)last_end : 0);
              lsum += lut.sum(v[u], lo_b, hi_b);
            }
          }
        }
        uint32_t w = __builtin_amdgcn_readlane(wave_scan<0, false>(fold16(lsum), 0u), 63);
        if (__builtin_amdgcn_readlane(rot, s)) w = rot8(w);
        if (lane == 0) atomicAdd(&acc[__builtin_amdgcn_readlane(slot, s)], (unsigned long long)w);
      }
      const uint32_t nl = is_long ? 0u : nch;
      if (__ballot(nl != 0) == 0) continue;
      rec[lane] = u32x4{(uint32_t)(uintptr_t)cp, (uint32_t)((uintptr_t)cp >> 32),
                        head | (eff << 4), (slot << 1) | rot | (nl << 8)};
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const uint32_t nsteps = (min(64u, S1 - r0) + S - 1) / S;
      for (uint32_t j = 0; j < nsteps; ++j) {
        const u32x4 rc = rec[j * S + gi];
        const uint8_t* cb = (const uint8_t*)(((uint64_t)rc.y << 32) | rc.x);
        const int h = (int)(rc.z & 15u);
        const int e = h + (int)(rc.z >> 4);
        const uint32_t nlg = rc.w >> 8;
        uint32_t sacc = 0;
        for (uint32_t k0 = 0;; k0 += G * U) {
          u32x4 v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t k = k0 + (uint32_t)(u * G + gl);
            if (k < nlg) v[u] = load_chunk(cb + 16u * k);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t k = k0 + (uint32_t)(u * G + gl);
            const uint32_t idx = k < nlg ? MaskLut::index(h - 16 * (int)k, e - 16 * (int)k) : 0u;
            sacc += lut.sum_oc_idx(v[u], idx);
          }
          if (__ballot(nlg > k0 + G * U) == 0) break;
        }
        uint32_t x = fold16_32(sacc);
        // inclusive sums inside 16-lane rows: lane G-1 of each group ends with
        // its group's total
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
        if constexpr (G >= 8) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
        if constexpr (G >= 16) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
        if (gl == G - 1 && nlg) {
          x = fold16_32(x);
          if (rc.w & 1u) x = rot8(x);
          atomicAdd(&acc[(rc.w >> 1) & 0x7fu], (unsigned long long)x);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane < np) {
      const uint32_t p = P0 + (uint32_t)lane;
      out[p] = finish(acc[lane] + (seed ? seed[p] : 0u), flags);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

// k_chains_pipe with ablations: 1 = no chunk arithmetic / binning (bytes
// xor-ed into a register), 2 = no loads, 3 = chunk sums but no binning.
// tile timeline of the kAbl = 12 variant (set by the host in timeline mode)
__device__ unsigned long long* g_ts;
__device__ uint32_t g_bc[2][16 * 2048];  // kAbl 21 / 22 block counters, two sets
__device__ uint32_t g_q[256];  // kAbl = 13 / 19 work queues (zero at load time)

template <int kAbl, int kPass, int kTile, typename OffT, typename LenT>
__global__ __launch_bounds__((kAbl == 21 || kAbl == 22) ? 768 : kBlock) __attribute__((amdgpu_waves_per_eu(6))) UINET_CHAINS_OCC void k_pipe_abl(const uint8_t* __restrict__ base,
                                                       const OffT* __restrict__ seg_off,
                                                       const LenT* __restrict__ seg_len,
                                                       const uint32_t* __restrict__ pkt_seg,
                                                       const uint32_t* __restrict__ plen,
                                                       const uint32_t* __restrict__ pskip,
                                                       const uint32_t* __restrict__ seed,
                                                       uint16_t* __restrict__ out, uint32_t n,
                                                       uint32_t flags, uint32_t long_ch) {
  static_assert(kTile >= 1 && kTile <= 63,
                "a tile's packets are one per lane, lane kTile reads the end of its segment "
                "range, and its 2 * kTile bins are one per lane");
  constexpr int kWin = 64 * kPass;  // chunks per batch of passes
  constexpr bool kBP = kAbl == 21 || kAbl == 22;
  constexpr int kWB = (kAbl == 16 || kAbl == 18) ? 1 : (kAbl == 17 ? 2 : ((kAbl == 21 || kAbl == 22) ? 12 : kWaves));  // waves per block
  __shared__ MaskLut lut;
  __shared__ unsigned long long lds_acc[kWB][2 * kTile];  // (slot, rot) bins
  __shared__ uint32_t lds_pkmark[kWB][64];  // packet-start markers (slot + 1)
  __shared__ uint8_t lds_mark[kWB][kWin];   // segment-start markers (lane + 1)
  lut.init();
  for (int i = threadIdx.x; i < kWB * 64; i += blockDim.x) (&lds_pkmark[0][0])[i] = 0;
  for (int i = threadIdx.x; i < kWB * kWin; i += blockDim.x) (&lds_mark[0][0])[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned long long* acc = lds_acc[wid];
  uint32_t* pkmark = lds_pkmark[wid];
  uint8_t* mark = lds_mark[wid];
  const uint32_t tiles = (n + kTile - 1) / kTile;
  const uint32_t wstride = gridDim.x * kWB;

  // the pipeline's register sets: the pending batch (issued, not yet
  // consumed; `pend` wave-uniform) in a, the one being issued in b
  u32x4 va[kPass], vb[kPass];
  uint32_t ka[kPass], kb[kPass];
  uint32_t pend = 0;
  uint32_t dummy = 0;
  auto consume = [&](const auto& v, const auto& key) {
    constexpr int NP = sizeof(key) / sizeof(key[0]);
    if constexpr (kAbl == 8 || kAbl == 11 || kAbl == 12 || kAbl == 13 || kAbl == 14 || kAbl == 15 || kAbl == 16 || kAbl == 17 || kAbl == 18 || kAbl == 19 || kAbl == 20 || kAbl == 21 || kAbl == 22) {
      // every pass's chunk sums first, then the passes' scans side by side
      // (independent DPP chains interleave), then the bin updates
      uint32_t P[NP], sl[NP], nx[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) P[q] = lut.sum_oc_idx(v[q], key[q] & 0xffffu);
#pragma unroll
      for (int q = 0; q < NP; ++q) { sl[q] = key[q] >> 16; nx[q] = wave_shl1(sl[q]); }
      wave_scan_n<NP>(P);
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        if (lane == 63 || nx[q] != sl[q]) {
          atomicAdd(&acc[sl[q]], (unsigned long long)P[q]);
          if (lane != 63) atomicAdd(&acc[nx[q]], (unsigned long long)(-(long long)P[q]));
        }
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      if constexpr (kAbl == 1) { dummy ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w ^ key[q]; continue; }
      const uint32_t w = lut.sum_oc_idx(v[q], key[q] & 0xffffu);  // < 2^17
      if constexpr (kAbl == 3) { dummy += w; continue; }
      const uint32_t sl = key[q] >> 16;
      if constexpr (kAbl == 6) { atomicAdd(&acc[sl], (unsigned long long)w); continue; }
      if constexpr (kAbl == 7) { atomicAdd(reinterpret_cast<uint32_t*>(&acc[sl]), w); continue; }
      const uint32_t P = wave_scan<0, false>(w, 0u);  // < 2^23
      const uint32_t nx = wave_shl1(sl);
      if (lane == 63 || nx != sl) {
        atomicAdd(&acc[sl], (unsigned long long)P);
        if (lane != 63) atomicAdd(&acc[nx], (unsigned long long)(-(long long)P));
      }
    }
  };

  // kAbl 13: tiles from a work queue (g_q[0]: next ticket, g_q[1]: waves
  // done; the last wave out resets both for the next launch on the stream)
  auto ticket = [&]() -> uint32_t {
    uint32_t x = 0;
    if (lane == 0) x = atomicAdd(&g_q[0], 1u);
    return __builtin_amdgcn_readfirstlane(x);
  };
  uint32_t t_next = 0;
  if constexpr (kAbl == 13) t_next = ticket();
  // kAbl 14 / 15: wave gw of W owns the contiguous packets [gw n / W,
  // (gw + 1) n / W) and walks them in tiles of kTile (15: + timeline)
  const uint32_t gw = blockIdx.x * kWB + wid;
  const uint32_t W = gridDim.x * kWB;
  const uint32_t r_lo = (uint32_t)((uint64_t)gw * n / W);
  const uint32_t r_hi = (uint32_t)((uint64_t)(gw + 1) * n / W);
  constexpr bool kRange = kAbl == 14 || kAbl == 15;
  // kAbl 19 / 20: 8 pools of tiles, one per XCD (workgroup i runs on XCD
  // i mod 8); pool x's first kStatic % of tiles split into contiguous
  // per-wave ranges, the rest taken one tile at a time from the pool's
  // counter (g_q[32 x], own 128-B line); the wave that takes the pool's last
  // failing ticket (one per pool wave) resets the counter. 20: + timeline.
  // kAbl 21 / 22: blocks of 12 waves (two per CU), block b owns the contiguous
  // tiles [b per, (b + 1) per) and its waves take them one at a time from the
  // block's counter g_bc[par][16 b]; the counters alternate between two sets
  // by launch parity (long_ch), and each launch zeroes the other set for the
  // next one.  A wave whose block is exhausted takes tiles from the next
  // kSteal blocks' counters.  22: + timeline.
  constexpr int kSteal = 4;
  const uint32_t par = long_ch & 1u;
  const uint32_t G_ = gridDim.x;
  const uint32_t per_blk = (tiles + G_ - 1) / G_;  // once, scalar
  auto blk_lo = [&](uint32_t v) { return min(v * per_blk, tiles); };
  auto bticket = [&](uint32_t v) -> uint32_t {  // wave-uniform
    uint32_t x = 0;
    if (lane == 0) x = atomicAdd(&g_bc[par][16 * v], 1u);
    return __builtin_amdgcn_readfirstlane(x);
  };
  uint32_t victim = 0;  // 0: own block, j: block + j
  auto bp_next = [&]() -> uint32_t {
    while (victim <= (uint32_t)kSteal) {
      uint32_t v = blockIdx.x + victim;
      if (v >= G_) v -= G_;
      const uint32_t lo = blk_lo(v), hi = blk_lo(v + 1);
      const uint32_t k = bticket(v);
      if (lo + k < hi) return lo + k;
      ++victim;
    }
    return 0xffffffffu;
  };
  constexpr bool kPool = kAbl == 19 || kAbl == 20;
  constexpr uint32_t kStaticPct = 70;
  const uint32_t px = blockIdx.x & 7u;
  const uint32_t nbx = (gridDim.x + 7u - px) >> 3;  // blocks of pool px
  const uint32_t Wx = nbx * kWB;
  const uint32_t wx = (blockIdx.x >> 3) * kWB + wid;
  const uint32_t p_lo = (uint32_t)((uint64_t)tiles * px / 8), p_hi = (uint32_t)((uint64_t)tiles * (px + 1) / 8);
  const uint32_t S = (p_hi - p_lo) * kStaticPct / 100;
  uint32_t s_cur = p_lo + (uint32_t)((uint64_t)S * wx / Wx);
  const uint32_t s_end = p_lo + (uint32_t)((uint64_t)S * (wx + 1) / Wx);
  auto pool_next = [&]() -> uint32_t {
    if (s_cur < s_end) return s_cur++;
    uint32_t x = 0;
    if (lane == 0) {
      x = atomicAdd(&g_q[32 * px], 1u);
      const uint32_t dyn = p_hi - p_lo - S;
      if (x == dyn + Wx - 1) atomicExch(&g_q[32 * px], 0u);  // the last ticket of this launch
    }
    x = __builtin_amdgcn_readfirstlane(x);
    return x < p_hi - p_lo - S ? p_lo + S + x : 0xffffffffu;
  };
  if constexpr (kBP) {  // the other set, for the next launch on this stream
    if (threadIdx.x == 0)
      for (uint32_t v = blockIdx.x; v < 2048u; v += G_) atomicExch(&g_bc[par ^ 1u][16 * v], 0u);
  }
  uint32_t it = 0;
  uint32_t bp_t = 0;
  if constexpr (kBP) bp_t = bp_next();
  for (uint32_t t = kBP ? bp_t : kPool ? pool_next() : kRange ? r_lo : (kAbl == 13 ? t_next : blockIdx.x * kWB + wid);
       kRange ? t < r_hi : t < tiles;
       t = kBP ? bp_t : kPool ? pool_next() : kRange ? t + kTile : (kAbl == 13 ? t_next : t + wstride), ++it) {
    if constexpr (kAbl == 13) t_next = ticket();  // one tile ahead
    if constexpr (kBP) bp_t = bp_next();  // one tile ahead
    uint64_t t_begin = 0;
    if constexpr (kAbl == 12 || kAbl == 15 || kAbl == 18 || kAbl == 20 || kAbl == 22) t_begin = wall_clock64();
    const uint32_t P0 = kRange ? t : t * kTile;
    const int np = (int)min((uint32_t)kTile, (kRange ? r_hi : n) - P0);
    const uint32_t ps = pkt_seg[P0 + (uint32_t)min(lane, np)];
    const uint32_t k_skip = (lane < np && pskip) ? pskip[P0 + lane] : 0u;
    const uint32_t k_len = (lane < np) ? (plen ? plen[P0 + lane] : 0xffffffffu) : 0u;
    const uint32_t S0 = __builtin_amdgcn_readfirstlane(ps);
    const uint32_t S1 = __builtin_amdgcn_readlane(ps, np);
    if (lane < 2 * kTile) acc[lane] = 0;
    if (kTile > 32 && lane + 64 < 2 * kTile) acc[lane + 64] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t carry_slot1 = 0;  // slot + 1 of the last segment of the previous round
    uint32_t carry_pos = 0;    // chain offset just past that segment
    uint64_t so_next = 0;
    uint32_t l_next = 0;
    auto fetch = [&](uint32_t r) {
      const uint32_t s = r + (uint32_t)lane;
      const uint32_t sc = s < S1 ? s : S1 - 1;
      so_next = (uint64_t)seg_off[sc];
      l_next = s < S1 ? (uint32_t)seg_len[sc] : 0u;
    };
    if (S0 < S1) fetch(S0);
    for (uint32_t r0 = S0; r0 < S1; r0 += 64) {
      // --- descriptor round: one segment per lane -------------------------
      const uint64_t so = so_next;
      const uint32_t l = l_next;
      if (r0 + 64 < S1) fetch(r0 + 64);
      const bool pk_in = lane < np && ps >= r0 && ps < r0 + 64;
      if (pk_in) atomicMax(&pkmark[ps - r0], (uint32_t)lane + 1);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const uint32_t pk = pkmark[lane];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (pk_in) pkmark[ps - r0] = 0;
      const uint32_t slot1 = max(wave_scan<1, false>(pk, 0u), carry_slot1);
      const uint32_t slot = slot1 - 1;
      // chain position: T = carry_pos + exclusive prefix of the lengths never
      // decreases along the lanes, so the max-scan of T at packet starts is
      // T at this segment's packet start (0 while the packet of the previous
      // round continues: its position is T itself)
      const uint32_t T = carry_pos + wave_scan<0, false>(l, 0u) - l;
      const uint32_t pos = T - wave_scan<1, false>(pk ? T : 0u, 0u);
      carry_slot1 = __builtin_amdgcn_readlane(slot1, 63);
      carry_pos = __builtin_amdgcn_readlane(pos + l, 63);
      const uint32_t sk = __shfl(k_skip, (int)slot);
      const uint32_t ln = __shfl(k_len, (int)slot);
      const uint32_t lo = sk > pos ? min(sk - pos, l) : 0u;
      const uint32_t hi = ln > pos ? min(ln - pos, l) : 0u;
      const uint32_t eff = hi > lo ? hi - lo : 0u;
      const uint64_t ao = so + lo;
      const uint32_t head = eff ? (uint32_t)(reinterpret_cast<uintptr_t>(base + ao) & 15) : 0u;
      // chunks touched, without forming head + eff (a u32 segment may be 4 GiB)
      const uint32_t nch = eff ? (eff >> 4) + ((head + (eff & 15u) + 15u) >> 4) : 0u;
      const uint64_t c0 = ao - head;
      const uint32_t rot = ((pos + lo - sk) ^ (uint32_t)reinterpret_cast<uintptr_t>(base + ao)) & 1u;
      const uint32_t meta = (slot << 1) | rot;
      const uint32_t c0_lo = (uint32_t)c0, c0_hi = (uint32_t)(c0 >> 32);
      // --- long segments: one wave-wide span each -------------------------
      const bool is_long = nch >= kListMax || (!kBP && long_ch != 0 && nch >= long_ch);
      for (uint64_t lm = __ballot(is_long); lm; lm &= lm - 1) {
        const int s = (int)__builtin_ctzll(lm);
        // head and length read separately: a segment may hold up to 4 GiB,
        // more than one packed 32-bit word (eff << 4 | head) keeps
        const uint32_t h = __builtin_amdgcn_readlane(head, s);
        const uint32_t el = __builtin_amdgcn_readlane(eff, s);
        const uint32_t mts = __builtin_amdgcn_readlane(meta, s);
        const uint8_t* cb = base + (((uint64_t)__builtin_amdgcn_readlane(c0_hi, s) << 32) |
                                    __builtin_amdgcn_readlane(c0_lo, s));
        const uint32_t nc = __builtin_amdgcn_readlane(nch, s);
        // chunk k keeps bytes [k ? 0 : h, k < nc - 1 ? 16 : last_end): only the
        // first and last chunks are partial, so no byte position is formed
        const uint32_t last_end = ((h + (el & 15u) + 15u) & 15u) + 1u;
        uint64_t lsum = 0;
        for (uint32_t k0 = 0; k0 < nc; k0 += 64 * kLongU) {
          u32x4 v[kLongU];
#pragma unroll
          for (int u = 0; u < kLongU; ++u)
            if (u == 0 || k0 + 64u * u < nc)
              v[u] = load_chunk(cb + 16ull * min(k0 + (uint32_t)(u * 64 + lane), nc - 1));
#pragma unroll
          for (int u = 0; u < kLongU; ++u) {
            if (u == 0 || k0 + 64u * u < nc) {
              const uint32_t k = k0 + (uint32_t)(u * 64 + lane);
              const int lo_b = k == 0 ? (int)h : (k < nc ? 0 : 16);
              const int hi_b = k + 1 < nc ? 16 : (k + 1 == nc ? (int)last_end : 0);
              lsum += lut.sum(v[u], lo_b, hi_b);
            }
          }
        }
        const uint32_t x = __builtin_amdgcn_readlane(wave_scan<0, false>(fold16(lsum), 0u), 63);
        if (lane == 0) atomicAdd(&acc[mts], (unsigned long long)x);
      }
      // --- the round's chunk list -----------------------------------------
      if constexpr (kAbl == 9) { dummy += nch ^ (uint32_t)c0; continue; }
      const uint32_t nch_l = is_long ? 0u : nch;
      const uint32_t ci = wave_scan<0, false>(nch_l, 0u);
      const uint32_t cst = ci - nch_l;
      const uint32_t C = __builtin_amdgcn_readlane(ci, 63);  // < 64 * kListMax
      const uint64_t lm_list = __ballot(nch_l != 0);
      if (lm_list == 0) continue;
      const int lf = (int)__builtin_ctzll(lm_list);
      const uint64_t R0 = ((uint64_t)__builtin_amdgcn_readlane(c0_hi, lf) << 32) |
                          __builtin_amdgcn_readlane(c0_lo, lf);
      const uint64_t rel = c0 - R0 + (1ull << 31);  // R0 - 2 GiB .. R0 + 2 GiB
      const bool window = __ballot(nch_l != 0 && rel >= (1ull << 32) - (1ull << 16)) == 0;
      const uint32_t q0 = head + 16u * cst;  // < 2^20
      const uint32_t recA = q0 | (meta << 20);
      const uint32_t recB = q0 + eff;
      const uint64_t dk = c0 - 16ull * cst;
      const uint32_t dkr = (uint32_t)rel - 16u * cst;  // mod 2^32; + 16 c lands in range
      const __amdgpu_buffer_rsrc_t rsrc = window_rsrc(base + (R0 - (1ull << 31)));
      uint32_t carry_seg1 = 0;  // segment + 1 of the chunk before the batch
      // Issue the batch at list chunk b into (v, key): segment lookup, mask
      // index and bin, loads.  Nothing here waits for packet bytes.
      auto issue = [&](uint32_t b, auto& v, auto& key, auto kWindow) {
        constexpr int NP = sizeof(key) / sizeof(key[0]);
        const bool mk = nch_l != 0 && cst >= b && cst < b + 64u * NP;
        if (mk) mark[cst - b] = (uint8_t)(lane + 1);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        uint32_t sc1[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) sc1[q] = mark[q * 64 + lane];
#pragma unroll
        for (int q = 0; q < NP; ++q) sc1[q] = wave_scan<1, false>(sc1[q], 0u);
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          const uint32_t last = __builtin_amdgcn_readlane(sc1[q], 63);
          sc1[q] = max(sc1[q], carry_seg1);
          carry_seg1 = max(carry_seg1, last);
        }
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          const uint32_t c = b + (uint32_t)(q * 64 + lane);
          const bool in = c < C;
          const uint32_t cc = in ? c : C - 1;  // past the end: the last chunk, masked
          const int seg = (int)sc1[q] - 1;
          // cross-lane reads stay outside any condition (a ds_bpermute under
          // a partial exec mask reads 0 from the inactive source lanes)
          const uint32_t a = (uint32_t)__shfl(recA, seg);
          const uint32_t bq = (uint32_t)__shfl(recB, seg);
          const int base16 = 16 * (int)c;
          const int s_lo = (int)(a & 0xfffffu) - base16;
          const int s_hi = in ? (int)bq - base16 : s_lo;
          key[q] = MaskLut::index(s_lo, s_hi) | ((a >> 20) << 16);
          if constexpr (decltype(kWindow)::value) {
            const uint32_t d = (uint32_t)__shfl(dkr, seg);
            if constexpr (kAbl == 2) v[q] = u32x4{d, cc, a, bq}; else
            v[q] = load_chunk_buf(rsrc, d + 16u * cc);
          } else {
            const uint32_t lo32 = (uint32_t)__shfl((uint32_t)dk, seg);
            const uint32_t hi32 = (uint32_t)__shfl((uint32_t)(dk >> 32), seg);
            v[q] = load_chunk(base + ((((uint64_t)hi32 << 32) | lo32) + 16ull * cc));
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (mk) mark[cst - b] = 0;
      };
      auto run = [&](auto kWindow) {
        if constexpr (kAbl == 4) {
          // ping-pong: batch k+1 is issued into the other register set while
          // batch k is consumed; no register copy, so no vmcnt(0) per batch
          issue(0, va, ka, kWindow);
          for (uint32_t b = 0;;) {
            const bool more1 = b + kWin < C;
            issue(b + kWin, vb, kb, kWindow);  // past the end: clamped, masked
            consume(va, ka);
            if (!more1) break;
            b += kWin;
            const bool more2 = b + kWin < C;
            issue(b + kWin, va, ka, kWindow);
            consume(vb, kb);
            if (!more2) break;
            b += kWin;
          }
        } else if constexpr (kAbl == 10 || kAbl == 11) {
          // full batches of kPass passes, then an odd last pass on its own
          // (issued before the last full batch is consumed): no empty pass
          const uint32_t npass = (C + 63u) / 64u;
          const uint32_t Cfull = (npass / kPass) * kWin;
          for (uint32_t b = 0; b < Cfull; b += kWin) {
            issue(b, vb, kb, kWindow);
            if (pend) consume(va, ka);
#pragma unroll
            for (int q = 0; q < kPass; ++q) {
              va[q] = vb[q];
              ka[q] = kb[q];
            }
            pend = 1;
          }
          if (Cfull < C) {
            u32x4 v1[1];
            uint32_t k1[1];
            issue(Cfull, v1, k1, kWindow);
            if (pend) consume(va, ka);
            consume(v1, k1);
          } else if (pend) {
            consume(va, ka);
          }
          pend = 0;
        } else {
        for (uint32_t b = 0; b < C; b += kWin) {
          issue(b, vb, kb, kWindow);
          if (pend) consume(va, ka);
#pragma unroll
          for (int q = 0; q < kPass; ++q) {
            va[q] = vb[q];
            ka[q] = kb[q];
          }
          pend = 1;
        }
        if (pend) consume(va, ka);  // drain at the end of the round
        pend = 0;
        }
      };
      if (window)
        run(std::true_type());
      else
        run(std::false_type());
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane < np) {
      const uint32_t p = P0 + (uint32_t)lane;
      const uint32_t odd = fold16(acc[2 * lane + 1]);
      out[p] = finish(acc[2 * lane] + rot8(odd) + (seed ? seed[p] : 0u) + (kAbl && kAbl != 4 && kAbl < 8 ? dummy : 0u), flags);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if constexpr (kAbl == 15) {
      const uint64_t t_end = wall_clock64();
      if (lane == 0 && it < 8) {
        g_ts[3 * ((uint64_t)gw * 8 + it)] = t_begin;
        g_ts[3 * ((uint64_t)gw * 8 + it) + 1] = t_end;
        g_ts[3 * ((uint64_t)gw * 8 + it) + 2] = 1;
      }
    }
    if constexpr (kAbl == 12 || kAbl == 18 || kAbl == 20 || kAbl == 22) {
      // tile timeline (100 MHz constant clock): begin, end, and HW_ID (which
      // CU / SIMD / wave slot) -- vector stores from lane 0
      const uint64_t t_end = wall_clock64();
      if (lane == 0) {
        g_ts[3 * (uint64_t)t] = t_begin;
        g_ts[3 * (uint64_t)t + 1] = t_end;
        g_ts[3 * (uint64_t)t + 2] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
      }
    }
  }
  if constexpr (kAbl == 13) {
    if (lane == 0) {
      const uint32_t d = atomicAdd(&g_q[1], 1u);
      if (d == gridDim.x * kWB - 1) {  // every other wave has taken its last ticket
        atomicExch(&g_q[0], 0u);
        atomicExch(&g_q[1], 0u);
      }
    }
  }
}


// k_chains_pipe with ablations: 1 = no chunk arithmetic / binning (bytes
// xor-ed into a register), 2 = no loads, 3 = chunk sums but no binning.
template <int kAbl, int kPass, int kTile, typename OffT, typename LenT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6))) UINET_CHAINS_OCC void k_pipe_xt(const uint8_t* __restrict__ base,
                                                       const OffT* __restrict__ seg_off,
                                                       const LenT* __restrict__ seg_len,
                                                       const uint32_t* __restrict__ pkt_seg,
                                                       const uint32_t* __restrict__ plen,
                                                       const uint32_t* __restrict__ pskip,
                                                       const uint32_t* __restrict__ seed,
                                                       uint16_t* __restrict__ out, uint32_t n,
                                                       uint32_t flags, uint32_t long_ch) {
  static_assert(kTile >= 1 && kTile <= 32,
                "a tile's packets are one per lane, lane kTile reads the end of its segment "
                "range, and its 2 * kTile bins are one per lane");
  constexpr int kWin = 64 * kPass;  // chunks per batch of passes
  __shared__ MaskLut lut;
  __shared__ unsigned long long lds_acc[kWaves][2 * kTile];  // (slot, rot) bins
  __shared__ uint32_t lds_pkmark[kWaves][64];  // packet-start markers (slot + 1)
  __shared__ uint8_t lds_mark[kWaves][kWin];   // segment-start markers (lane + 1)
  lut.init();
  for (int i = threadIdx.x; i < kWaves * 64; i += blockDim.x) (&lds_pkmark[0][0])[i] = 0;
  for (int i = threadIdx.x; i < kWaves * kWin; i += blockDim.x) (&lds_mark[0][0])[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned long long* acc = lds_acc[wid];
  uint32_t* pkmark = lds_pkmark[wid];
  uint8_t* mark = lds_mark[wid];
  const uint32_t tiles = (n + kTile - 1) / kTile;
  const uint32_t wstride = gridDim.x * kWaves;

  // the pipeline's register sets: the pending batch (issued, not yet
  // consumed; `pend` wave-uniform) in a, the one being issued in b
  u32x4 va[kPass], vb[kPass];
  uint32_t ka[kPass], kb[kPass];
  uint32_t pend = 0;
  uint32_t dummy = 0;
  auto consume = [&](const u32x4 (&v)[kPass], const uint32_t (&key)[kPass]) {
    if constexpr (kAbl == 8) {
      // every pass's chunk sums first, then the passes' scans side by side
      // (independent DPP chains interleave), then the bin updates
      uint32_t P[kPass], sl[kPass], nx[kPass];
#pragma unroll
      for (int q = 0; q < kPass; ++q) P[q] = lut.sum_oc_idx(v[q], key[q] & 0xffffu);
#pragma unroll
      for (int q = 0; q < kPass; ++q) { sl[q] = key[q] >> 16; nx[q] = wave_shl1(sl[q]); }
      wave_scan_n<kPass>(P);
#pragma unroll
      for (int q = 0; q < kPass; ++q) {
        if (lane == 63 || nx[q] != sl[q]) {
          atomicAdd(&acc[sl[q]], (unsigned long long)P[q]);
          if (lane != 63) atomicAdd(&acc[nx[q]], (unsigned long long)(-(long long)P[q]));
        }
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < kPass; ++q) {
      if constexpr (kAbl == 1) { dummy ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w ^ key[q]; continue; }
      const uint32_t w = lut.sum_oc_idx(v[q], key[q] & 0xffffu);  // < 2^17
      if constexpr (kAbl == 3) { dummy += w; continue; }
      const uint32_t sl = key[q] >> 16;
      if constexpr (kAbl == 6) { atomicAdd(&acc[sl], (unsigned long long)w); continue; }
      if constexpr (kAbl == 7) { atomicAdd(reinterpret_cast<uint32_t*>(&acc[sl]), w); continue; }
      const uint32_t P = wave_scan<0, false>(w, 0u);  // < 2^23
      const uint32_t nx = wave_shl1(sl);
      if (lane == 63 || nx != sl) {
        atomicAdd(&acc[sl], (unsigned long long)P);
        if (lane != 63) atomicAdd(&acc[nx], (unsigned long long)(-(long long)P));
      }
    }
  };

  // cross-tile prefetch: tile t+wstride's packet descriptors load at the
  // start of tile t, and its first descriptor round during tile t's last
  // round, so a tile never starts on two dependent global loads
  uint64_t so_next = 0;
  uint32_t l_next = 0;
  auto fetch_s = [&](uint32_t r, uint32_t s1) {
    const uint32_t s = r + (uint32_t)lane;
    const uint32_t sc = s < s1 ? s : s1 - 1;
    so_next = (uint64_t)seg_off[sc];
    l_next = s < s1 ? (uint32_t)seg_len[sc] : 0u;
  };
  uint32_t ps_n = 0, skip_n = 0, len_n = 0;
  auto tile_desc = [&](uint32_t tt) {
    const uint32_t Q0 = tt * kTile;
    const int nq = (int)min((uint32_t)kTile, n - Q0);
    ps_n = pkt_seg[Q0 + (uint32_t)min(lane, nq)];
    skip_n = (lane < nq && pskip) ? pskip[Q0 + lane] : 0u;
    len_n = (lane < nq) ? (plen ? plen[Q0 + lane] : 0xffffffffu) : 0u;
  };
  uint32_t t = blockIdx.x * kWaves + wid;
  if (t < tiles) {
    tile_desc(t);
    const int nq = (int)min((uint32_t)kTile, n - t * kTile);
    const uint32_t s0 = __builtin_amdgcn_readfirstlane(ps_n);
    const uint32_t s1 = __builtin_amdgcn_readlane(ps_n, nq);
    if (s0 < s1) fetch_s(s0, s1);
  }
  for (; t < tiles; t += wstride) {
    const uint32_t P0 = t * kTile;
    const int np = (int)min((uint32_t)kTile, n - P0);
    const uint32_t ps = ps_n;
    const uint32_t k_skip = skip_n;
    const uint32_t k_len = len_n;
    const uint32_t tn = t + wstride;
    if (tn < tiles) tile_desc(tn);
    const uint32_t S0 = __builtin_amdgcn_readfirstlane(ps);
    const uint32_t S1 = __builtin_amdgcn_readlane(ps, np);
    if (lane < 2 * kTile) acc[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t carry_slot1 = 0;  // slot + 1 of the last segment of the previous round
    uint32_t carry_pos = 0;    // chain offset just past that segment
    for (uint32_t r0 = S0; r0 < S1; r0 += 64) {
      // --- descriptor round: one segment per lane -------------------------
      const uint64_t so = so_next;
      const uint32_t l = l_next;
      if (r0 + 64 < S1) {
        fetch_s(r0 + 64, S1);
      } else if (tn < tiles) {
        const int nq = (int)min((uint32_t)kTile, n - tn * kTile);
        const uint32_t s0 = __builtin_amdgcn_readfirstlane(ps_n);
        const uint32_t s1 = __builtin_amdgcn_readlane(ps_n, nq);
        if (s0 < s1) fetch_s(s0, s1);
      }
      const bool pk_in = lane < np && ps >= r0 && ps < r0 + 64;
      if (pk_in) atomicMax(&pkmark[ps - r0], (uint32_t)lane + 1);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const uint32_t pk = pkmark[lane];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (pk_in) pkmark[ps - r0] = 0;
      const uint32_t slot1 = max(wave_scan<1, false>(pk, 0u), carry_slot1);
      const uint32_t slot = slot1 - 1;
      // chain position: T = carry_pos + exclusive prefix of the lengths never
      // decreases along the lanes, so the max-scan of T at packet starts is
      // T at this segment's packet start (0 while the packet of the previous
      // round continues: its position is T itself)
      const uint32_t T = carry_pos + wave_scan<0, false>(l, 0u) - l;
      const uint32_t pos = T - wave_scan<1, false>(pk ? T : 0u, 0u);
      carry_slot1 = __builtin_amdgcn_readlane(slot1, 63);
      carry_pos = __builtin_amdgcn_readlane(pos + l, 63);
      const uint32_t sk = __shfl(k_skip, (int)slot);
      const uint32_t ln = __shfl(k_len, (int)slot);
      const uint32_t lo = sk > pos ? min(sk - pos, l) : 0u;
      const uint32_t hi = ln > pos ? min(ln - pos, l) : 0u;
      const uint32_t eff = hi > lo ? hi - lo : 0u;
      const uint64_t ao = so + lo;
      const uint32_t head = eff ? (uint32_t)(reinterpret_cast<uintptr_t>(base + ao) & 15) : 0u;
      // chunks touched, without forming head + eff (a u32 segment may be 4 GiB)
      const uint32_t nch = eff ? (eff >> 4) + ((head + (eff & 15u) + 15u) >> 4) : 0u;
      const uint64_t c0 = ao - head;
      const uint32_t rot = ((pos + lo - sk) ^ (uint32_t)reinterpret_cast<uintptr_t>(base + ao)) & 1u;
      const uint32_t meta = (slot << 1) | rot;
      const uint32_t c0_lo = (uint32_t)c0, c0_hi = (uint32_t)(c0 >> 32);
      // --- long segments: one wave-wide span each -------------------------
      const bool is_long = nch >= kListMax || (long_ch != 0 && nch >= long_ch);
      for (uint64_t lm = __ballot(is_long); lm; lm &= lm - 1) {
        const int s = (int)__builtin_ctzll(lm);
        // head and length read separately: a segment may hold up to 4 GiB,
        // more than one packed 32-bit word (eff << 4 | head) keeps
        const uint32_t h = __builtin_amdgcn_readlane(head, s);
        const uint32_t el = __builtin_amdgcn_readlane(eff, s);
        const uint32_t mts = __builtin_amdgcn_readlane(meta, s);
        const uint8_t* cb = base + (((uint64_t)__builtin_amdgcn_readlane(c0_hi, s) << 32) |
                                    __builtin_amdgcn_readlane(c0_lo, s));
        const uint32_t nc = __builtin_amdgcn_readlane(nch, s);
        // chunk k keeps bytes [k ? 0 : h, k < nc - 1 ? 16 : last_end): only the
        // first and last chunks are partial, so no byte position is formed
        const uint32_t last_end = ((h + (el & 15u) + 15u) & 15u) + 1u;
        uint64_t lsum = 0;
        for (uint32_t k0 = 0; k0 < nc; k0 += 64 * kLongU) {
          u32x4 v[kLongU];
#pragma unroll
          for (int u = 0; u < kLongU; ++u)
            if (u == 0 || k0 + 64u * u < nc)
              v[u] = load_chunk(cb + 16ull * min(k0 + (uint32_t)(u * 64 + lane), nc - 1));
#pragma unroll
          for (int u = 0; u < kLongU; ++u) {
            if (u == 0 || k0 + 64u * u < nc) {
              const uint32_t k = k0 + (uint32_t)(u * 64 + lane);
              const int lo_b = k == 0 ? (int)h : (k < nc ? 0 : 16);
              const int hi_b = k + 1 < nc ? 16 : (k + 1 == nc ? (int)last_end : 0);
              lsum += lut.sum(v[u], lo_b, hi_b);
            }
          }
        }
        const uint32_t x = __builtin_amdgcn_readlane(wave_scan<0, false>(fold16(lsum), 0u), 63);
        if (lane == 0) atomicAdd(&acc[mts], (unsigned long long)x);
      }
      // --- the round's chunk list -----------------------------------------
      if constexpr (kAbl == 9) { dummy += nch ^ (uint32_t)c0; continue; }
      const uint32_t nch_l = is_long ? 0u : nch;
      const uint32_t ci = wave_scan<0, false>(nch_l, 0u);
      const uint32_t cst = ci - nch_l;
      const uint32_t C = __builtin_amdgcn_readlane(ci, 63);  // < 64 * kListMax
      const uint64_t lm_list = __ballot(nch_l != 0);
      if (lm_list == 0) continue;
      const int lf = (int)__builtin_ctzll(lm_list);
      const uint64_t R0 = ((uint64_t)__builtin_amdgcn_readlane(c0_hi, lf) << 32) |
                          __builtin_amdgcn_readlane(c0_lo, lf);
      const uint64_t rel = c0 - R0 + (1ull << 31);  // R0 - 2 GiB .. R0 + 2 GiB
      const bool window = __ballot(nch_l != 0 && rel >= (1ull << 32) - (1ull << 16)) == 0;
      const uint32_t q0 = head + 16u * cst;  // < 2^20
      const uint32_t recA = q0 | (meta << 20);
      const uint32_t recB = q0 + eff;
      const uint64_t dk = c0 - 16ull * cst;
      const uint32_t dkr = (uint32_t)rel - 16u * cst;  // mod 2^32; + 16 c lands in range
      const __amdgpu_buffer_rsrc_t rsrc = window_rsrc(base + (R0 - (1ull << 31)));
      uint32_t carry_seg1 = 0;  // segment + 1 of the chunk before the batch
      // Issue the batch at list chunk b into (v, key): segment lookup, mask
      // index and bin, loads.  Nothing here waits for packet bytes.
      auto issue = [&](uint32_t b, u32x4 (&v)[kPass], uint32_t (&key)[kPass], auto kWindow) {
        const bool mk = nch_l != 0 && cst >= b && cst < b + kWin;
        if (mk) mark[cst - b] = (uint8_t)(lane + 1);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        uint32_t sc1[kPass];
#pragma unroll
        for (int q = 0; q < kPass; ++q) sc1[q] = mark[q * 64 + lane];
#pragma unroll
        for (int q = 0; q < kPass; ++q) sc1[q] = wave_scan<1, false>(sc1[q], 0u);
#pragma unroll
        for (int q = 0; q < kPass; ++q) {
          const uint32_t last = __builtin_amdgcn_readlane(sc1[q], 63);
          sc1[q] = max(sc1[q], carry_seg1);
          carry_seg1 = max(carry_seg1, last);
        }
#pragma unroll
        for (int q = 0; q < kPass; ++q) {
          const uint32_t c = b + (uint32_t)(q * 64 + lane);
          const bool in = c < C;
          const uint32_t cc = in ? c : C - 1;  // past the end: the last chunk, masked
          const int seg = (int)sc1[q] - 1;
          // cross-lane reads stay outside any condition (a ds_bpermute under
          // a partial exec mask reads 0 from the inactive source lanes)
          const uint32_t a = (uint32_t)__shfl(recA, seg);
          const uint32_t bq = (uint32_t)__shfl(recB, seg);
          const int base16 = 16 * (int)c;
          const int s_lo = (int)(a & 0xfffffu) - base16;
          const int s_hi = in ? (int)bq - base16 : s_lo;
          key[q] = MaskLut::index(s_lo, s_hi) | ((a >> 20) << 16);
          if constexpr (decltype(kWindow)::value) {
            const uint32_t d = (uint32_t)__shfl(dkr, seg);
            if constexpr (kAbl == 2) v[q] = u32x4{d, cc, a, bq}; else
            v[q] = load_chunk_buf(rsrc, d + 16u * cc);
          } else {
            const uint32_t lo32 = (uint32_t)__shfl((uint32_t)dk, seg);
            const uint32_t hi32 = (uint32_t)__shfl((uint32_t)(dk >> 32), seg);
            v[q] = load_chunk(base + ((((uint64_t)hi32 << 32) | lo32) + 16ull * cc));
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (mk) mark[cst - b] = 0;
      };
      auto run = [&](auto kWindow) {
        if constexpr (kAbl == 4) {
          // ping-pong: batch k+1 is issued into the other register set while
          // batch k is consumed; no register copy, so no vmcnt(0) per batch
          issue(0, va, ka, kWindow);
          for (uint32_t b = 0;;) {
            const bool more1 = b + kWin < C;
            issue(b + kWin, vb, kb, kWindow);  // past the end: clamped, masked
            consume(va, ka);
            if (!more1) break;
            b += kWin;
            const bool more2 = b + kWin < C;
            issue(b + kWin, va, ka, kWindow);
            consume(vb, kb);
            if (!more2) break;
            b += kWin;
          }
        } else {
        for (uint32_t b = 0; b < C; b += kWin) {
          issue(b, vb, kb, kWindow);
          if (pend) consume(va, ka);
#pragma unroll
          for (int q = 0; q < kPass; ++q) {
            va[q] = vb[q];
            ka[q] = kb[q];
          }
          pend = 1;
        }
        if (pend) consume(va, ka);  // drain at the end of the round
        pend = 0;
        }
      };
      if (window)
        run(std::true_type());
      else
        run(std::false_type());
    }
    if (S0 >= S1 && tn < tiles) {
      const int nq = (int)min((uint32_t)kTile, n - tn * kTile);
      const uint32_t s0 = __builtin_amdgcn_readfirstlane(ps_n);
      const uint32_t s1 = __builtin_amdgcn_readlane(ps_n, nq);
      if (s0 < s1) fetch_s(s0, s1);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane < np) {
      const uint32_t p = P0 + (uint32_t)lane;
      const uint32_t odd = fold16(acc[2 * lane + 1]);
      out[p] = finish(acc[2 * lane] + rot8(odd) + (seed ? seed[p] : 0u) + (kAbl && kAbl != 4 && kAbl < 8 ? dummy : 0u), flags);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}


}  // namespace lab
}  // namespace uinet

using namespace uinet;

struct Dev {
  uint8_t* arena;
  uint64_t* seg_off;
  uint32_t* seg_len;
  uint32_t* pkt_seg;
  uint32_t* len;
  uint32_t* skip;
  uint32_t n;
  uint64_t bytes;
};

// config 3: lengths uniform over {64, 576, 1500}, each cut into 1..256-B
// pieces, laid out in order with 0..7-B gaps; in_cksum_skip(m, len, 20)
static Dev build_config3(uint32_t n, uint32_t seed) {
  std::mt19937_64 rng(seed);
  const uint32_t choices[3] = {64, 576, 1500};
  std::vector<uint32_t> lens(n);
  std::vector<uint64_t> so;
  std::vector<uint32_t> sl, ps(n + 1);
  uint64_t cursor = 0, bytes = 0;
  for (uint32_t p = 0; p < n; ++p) {
    lens[p] = choices[rng() % 3];
    bytes += lens[p] - 20;
    ps[p] = (uint32_t)sl.size();
    uint32_t left = lens[p];
    while (left) {
      uint32_t piece = std::min<uint32_t>(left, 1 + (uint32_t)(rng() % 256));
      cursor += rng() % 8;
      so.push_back(cursor);
      sl.push_back(piece);
      cursor += piece;
      left -= piece;
    }
  }
  ps[n] = (uint32_t)sl.size();
  const uint64_t arena_bytes = cursor + 64;
  std::vector<uint8_t> host(arena_bytes);
  for (uint64_t i = 0; i + 8 <= arena_bytes; i += 8) {
    uint64_t r = rng();
    memcpy(&host[i], &r, 8);
  }
  std::vector<uint32_t> skip(n, 20);
  Dev d{};
  d.n = n;
  d.bytes = bytes;
  CK(hipMalloc(&d.arena, arena_bytes));
  CK(hipMalloc(&d.seg_off, so.size() * 8));
  CK(hipMalloc(&d.seg_len, sl.size() * 4));
  CK(hipMalloc(&d.pkt_seg, ps.size() * 4));
  CK(hipMalloc(&d.len, n * 4));
  CK(hipMalloc(&d.skip, n * 4));
  CK(hipMemcpy(d.arena, host.data(), arena_bytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(d.seg_off, so.data(), so.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d.seg_len, sl.data(), sl.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d.pkt_seg, ps.data(), ps.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d.len, lens.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d.skip, skip.data(), n * 4, hipMemcpyHostToDevice));
  fprintf(stderr, "config3: %u packets, %zu segments, %llu algorithmic bytes, arena %llu\n", n,
          sl.size(), (unsigned long long)bytes, (unsigned long long)arena_bytes);
  return d;
}

struct Variant {
  std::string name;
  bool exact;  // must equal the shipped kernel's results
  std::function<void(const Dev&, uint16_t*)> run;
};

static int grid_for_tiles(uint32_t n, int tile) {
  const uint32_t tiles = (n + tile - 1) / tile;
  uint64_t blocks = (tiles + kWaves - 1) / kWaves;
  const uint64_t cap = 256ull * 64;
  return (int)std::min<uint64_t>(blocks, cap);
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 0) : (1u << 20);
  const int rounds = argc > 2 ? atoi(argv[2]) : 8;
  const int launches = 20;
  Dev d = build_config3(n, 3);
  if (const char* tl = getenv("LAB_TIMELINE")) {
    // tile timeline of the shipped scheme (kAbl = 12: consume interleaved +
    // timestamps): 10 warm launches, then the raw (begin, end, hw_id) per
    // tile of one launch into the file named by LAB_TIMELINE
    const int tl_grid0 = getenv("LAB_TL_GRID") ? atoi(getenv("LAB_TL_GRID")) : grid_for_tiles(d.n, 32);
    const bool tl_range = getenv("LAB_TL_RANGE") != nullptr;
    const uint32_t tiles = std::max<uint32_t>((d.n + 31) / 32, tl_range ? tl_grid0 * kWaves * 8 : 0);
    unsigned long long* ts;
    CK(hipMalloc(&ts, tiles * 24ull));
    CK(hipMemset(ts, 0, tiles * 24ull));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(lab::g_ts), &ts, sizeof(ts)));
    uint16_t* o;
    CK(hipMalloc(&o, d.n * 2));
    hipEvent_t a0, a1;
    CK(hipEventCreate(&a0));
    CK(hipEventCreate(&a1));
    float ms = 0;
    const int tl_grid = tl_grid0;
    for (int r = 0; r < 11; ++r) {
      CK(hipEventRecord(a0, 0));
      static uint32_t tl_ep = 1000;
      if (getenv("LAB_TL_BP"))
        hipLaunchKernelGGL((lab::k_pipe_abl<22, 2, 32, uint64_t, uint32_t>), dim3(512),
                           dim3(768), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip,
                           nullptr, o, d.n, 0u, ++tl_ep);
      else if (getenv("LAB_TL_POOL"))
        hipLaunchKernelGGL((lab::k_pipe_abl<20, 2, 32, uint64_t, uint32_t>), dim3(tl_grid),
                           dim3(kBlock), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip,
                           nullptr, o, d.n, 0u, 128u);
      else if (getenv("LAB_TL_WPB1"))
        hipLaunchKernelGGL((lab::k_pipe_abl<18, 2, 32, uint64_t, uint32_t>), dim3((d.n + 31) / 32),
                           dim3(64), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip,
                           nullptr, o, d.n, 0u, 128u);
      else if (tl_range)
        hipLaunchKernelGGL((lab::k_pipe_abl<15, 2, 32, uint64_t, uint32_t>), dim3(tl_grid),
                           dim3(kBlock), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip,
                           nullptr, o, d.n, 0u, 128u);
      else
        hipLaunchKernelGGL((lab::k_pipe_abl<12, 2, 32, uint64_t, uint32_t>), dim3(tl_grid),
                           dim3(kBlock), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip,
                           nullptr, o, d.n, 0u, 128u);
      CK(hipEventRecord(a1, 0));
      CK(hipEventSynchronize(a1));
      CK(hipEventElapsedTime(&ms, a0, a1));
    }
    std::vector<unsigned long long> h(tiles * 3ull);
    CK(hipMemcpy(h.data(), ts, tiles * 24ull, hipMemcpyDeviceToHost));
    FILE* f = fopen(tl, "wb");
    if (!f) return 1;
    fwrite(h.data(), 8, h.size(), f);
    fclose(f);
    printf("{\"packets\": %u, \"tiles\": %u, \"grid\": %d, \"last_launch_ms\": %.5f}\n", d.n, tiles,
           tl_grid, ms);
    return 0;
  }
  std::vector<Variant> vs;
  vs.push_back({"pipe<2,32> (shipped)", true, [](const Dev& d, uint16_t* o) {
                  launch_chains(d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip, nullptr,
                                o, d.n, 0, 0, 0);
                }});
  const char* only = getenv("LAB_ONLY");  // substring filter on variant names
  auto want = [&](const char* name) {  // LAB_ONLY: comma-separated substrings
    if (!only) return true;
    std::string l(only);
    for (size_t p = 0, q; p <= l.size(); p = q + 1) {
      q = l.find(',', p);
      if (q == std::string::npos) q = l.size();
      if (q > p && strstr(name, l.substr(p, q - p).c_str())) return true;
    }
    return false;
  };
#define ADD(NAME, EXACT, ...)                                                 \
  if (want(NAME) || !vs.size())                                               \
    vs.push_back({NAME, EXACT, [](const Dev& d, uint16_t* o) { __VA_ARGS__; }});
#define KARGS                                                                   \
  dim3(kBlock), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip, nullptr, o, d.n, \
      0u, 128u
  // lab14: the library's kernel launched directly (build with
  // -DUINET_CHAINS_LAB_NOLOAD for the no-load ablation); the bitmap lookup it
  // was compared with was removed in round 3 (profiles/r03/pruned/)
  ADD("direct", true, hipLaunchKernelGGL((k_chains_pipe<2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  // lab1: one lane per segment
  ADD("lps<2,32>", true, hipLaunchKernelGGL((lab::k_lps<2, 32>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("lps<4,32>", true, hipLaunchKernelGGL((lab::k_lps<4, 32>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("lps<4,8>", true, hipLaunchKernelGGL((lab::k_lps<4, 8>), dim3(grid_for_tiles(d.n, 8)), KARGS))
  ADD("lps<6,32>", true, hipLaunchKernelGGL((lab::k_lps<6, 32>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  // lab2: ablations of the shipped kernel (results deliberately wrong)
  ADD("abl0 copy of pipe", true, hipLaunchKernelGGL((lab::k_pipe_abl<0, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("abl1 no chunk math", false, hipLaunchKernelGGL((lab::k_pipe_abl<1, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("abl2 no loads", false, hipLaunchKernelGGL((lab::k_pipe_abl<2, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("abl3 no binning", false, hipLaunchKernelGGL((lab::k_pipe_abl<3, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  // lab3: real two-batch pipelining (ping-pong register sets, no copy)
  ADD("pingpong P2", true, hipLaunchKernelGGL((lab::k_pipe_abl<4, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("pingpong P1", true, hipLaunchKernelGGL((lab::k_pipe_abl<4, 1, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("pingpong P3", true, hipLaunchKernelGGL((lab::k_pipe_abl<4, 3, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  // lab7: descriptor rounds only (no chunk list, no loads of packet bytes)
  ADD("abl9 descriptor rounds only", false, hipLaunchKernelGGL((lab::k_pipe_abl<9, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  // lab9: tiles of 63 / 16 packets (fewer / more partial descriptor rounds)
  ADD("tile63 consume interleaved", true, hipLaunchKernelGGL((lab::k_pipe_abl<8, 2, 63, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 63)), KARGS))
  ADD("tile48 consume interleaved", true, hipLaunchKernelGGL((lab::k_pipe_abl<8, 2, 48, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 48)), KARGS))
  ADD("tile16 consume interleaved", true, hipLaunchKernelGGL((lab::k_pipe_abl<8, 2, 16, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 16)), KARGS))
  // lab8: no empty pass at a round's end (+ interleaved consume)
  ADD("odd tail pass", true, hipLaunchKernelGGL((lab::k_pipe_abl<10, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("odd tail pass + consume interleaved", true, hipLaunchKernelGGL((lab::k_pipe_abl<11, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  // lab10: tiles from a work queue, resident grids of 6 / 12 / 24 blocks per CU
  ADD("queue bpc6", true, hipLaunchKernelGGL((lab::k_pipe_abl<13, 2, 32, uint64_t, uint32_t>), dim3(256 * 6), KARGS))
  ADD("queue bpc12", true, hipLaunchKernelGGL((lab::k_pipe_abl<13, 2, 32, uint64_t, uint32_t>), dim3(256 * 12), KARGS))
  ADD("queue bpc24", true, hipLaunchKernelGGL((lab::k_pipe_abl<13, 2, 32, uint64_t, uint32_t>), dim3(256 * 24), KARGS))
  ADD("queue bpc6 tile8", true, hipLaunchKernelGGL((lab::k_pipe_abl<13, 2, 8, uint64_t, uint32_t>), dim3(256 * 6), KARGS))
  ADD("range bpc6", true, hipLaunchKernelGGL((lab::k_pipe_abl<14, 2, 32, uint64_t, uint32_t>), dim3(256 * 6), KARGS))
  ADD("range bpc12", true, hipLaunchKernelGGL((lab::k_pipe_abl<14, 2, 32, uint64_t, uint32_t>), dim3(256 * 12), KARGS))
  ADD("range bpc6 tile16", true, hipLaunchKernelGGL((lab::k_pipe_abl<14, 2, 16, uint64_t, uint32_t>), dim3(256 * 6), KARGS))
  // lab11: one / two waves per block (a finished wave's slot is refilled at once)
  ADD("wpb1", true, hipLaunchKernelGGL((lab::k_pipe_abl<16, 2, 32, uint64_t, uint32_t>), dim3((d.n + 31) / 32), dim3(64), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip, nullptr, o, d.n, 0u, 128u))
  ADD("wpb2", true, hipLaunchKernelGGL((lab::k_pipe_abl<17, 2, 32, uint64_t, uint32_t>), dim3((d.n + 63) / 64), dim3(128), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip, nullptr, o, d.n, 0u, 128u))
  // lab12: XCD pools, 70 % static ranges + per-pool tile counters
  ADD("pool bpc6", true, hipLaunchKernelGGL((lab::k_pipe_abl<19, 2, 32, uint64_t, uint32_t>), dim3(256 * 6), KARGS))
  ADD("pool bpc5", true, hipLaunchKernelGGL((lab::k_pipe_abl<19, 2, 32, uint64_t, uint32_t>), dim3(256 * 5), KARGS))
  // lab13: 12-wave blocks, per-block tile ranges and counters, stealing at the end
  ADD("bp12 x512", true, { static uint32_t ep = 0; ++ep; hipLaunchKernelGGL((lab::k_pipe_abl<21, 2, 32, uint64_t, uint32_t>), dim3(512), dim3(768), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip, nullptr, o, d.n, 0u, ep); })
  ADD("bp12 x1024", true, { static uint32_t ep = 0; ++ep; hipLaunchKernelGGL((lab::k_pipe_abl<21, 2, 32, uint64_t, uint32_t>), dim3(1024), dim3(768), 0, 0, d.arena, d.seg_off, d.seg_len, d.pkt_seg, d.len, d.skip, nullptr, o, d.n, 0u, ep); })
  ADD("static bpc6", true, hipLaunchKernelGGL((lab::k_pipe_abl<8, 2, 32, uint64_t, uint32_t>), dim3(256 * 6), KARGS))
  // lab7: consume with the passes' scans interleaved
  ADD("consume interleaved", true, hipLaunchKernelGGL((lab::k_pipe_abl<8, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  // lab6: per-chunk LDS atomics instead of the telescoping scan (u64 / low u32 word)
  ADD("direct atomics u64", true, hipLaunchKernelGGL((lab::k_pipe_abl<6, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("direct atomics u32", false, hipLaunchKernelGGL((lab::k_pipe_abl<7, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  // lab4: G lanes per segment
  ADD("grp<8,2>", true, hipLaunchKernelGGL((lab::k_grp<8, 2, 32>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("grp<4,4>", true, hipLaunchKernelGGL((lab::k_grp<4, 4, 32>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("grp<16,1>", true, hipLaunchKernelGGL((lab::k_grp<16, 1, 32>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("grp<8,1>", true, hipLaunchKernelGGL((lab::k_grp<8, 1, 32>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("grp<4,2>", true, hipLaunchKernelGGL((lab::k_grp<4, 2, 32>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  // lab5: next tile's descriptors prefetched across tiles
  ADD("xtile prefetch", true, hipLaunchKernelGGL((lab::k_pipe_xt<0, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
  ADD("xtile prefetch + pingpong", true, hipLaunchKernelGGL((lab::k_pipe_xt<4, 2, 32, uint64_t, uint32_t>), dim3(grid_for_tiles(d.n, 32)), KARGS))
#undef KARGS
#undef ADD
  std::vector<uint16_t*> outs(vs.size());
  for (auto& o : outs) CK(hipMalloc(&o, d.n * 2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vs.size());
  for (size_t i = 0; i < vs.size(); ++i) {  // warm + results
    CK(hipMemset(outs[i], 0, d.n * 2));
    vs[i].run(d, outs[i]);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  std::vector<uint16_t> ref(d.n), got(d.n);
  CK(hipMemcpy(ref.data(), outs[0], d.n * 2, hipMemcpyDeviceToHost));
  std::vector<long> mism(vs.size(), 0);
  for (size_t i = 1; i < vs.size(); ++i) {
    CK(hipMemcpy(got.data(), outs[i], d.n * 2, hipMemcpyDeviceToHost));
    for (uint32_t p = 0; p < d.n; ++p) mism[i] += got[p] != ref[p];
  }
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      vs[i].run(d, outs[i]);
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < launches; ++k) vs[i].run(d, outs[i]);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[i].push_back(t / launches);
    }
  }
  printf("{\"packets\": %u, \"bytes\": %llu, \"results\": [\n", d.n, (unsigned long long)d.bytes);
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = ms[i];
    std::sort(v.begin(), v.end());
    const float med = v[v.size() / 2];
    printf("%s {\"variant\": \"%s\", \"median_ms\": %.5f, \"min_ms\": %.5f, \"GBps\": %.1f, "
           "\"mismatches\": %ld}\n",
           i ? "," : "", vs[i].name.c_str(), med, v[0], d.bytes / (med * 1e-3) / 1e9, mism[i]);
  }
  printf("]}\n");
  return 0;
}
