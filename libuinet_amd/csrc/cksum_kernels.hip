// MI355X (gfx950) span kernels: one contiguous span per packet.
//
//  * G lanes own one packet (G = 8..64 picked from the mean length); each
//    lane issues U 16-byte aligned, non-temporal `global_load_dwordx4`s of the
//    chunks that hold at least one byte of the span, back to back; bytes
//    outside the span are masked off in registers.
//  * Each lane sums 32-bit words in a 64-bit register; the lane sums are
//    folded with end-around carry, byte-rotated once when the span's address
//    parity differs from its logical parity, and meet in a butterfly of
//    cross-lane shuffles (cksum_device.h has the arithmetic and its
//    reference citations).
//  * Software-pipelined over the packets a group owns (p, p + stride, ...):
//    the data loads of packet p are issued first, then the descriptors of the
//    next packet, so waiting for p's bytes never waits for the prefetch and
//    the prefetch latency hides under p's fold.
//  * No LDS and no MFMA: an HBM-bound integer fold (~0.25 adds per byte).
//
// Index arithmetic is 32-bit (a span is < 2 GiB) and addresses are formed by
// pointer arithmetic only, so every load stays in the global address space
// (integer-cast pointers became flat loads and 64-bit min/max went through
// f64 in a first version that ran at 56 % of this one's speed).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "cksum_device.h"

namespace uinet {
namespace {

template <int G, int U, bool kStrided, typename OffT = uint64_t, typename LenT = uint32_t>
__global__ __launch_bounds__(kBlock) void k_spans(const uint8_t* __restrict__ base,
                                                 const OffT* __restrict__ off,
                                                 const LenT* __restrict__ len,
                                                 const uint32_t* __restrict__ seed,
                                                 const uint8_t* __restrict__ parity,
                                                 uint64_t pkt_stride, uint32_t fixed_len,
                                                 uint16_t* __restrict__ out, uint32_t n,
                                                 uint32_t flags, uint32_t remap) {
  constexpr uint32_t kGroups = kBlock / G;
  __shared__ MaskLut lut;
  const int gl = threadIdx.x & (G - 1);
  // round r of the grid covers packets [r S, (r + 1) S), S = the grid's
  // group count (a group's packets lie S apart)
  const uint32_t S = gridDim.x * kGroups;
  const uint32_t stride = S;
  uint32_t p = logical_block(remap) * kGroups + threadIdx.x / G;
  const uint32_t pend = n;
  const bool live = p < pend;
  uint64_t o = 0;
  uint32_t l = 0;
  if (live) {
    o = kStrided ? (uint64_t)p * pkt_stride : (uint64_t)off[p];
    l = kStrided ? fixed_len : (uint32_t)len[p];
  }
  const uint8_t* a = base + o;
  Span<G, U> sp;
  sp.init(a, l);
  if (l) sp.load(0, gl);  // the first packet's bytes are in flight ...
  lut.init();             // ... while the block fills its mask table (every thread
                          // reaches this barrier: no exit before it)
  if (!live) return;      // whole groups leave together
  for (;;) {
    // prefetch the next packet's descriptors behind this packet's loads
    const uint32_t pn = p + stride;
    const uint32_t pc = min(pn, n - 1);
    uint64_t on;
    uint32_t ln;
    on = kStrided ? (uint64_t)pc * pkt_stride : (uint64_t)off[pc];
    ln = kStrided ? fixed_len : (uint32_t)len[pc];
    // a span of one round folds its 32-bit sum (< U * 2^19) directly
    const uint32_t a0 = l ? sp.sum_lut_first(lut, gl) : 0u;
    uint32_t x =
        sp.nch > (uint32_t)(G * U) ? fold16((uint64_t)a0 + sp.rest_lut(lut, gl)) : fold16_32(a0);
    const uint32_t lp = parity ? parity[p] : 0u;
    if ((lp ^ (uint32_t)reinterpret_cast<uintptr_t>(a)) & 1) x = rot8(x);
    x = group_sum<G>(x);
    if (gl == 0) out[p] = finish((uint64_t)x + (seed ? seed[p] : 0u), flags);
    if (pn >= pend) break;
    p = pn;
    o = on;
    l = ln;
    a = base + o;
    sp.init(a, l);
    if (l) sp.load(0, gl);
  }
}

// k_spans_pp (round 2's default: two packets in flight per lane group, 54
// vector instructions per KiB) was removed in round 3: k_spans_lean replaced
// it (profiles/r03/pruned/spans_pp.diff).

struct Geometry {
  int g, u;
};

// Lanes per packet and loads in flight per lane from the mean length: one
// unrolled round per packet with most lanes holding a chunk (1500 B -> 32
// lanes x 3 loads = 96 chunks >= the 95 a 1500-B span can touch).
Geometry pick_geometry(uint32_t mean_len) {
  if (mean_len == 0) return {64, 3};  // unknown: any length, the lean kernel's rounds
  if (mean_len <= 64) return {4, 2};  // 16 packets per wave; an unaligned 64-B span spans 5 chunks
  if (mean_len <= 96) return {8, 1};
  if (mean_len <= 224) return {8, 2};
  if (mean_len <= 720) return {16, 3};
  if (mean_len <= 1520) return {32, 3};
  // 64 lanes x 9 loads: a 9000-B frame in one round, two frames in flight per
  // wave (config 5 +2.6 % over three 3-KB rounds, profiles/r04/r04c5u9/)
  if (mean_len > 6144) return {64, 9};
  return {64, 3};
}

int grid_for(uint32_t n, int g, int bpc) {
  const uint32_t groups_per_block = kBlock / g;
  uint64_t blocks = ((uint64_t)n + groups_per_block - 1) / groups_per_block;
  const uint64_t cap = 256ull * (uint64_t)blocks_per_cu(bpc);
  if (blocks > cap) blocks = cap;
  if (blocks == 0) blocks = 1;
  return (int)blocks;
}

// The geometries k_spans runs (G * 16 + U): 8 and 16 lanes per packet, and 4
// x 2 for the strided form of unaligned small packets.  32 and 64 lanes run
// k_spans_lean and 4 x 1 / 4 x 2 spans k_spans_quad (cksum_spans.hip).  16 x 6
// and 8 x 12 (the 96 chunks of 32 x 3 with twice / four times the bytes in
// flight per lane) needed 82 / 132 VGPRs and ran 2-3 % slower on config 2
// (profiles/r02/ab_geo/), so they are not built; the spans_geo / spans_pipe
// knobs that forced other geometries and a one-shot k_spans at 32 / 64 lanes
// were removed in round 6 (profiles/r06/pruned/).
#define UINET_DISPATCH_GEOMETRY(GEO, LAUNCH)          \
  switch ((GEO).g * 16 + (GEO).u) {                   \
    case 4 * 16 + 2: LAUNCH(4, 2); break;             \
    case 8 * 16 + 1: LAUNCH(8, 1); break;             \
    case 8 * 16 + 2: LAUNCH(8, 2); break;             \
    default: LAUNCH(16, 3); break;                    \
  }

}  // namespace

// Blocks per CU.  Measured on MI355X by interleaved A/B (config 2,
// profiles/r01/ab/): the span kernel peaks at 256 (2 packets per group --
// the second packet's descriptors load under the first one's bytes; one
// packet per group exposes the descriptor latency and loses 9 %); the
// strided kernel has no descriptors and prefers one packet per group (no
// cap).  UINET_CKSUM_BLOCKS_PER_CU overrides every kernel's default.
int blocks_per_cu(int dflt) {
  const int v = tuning().blocks_per_cu;
  return v > 0 ? v : dflt;
}

// The span kernel family by geometry: 4 lanes per packet (mean length <= 64
// B) k_spans_quad; 32 and 64 lanes k_spans_lean (cksum_spans.hip): persistent
// waves, scalar descriptors, mask-free whole chunks -- 23 VALU instructions
// per KiB, no power-ramp dip in the driver's window (profiles/r03/r03d/);
// 8 and 16 lanes k_spans.  Packed descriptors (uinet_cksum_spans32) take the
// same kernels.
template <typename OffT, typename LenT>
static int launch_spans_t(const void* base, const OffT* off, const LenT* len,
                          const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                          uint32_t flags, uint32_t len_hint, hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  const bool host_bytes = (flags & kFlagHostBytes) != 0;
  flags &= ~kFlagHostBytes;
  const Geometry geo = pick_geometry(len_hint);
  if (geo.g == 4)
    return launch_spans_quad(base, off, len, seed, parity, out, n, flags, geo.u, false, 0, 0,
                             blocks_per_cu(128), stream);
  if (geo.g >= 32)
    return launch_spans_lean(base, off, len, seed, parity, out, n, flags, geo.g, geo.u, false, 0,
                             0, tuning().blocks_per_cu, stream, host_bytes);
  const int grid = grid_for(n, geo.g, 256);
#define L(G, U)                                                                          \
  UINET_LAUNCH((k_spans<G, U, false, OffT, LenT>), dim3(grid), dim3(kBlock), 0, stream,  \
               static_cast<const uint8_t*>(base), off, len, seed, parity, 0ull, 0u, out, n,   \
               flags, (uint32_t)tuning().xcd_remap)
  UINET_DISPATCH_GEOMETRY(geo, L)
#undef L
  return check_launch();
}

int launch_spans(const void* base, const uint64_t* off, const uint32_t* len,
                 const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                 uint32_t flags, uint32_t len_hint, hipStream_t stream) {
  return launch_spans_t(base, off, len, seed, parity, out, n, flags, len_hint, stream);
}

int launch_spans32(const void* base, const uint32_t* off, const uint16_t* len,
                   const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                   uint32_t flags, uint32_t len_hint, hipStream_t stream) {
  return launch_spans_t(base, off, len, seed, parity, out, n, flags, len_hint, stream);
}

int launch_strided(const void* base, uint64_t pkt_stride, uint32_t len, const uint32_t* seed,
                   uint16_t* out, uint32_t n, uint32_t flags, hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  Geometry geo = pick_geometry(len);
  // 16-B aligned packets of at most 64 B hold at most 4 chunks: one per lane
  if (len <= 64 && ((reinterpret_cast<uintptr_t>(base) | pkt_stride) & 15) == 0) geo = {4, 1};
  // small packets laid (nearly) back to back and off 16-B alignment: one dense
  // run of chunks per wave, 5 % faster than k_spans<4, 2> on 2su; aligned
  // ones stay on k_spans_quad<1>, 14 % faster than it (profiles/r03/r03s2m/)
  if (len <= 256 && ((reinterpret_cast<uintptr_t>(base) | pkt_stride) & 15) != 0) {
    const int rc = launch_strided_dense(base, pkt_stride, len, seed, out, n, flags,
                                        blocks_per_cu(128), stream);
    if (rc != 1) return rc;
  }
  // k_spans_quad for 16-B aligned packets of <= 64 B (one chunk per lane);
  // unaligned ones run k_spans<4, 2>, 5 % faster there (profiles/r03/r03p/)
  if (geo.g == 4 && geo.u == 1)
    return launch_spans_quad<uint64_t, uint32_t>(base, nullptr, nullptr, seed, nullptr, out, n,
                                                 flags, 1, true, pkt_stride, len,
                                                 blocks_per_cu(128), stream);
  if (geo.g >= 32)
    return launch_spans_lean<uint64_t, uint32_t>(base, nullptr, nullptr, seed, nullptr, out, n,
                                                 flags, geo.g, geo.u, true, pkt_stride, len,
                                                 tuning().blocks_per_cu, stream);
  // one packet per group suits long packets; small ones want groups that
  // loop (64-B packets: 256 per CU 4.88 vs unbounded 3.96 TB/s, profiles/r01/small/)
  const int grid = grid_for(n, geo.g, len <= 96 ? 256 : 4096);
#define L(G, U)                                                                        \
  UINET_LAUNCH((k_spans<G, U, true, uint64_t, uint32_t>), dim3(grid),             \
                     dim3(kBlock), 0, stream,                                          \
                     static_cast<const uint8_t*>(base), nullptr, nullptr, seed, nullptr, \
                     pkt_stride, len, out, n, flags, (uint32_t)tuning().xcd_remap)
  UINET_DISPATCH_GEOMETRY(geo, L)
#undef L
  return check_launch();
}

}  // namespace uinet
