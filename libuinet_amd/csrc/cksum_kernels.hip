// MI355X (gfx950) kernels for libuinet's Internet checksum.
//
// What is computed (reference: /root/reference/sys/amd64/amd64/in_cksum.c):
// every byte at logical position p of a packet contributes byte * 256^(p&1)
// to a one's-complement sum that is folded with end-around carry and
// complemented (in_cksum_skip :193-232, in_cksum_pseudo_header :241-276,
// in_cksum_hdr :278-285).  The kernels reproduce it bit for bit:
//
//  * Loads are 16-byte aligned `global_load_dwordx4`s of the chunks that
//    hold at least one byte of a span (an aligned 16-B chunk never crosses a
//    page, so the over-read at a span's head and tail can never fault --
//    the same property in_cksumdata relies on, in_cksum.c:106-115,165-167).
//    Bytes outside the span are masked off in registers.
//  * Each lane sums the 32-bit words of its chunks in a 64-bit register.  A
//    word loaded from an aligned address weights its bytes by 256^(addr&1)
//    modulo 65535, exactly like in_cksumdata; a span whose first byte's
//    address parity differs from its logical parity is byte-rotated once
//    after folding (the "<< 8" of in_cksum.c:222-225).
//  * Folding is always end-around carry, never "% 65535", so an all-zero
//    packet (sum 0 -> 0xffff) stays distinct from a sum of 0xffff (-> 0).
//  * G lanes own one packet (G = 8..64 picked from the mean length); a
//    packet's lanes issue U loads back to back before summing, and the G
//    partial sums meet in a butterfly of cross-lane shuffles.  No LDS and no
//    MFMA: this is an HBM-bound integer fold (~0.25 adds per byte).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cksum_internal.h"

namespace uinet {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t fold16(uint64_t s) {
  uint64_t t = (s & 0xffffffffull) + (s >> 32);  // <= 2^33
  t = (t & 0xffff) + (t >> 16);                  // <= 0x2fffe
  t = (t & 0xffff) + (t >> 16);                  // <= 0x10001
  t = (t & 0xffff) + (t >> 16);                  // <= 0xffff
  return (uint32_t)t;
}

__device__ __forceinline__ uint32_t rot8(uint32_t x) {  // x * 256 mod 65535
  return ((x << 8) | (x >> 8)) & 0xffff;
}

// Mask of bytes [s, e) of a 64-bit little-endian half-chunk; s, e may lie
// outside [0, 8] and are clamped.
__device__ __forceinline__ uint64_t byte_mask64(int s, int e) {
  s = min(max(s, 0), 8);
  e = min(max(e, 0), 8);
  const uint64_t lo = (s >= 8) ? 0ull : (~0ull << (8 * s));
  const uint64_t hi = (e >= 8) ? ~0ull : ~(~0ull << (8 * e));
  return lo & hi;
}

// Sum of the 32-bit words of one 16-byte chunk restricted to bytes [s, e).
__device__ __forceinline__ uint64_t chunk_sum(uint4 v, int s, int e) {
  uint64_t a = ((uint64_t)v.y << 32) | v.x;
  uint64_t b = ((uint64_t)v.w << 32) | v.z;
  a &= byte_mask64(s, e);
  b &= byte_mask64(s - 8, e - 8);
  return (a & 0xffffffffull) + (a >> 32) + (b & 0xffffffffull) + (b >> 32);
}

__device__ __forceinline__ uint4 load16(const uint8_t* p) {
  return *reinterpret_cast<const uint4*>(p);
}

// Per-lane partial sum of the span [a, a + len) over the G lanes of a group.
// Chunk k (relative to the aligned-down start) goes to lane k mod G; lanes
// past the last chunk re-load the last chunk (same cache line, so the load
// coalesces with a live lane's) and mask it away completely.
template <int G, int U>
__device__ __forceinline__ uint64_t span_lane_sum(const uint8_t* a, uint32_t len, int gl) {
  const uintptr_t ua = reinterpret_cast<uintptr_t>(a);
  const uint8_t* c0 = reinterpret_cast<const uint8_t*>(ua & ~uintptr_t(15));
  const int head = (int)(ua & 15);
  const uint32_t nch = (uint32_t)((head + (uint64_t)len + 15) >> 4);
  uint64_t acc = 0;
  if (nch == 0) return 0;
  for (uint32_t k0 = 0; k0 < nch; k0 += G * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k = min(k0 + (uint32_t)(u * G + gl), nch - 1);
      v[u] = load16(c0 + 16ull * k);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = (int64_t)k0 + u * G + gl;
      const int64_t s = (int64_t)head - 16 * k;
      const int64_t e = s + (int64_t)len;
      // Interior chunks (the common case) have s <= 0 and e >= 16; the
      // clamps below turn everything else into exact byte masks.
      acc += chunk_sum(v[u], (int)max<int64_t>(min<int64_t>(s, 16), -16),
                       (int)max<int64_t>(min<int64_t>(e, 32), -16));
    }
  }
  return acc;
}

template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
#pragma unroll
  for (int m = G / 2; m > 0; m >>= 1) x += __shfl_xor(x, m, G);
  return x;
}

__device__ __forceinline__ uint16_t finish(uint64_t s, uint32_t flags) {
  const uint32_t f = fold16(s);
  if (flags & UINET_CKSUM_F_NO_COMPLEMENT) return (uint16_t)f;
  uint16_t r = (uint16_t)(~f & 0xffff);
  if ((flags & UINET_CKSUM_F_UDP) && r == 0) r = 0xffff;  // ip_output.c:962-963
  return r;
}

// ---- one span per packet -------------------------------------------------

template <int G, int U>
__global__ __launch_bounds__(kBlock) void k_spans(const uint8_t* __restrict__ base,
                                                 const uint64_t* __restrict__ off,
                                                 const uint32_t* __restrict__ len,
                                                 const uint32_t* __restrict__ seed,
                                                 const uint8_t* __restrict__ parity,
                                                 uint16_t* __restrict__ out, uint32_t n,
                                                 uint32_t flags) {
  constexpr uint32_t kGroups = kBlock / G;
  const int gl = threadIdx.x & (G - 1);
  const uint32_t stride = gridDim.x * kGroups;
  for (uint32_t p = blockIdx.x * kGroups + threadIdx.x / G; p < n; p += stride) {
    const uint8_t* a = base + off[p];
    const uint64_t acc = span_lane_sum<G, U>(a, len[p], gl);
    uint32_t x = fold16(acc);
    const uint32_t lp = parity ? parity[p] : 0u;
    if ((lp ^ (uint32_t)reinterpret_cast<uintptr_t>(a)) & 1) x = rot8(x);
    x = group_sum<G>(x);
    if (gl == 0) out[p] = finish((uint64_t)x + (seed ? seed[p] : 0u), flags);
  }
}

template <int G, int U>
__global__ __launch_bounds__(kBlock) void k_strided(const uint8_t* __restrict__ base,
                                                   uint64_t pkt_stride, uint32_t len,
                                                   const uint32_t* __restrict__ seed,
                                                   uint16_t* __restrict__ out, uint32_t n,
                                                   uint32_t flags) {
  constexpr uint32_t kGroups = kBlock / G;
  const int gl = threadIdx.x & (G - 1);
  const uint32_t stride = gridDim.x * kGroups;
  for (uint32_t p = blockIdx.x * kGroups + threadIdx.x / G; p < n; p += stride) {
    const uint8_t* a = base + (uint64_t)p * pkt_stride;
    uint32_t x = fold16(span_lane_sum<G, U>(a, len, gl));
    if (reinterpret_cast<uintptr_t>(a) & 1) x = rot8(x);
    x = group_sum<G>(x);
    if (gl == 0) out[p] = finish((uint64_t)x + (seed ? seed[p] : 0u), flags);
  }
}

// ---- chained packets (segment lists) ---------------------------------------
//
// in_cksum_skip(m, len, skip) over a device-resident chain whose mbufs are the
// segments [pkt_seg[p], pkt_seg[p+1]): the chain bytes [skip, len) are summed
// (in_cksum.c:203-229 -- len counts from the chain start, zero-length mbufs
// contribute nothing, a short chain sums what it has), with the logical
// parity counted from `skip`.  len == NULL means "the whole chain",
// skip == NULL means 0.

template <int G, int U>
__global__ __launch_bounds__(kBlock) void k_chains(const uint8_t* __restrict__ base,
                                                  const uint64_t* __restrict__ seg_off,
                                                  const uint32_t* __restrict__ seg_len,
                                                  const uint32_t* __restrict__ pkt_seg,
                                                  const uint32_t* __restrict__ plen,
                                                  const uint32_t* __restrict__ pskip,
                                                  const uint32_t* __restrict__ seed,
                                                  uint16_t* __restrict__ out, uint32_t n,
                                                  uint32_t flags) {
  constexpr uint32_t kGroups = kBlock / G;
  const int gl = threadIdx.x & (G - 1);
  const uint32_t stride = gridDim.x * kGroups;
  for (uint32_t p = blockIdx.x * kGroups + threadIdx.x / G; p < n; p += stride) {
    const uint32_t s0 = pkt_seg[p], s1 = pkt_seg[p + 1];
    const uint64_t lo_want = pskip ? pskip[p] : 0u;
    const uint64_t hi_want = plen ? (uint64_t)plen[p] : ~0ull;
    uint64_t tot = 0;
    uint64_t pos = 0;  // chain offset of segment s
    for (uint32_t s = s0; s < s1 && pos < hi_want; ++s) {
      const uint64_t l = seg_len[s];
      const uint64_t lo = lo_want > pos ? min(lo_want - pos, l) : 0;
      const uint64_t hi = min(hi_want - pos, l);
      if (hi > lo) {
        const uint8_t* a = base + seg_off[s] + lo;
        uint32_t x = fold16(span_lane_sum<G, U>(a, (uint32_t)(hi - lo), gl));
        const uint32_t lpar = (uint32_t)(pos + lo - lo_want);  // logical offset
        if ((lpar ^ (uint32_t)reinterpret_cast<uintptr_t>(a)) & 1) x = rot8(x);
        tot += x;
      }
      pos += l;
    }
    const uint32_t x = group_sum<G>(fold16(tot));
    if (gl == 0) out[p] = finish((uint64_t)x + (seed ? seed[p] : 0u), flags);
  }
}

// ---- geometry ---------------------------------------------------------------

struct Geometry {
  int g, u;
};

// Lanes per packet and loads in flight per lane from the mean packet length:
// aim for one unrolled round per packet with most lanes holding a chunk.
Geometry pick_geometry(uint32_t mean_len) {
  if (mean_len == 0) return {64, 2};
  if (mean_len <= 96) return {8, 1};
  if (mean_len <= 224) return {8, 2};
  if (mean_len <= 720) return {16, 3};
  if (mean_len <= 1520) return {32, 3};
  return {64, 3};
}

int grid_for(uint32_t n, int g) {
  const uint32_t groups_per_block = kBlock / g;
  uint64_t blocks = ((uint64_t)n + groups_per_block - 1) / groups_per_block;
  // Enough blocks to fill 256 CUs at full occupancy, then grid-stride.
  const uint64_t cap = 256ull * 8;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) blocks = 1;
  return (int)blocks;
}

#define UINET_DISPATCH_GEOMETRY(GEO, LAUNCH)          \
  switch ((GEO).g * 16 + (GEO).u) {                   \
    case 8 * 16 + 1: LAUNCH(8, 1); break;             \
    case 8 * 16 + 2: LAUNCH(8, 2); break;             \
    case 16 * 16 + 3: LAUNCH(16, 3); break;           \
    case 32 * 16 + 3: LAUNCH(32, 3); break;           \
    case 64 * 16 + 2: LAUNCH(64, 2); break;           \
    default: LAUNCH(64, 3); break;                    \
  }

}  // namespace

int launch_spans(const void* base, const uint64_t* off, const uint32_t* len,
                 const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                 uint32_t flags, uint32_t len_hint, hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  const Geometry geo = pick_geometry(len_hint);
  const int grid = grid_for(n, geo.g);
#define L(G, U)                                                                   \
  hipLaunchKernelGGL((k_spans<G, U>), dim3(grid), dim3(kBlock), 0, stream,        \
                     static_cast<const uint8_t*>(base), off, len, seed, parity, out, n, flags)
  UINET_DISPATCH_GEOMETRY(geo, L)
#undef L
  return check_launch();
}

int launch_strided(const void* base, uint64_t pkt_stride, uint32_t len, const uint32_t* seed,
                   uint16_t* out, uint32_t n, uint32_t flags, hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  const Geometry geo = pick_geometry(len);
  const int grid = grid_for(n, geo.g);
#define L(G, U)                                                                  \
  hipLaunchKernelGGL((k_strided<G, U>), dim3(grid), dim3(kBlock), 0, stream,     \
                     static_cast<const uint8_t*>(base), pkt_stride, len, seed, out, n, flags)
  UINET_DISPATCH_GEOMETRY(geo, L)
#undef L
  return check_launch();
}

int launch_chains(const void* base, const uint64_t* seg_off, const uint32_t* seg_len,
                  const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                  const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                  uint32_t len_hint, hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  // len_hint is the mean SEGMENT length here: the group walks one segment
  // at a time, so its width follows the segment, not the packet.
  const Geometry geo = pick_geometry(len_hint);
  const int grid = grid_for(n, geo.g);
#define L(G, U)                                                                   \
  hipLaunchKernelGGL((k_chains<G, U>), dim3(grid), dim3(kBlock), 0, stream,       \
                     static_cast<const uint8_t*>(base), seg_off, seg_len, pkt_seg, len, skip,  \
                     seed, out, n, flags)
  UINET_DISPATCH_GEOMETRY(geo, L)
#undef L
  return check_launch();
}

}  // namespace uinet
