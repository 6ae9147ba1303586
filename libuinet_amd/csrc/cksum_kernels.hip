// MI355X (gfx950) kernels for libuinet's Internet checksum.
//
// What is computed (reference: /root/reference/sys/amd64/amd64/in_cksum.c):
// every byte at logical position p of a packet contributes byte * 256^(p&1)
// to a one's-complement sum that is folded with end-around carry and
// complemented (in_cksum_skip :193-232, in_cksum_pseudo_header :241-276,
// in_cksum_hdr :278-285).  The kernels reproduce it bit for bit:
//
//  * Loads are 16-byte aligned, non-temporal `global_load_dwordx4`s of the
//    chunks that hold at least one byte of a span (an aligned 16-B chunk
//    never crosses a page, so the over-read at a span's head and tail cannot
//    fault -- the property in_cksumdata relies on, in_cksum.c:106-115,165-167).
//    Bytes outside the span are masked off in registers.
//  * Each lane sums the 32-bit words of its chunks in a 64-bit register.  A
//    word loaded from an aligned address weights its bytes by 256^(addr&1)
//    modulo 65535, exactly like in_cksumdata; a span whose first byte's
//    address parity differs from its logical parity is byte-rotated once
//    after folding (the "<< 8" of in_cksum.c:222-225).
//  * Folding is always end-around carry, never "% 65535", so an all-zero
//    packet (sum 0 -> 0xffff) stays distinct from a sum of 0xffff (-> 0).
//  * G lanes own one packet (G = 8..64 picked from the mean length); a
//    packet's lanes issue U loads back to back, the next packet's
//    descriptors are fetched behind them, and the G partial sums meet in a
//    butterfly of cross-lane shuffles.  No LDS and no MFMA: an HBM-bound
//    integer fold (~0.25 adds per byte).
//
// Index arithmetic is 32-bit (a span is < 2 GiB) and addresses are formed by
// pointer arithmetic only, so every load stays in the global address space.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "cksum_internal.h"

namespace uinet {
namespace {

constexpr int kBlock = 256;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

__device__ __forceinline__ int clampi(int x, int lo, int hi) { return min(max(x, lo), hi); }

// Mask of bytes [s, e) of an 8-byte little-endian half-chunk (s, e clamped).
__device__ __forceinline__ uint64_t byte_mask64(int s, int e) {
  s = clampi(s, 0, 8);
  e = clampi(e, 0, 8);
  const uint64_t lo = (s >= 8) ? 0ull : (~0ull << (8 * s));
  const uint64_t hi = (e >= 8) ? ~0ull : ~(~0ull << (8 * e));
  return lo & hi;
}

// Sum of the 32-bit words of one 16-byte chunk restricted to bytes [s, e).
__device__ __forceinline__ uint64_t chunk_sum(u32x4 v, int s, int e) {
  s = clampi(s, 0, 16);
  e = clampi(e, 0, 16);
  const uint64_t m0 = byte_mask64(s, e);
  const uint64_t m1 = byte_mask64(s - 8, e - 8);
  const uint32_t w0 = v.x & (uint32_t)m0;
  const uint32_t w1 = v.y & (uint32_t)(m0 >> 32);
  const uint32_t w2 = v.z & (uint32_t)m1;
  const uint32_t w3 = v.w & (uint32_t)(m1 >> 32);
  return (uint64_t)w0 + w1 + w2 + w3;
}

__device__ __forceinline__ u32x4 load_chunk(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// One span [a, a + len) seen by the G lanes of a group, in rounds of G*U
// chunks; chunk k (relative to the 16-B aligned-down start c0) belongs to
// lane k mod G.  Lanes past the last chunk re-load the last chunk (the same
// cache line as a live lane's load) and mask it away completely.
template <int G, int U>
struct Span {
  const uint8_t* c0;
  int head;      // a - c0, 0..15
  int end;       // head + len
  uint32_t nch;  // chunks holding at least one byte
  u32x4 v[U];

  __device__ __forceinline__ void init(const uint8_t* a, uint32_t len) {
    head = (int)(reinterpret_cast<uintptr_t>(a) & 15);
    c0 = a - head;
    end = head + (int)len;
    nch = (uint32_t)(end + 15) >> 4;
  }
  __device__ __forceinline__ void load(uint32_t k0, int gl) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k = min(k0 + (uint32_t)(u * G + gl), nch - 1);
      v[u] = load_chunk(c0 + 16u * k);
    }
  }
  __device__ __forceinline__ uint64_t sum(uint32_t k0, int gl) const {
    uint64_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = 16 * (int)(k0 + (uint32_t)(u * G + gl));
      acc += chunk_sum(v[u], head - b, end - b);
    }
    return acc;
  }
  // The rounds after the first (spans longer than G*U chunks).
  __device__ __forceinline__ uint64_t rest(int gl) {
    uint64_t acc = 0;
    for (uint32_t k0 = G * U; k0 < nch; k0 += G * U) {
      load(k0, gl);
      acc += sum(k0, gl);
    }
    return acc;
  }
};

// Whole-span lane sum (no prefetch interleave): used by the chain walker.
template <int G, int U>
__device__ __forceinline__ uint64_t span_lane_sum(const uint8_t* a, uint32_t len, int gl) {
  if (len == 0) return 0;
  Span<G, U> sp;
  sp.init(a, len);
  sp.load(0, gl);
  uint64_t acc = sp.sum(0, gl);
  if (sp.nch > (uint32_t)(G * U)) acc += sp.rest(gl);
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
//
// Software-pipelined over the packets a group owns (p, p + stride, ...): the
// data loads of packet p are issued first, then the descriptors of the next
// packet, so waiting for p's bytes never waits for the prefetch and the
// prefetch latency hides under p's fold.

template <int G, int U, bool kStrided>
__global__ __launch_bounds__(kBlock) void k_spans(const uint8_t* __restrict__ base,
                                                 const uint64_t* __restrict__ off,
                                                 const uint32_t* __restrict__ len,
                                                 const uint32_t* __restrict__ seed,
                                                 const uint8_t* __restrict__ parity,
                                                 uint64_t pkt_stride, uint32_t fixed_len,
                                                 uint16_t* __restrict__ out, uint32_t n,
                                                 uint32_t flags) {
  constexpr uint32_t kGroups = kBlock / G;
  const int gl = threadIdx.x & (G - 1);
  const uint32_t stride = gridDim.x * kGroups;
  uint32_t p = blockIdx.x * kGroups + threadIdx.x / G;
  if (p >= n) return;  // whole groups leave together
  uint64_t o = kStrided ? (uint64_t)p * pkt_stride : off[p];
  uint32_t l = kStrided ? fixed_len : len[p];
  for (;;) {
    const uint8_t* a = base + o;
    Span<G, U> sp;
    sp.init(a, l);
    if (l) sp.load(0, gl);
    // prefetch the next packet's descriptors behind this packet's loads
    const uint32_t pn = p + stride;
    const uint32_t pc = min(pn, n - 1);
    const uint64_t on = kStrided ? (uint64_t)pc * pkt_stride : off[pc];
    const uint32_t ln = kStrided ? fixed_len : len[pc];
    uint64_t acc = l ? sp.sum(0, gl) : 0;
    if (sp.nch > (uint32_t)(G * U)) acc += sp.rest(gl);
    uint32_t x = fold16(acc);
    const uint32_t lp = parity ? parity[p] : 0u;
    if ((lp ^ (uint32_t)reinterpret_cast<uintptr_t>(a)) & 1) x = rot8(x);
    x = group_sum<G>(x);
    if (gl == 0) out[p] = finish((uint64_t)x + (seed ? seed[p] : 0u), flags);
    if (pn >= n) break;
    p = pn;
    o = on;
    l = ln;
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
    const uint32_t lo_want = pskip ? pskip[p] : 0u;
    const uint32_t hi_want = plen ? plen[p] : 0xffffffffu;
    uint64_t tot = 0;
    uint32_t pos = 0;  // chain offset of segment s
    for (uint32_t s = s0; s < s1 && pos < hi_want; ++s) {
      const uint32_t l = seg_len[s];
      const uint32_t lo = lo_want > pos ? min(lo_want - pos, l) : 0u;
      const uint32_t hi = min(hi_want - pos, l);
      if (hi > lo) {
        const uint8_t* a = base + seg_off[s] + lo;
        uint32_t x = fold16(span_lane_sum<G, U>(a, hi - lo, gl));
        const uint32_t lpar = pos + lo - lo_want;  // logical offset of a
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

// Lanes per packet and loads in flight per lane from the mean length: one
// unrolled round per packet with most lanes holding a chunk.
Geometry pick_geometry(uint32_t mean_len) {
  if (mean_len == 0) return {64, 2};
  if (mean_len <= 96) return {8, 1};
  if (mean_len <= 224) return {8, 2};
  if (mean_len <= 720) return {16, 3};
  if (mean_len <= 1520) return {32, 3};
  return {64, 3};
}

// Blocks per CU of the grid-stride launch.  Measured on MI355X (config 2,
// profiles/r01): the span kernel peaks at 64 (8 packets per group -- enough
// rounds for the descriptor prefetch to pay, few enough that the tail is
// short); the strided kernel has no descriptors and prefers one packet per
// group (no cap).  UINET_CKSUM_BLOCKS_PER_CU overrides both.
int blocks_per_cu(int dflt) {
  static int v = [] {
    const char* e = getenv("UINET_CKSUM_BLOCKS_PER_CU");
    const int x = e ? atoi(e) : 0;
    return (x > 0 && x <= 4096) ? x : 0;
  }();
  return v ? v : dflt;
}

int grid_for(uint32_t n, int g, int bpc = 64) {
  const uint32_t groups_per_block = kBlock / g;
  uint64_t blocks = ((uint64_t)n + groups_per_block - 1) / groups_per_block;
  const uint64_t cap = 256ull * (uint64_t)blocks_per_cu(bpc);
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
#define L(G, U)                                                                    \
  hipLaunchKernelGGL((k_spans<G, U, false>), dim3(grid), dim3(kBlock), 0, stream,  \
                     static_cast<const uint8_t*>(base), off, len, seed, parity, 0ull, 0u, out, \
                     n, flags)
  UINET_DISPATCH_GEOMETRY(geo, L)
#undef L
  return check_launch();
}

int launch_strided(const void* base, uint64_t pkt_stride, uint32_t len, const uint32_t* seed,
                   uint16_t* out, uint32_t n, uint32_t flags, hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  const Geometry geo = pick_geometry(len);
  const int grid = grid_for(n, geo.g, 4096);
#define L(G, U)                                                                     \
  hipLaunchKernelGGL((k_spans<G, U, true>), dim3(grid), dim3(kBlock), 0, stream,    \
                     static_cast<const uint8_t*>(base), nullptr, nullptr, seed, nullptr, \
                     pkt_stride, len, out, n, flags)
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
