// Device-side building blocks shared by the span and chain kernels.
//
// Arithmetic (reference: /root/reference/sys/amd64/amd64/in_cksum.c): every
// byte at logical position p of a packet contributes byte * 256^(p&1) to a
// one's-complement sum folded with end-around carry (REDUCE16, :65-71) and
// complemented.  A 32-bit word loaded from an aligned address weights its
// bytes by 256^(addr&1) modulo 65535, exactly as in_cksumdata (:91-170) does;
// a run of bytes whose address parity differs from its logical parity is
// byte-rotated after folding (the "<< 8" of :222-225).  Folding is always
// end-around carry, never "% 65535", so an all-zero packet (-> 0xffff) stays
// distinct from a sum of 0xffff (-> 0).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cksum_internal.h"

namespace uinet {

constexpr int kBlock = 256;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Blocks per CU of a grid-stride launch (UINET_CKSUM_BLOCKS_PER_CU overrides).
int blocks_per_cu(int dflt);

__device__ __forceinline__ uint32_t fold16(uint64_t s) {
  uint64_t t = (s & 0xffffffffull) + (s >> 32);  // <= 2^33
  t = (t & 0xffff) + (t >> 16);                  // <= 0x2fffe
  t = (t & 0xffff) + (t >> 16);                  // <= 0x10001
  t = (t & 0xffff) + (t >> 16);                  // <= 0xffff
  return (uint32_t)t;
}

// Fold of a value < 2^32.
__device__ __forceinline__ uint32_t fold16_32(uint32_t s) {
  s = (s & 0xffff) + (s >> 16);  // <= 0x1fffe
  s = (s & 0xffff) + (s >> 16);  // <= 0xffff
  return s;
}

__device__ __forceinline__ uint32_t rot8(uint32_t x) {  // x * 256 mod 65535
  return ((x << 8) | (x >> 8)) & 0xffff;
}

__device__ __forceinline__ int clampi(int x, int lo, int hi) { return min(max(x, lo), hi); }

// v_readlane as an unsigned word.  The builtin returns int: OR-ed into the low
// half of a 64-bit value it sign-extends, and a word with bit 31 set turns the
// high half to all ones (a bitmap word whose chunk 31 starts a segment; an
// arena offset of 2 GiB or more).
__device__ __forceinline__ uint32_t readlane_u32(uint32_t x, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, lane);
}
__device__ __forceinline__ uint64_t readlane_u64(uint32_t lo, uint32_t hi, int lane) {
  return ((uint64_t)readlane_u32(hi, lane) << 32) | readlane_u32(lo, lane);
}

// Mask of bytes [s, e) of an 8-byte little-endian half-chunk (s, e clamped).
__device__ __forceinline__ uint64_t byte_mask64(int s, int e) {
  s = clampi(s, 0, 8);
  e = clampi(e, 0, 8);
  const uint64_t lo = (s >= 8) ? 0ull : (~0ull << (8 * s));
  const uint64_t hi = (e >= 8) ? ~0ull : ~(~0ull << (8 * e));
  return lo & hi;
}

// The 16-byte mask keeping bytes [s, e) (s, e in [0, 16]).
__device__ __forceinline__ u32x4 chunk_mask(int s, int e) {
  const uint64_t m0 = byte_mask64(s, e), m1 = byte_mask64(s - 8, e - 8);
  u32x4 m;
  m.x = (uint32_t)m0;
  m.y = (uint32_t)(m0 >> 32);
  m.z = (uint32_t)m1;
  m.w = (uint32_t)(m1 >> 32);
  return m;
}

__device__ __forceinline__ uint64_t masked_sum(u32x4 v, u32x4 m) {
  return (uint64_t)(v.x & m.x) + (v.y & m.y) + (v.z & m.z) + (v.w & m.w);
}

// Sum of the 32-bit words of one 16-byte chunk restricted to bytes [s, e).
__device__ __forceinline__ uint64_t chunk_sum(u32x4 v, int s, int e) {
  return masked_sum(v, chunk_mask(clampi(s, 0, 16), clampi(e, 0, 16)));
}

// Sum of the eight 16-bit halves of a chunk, plus acc: the exact integer sum
// of its bytes weighted 256^(address & 1), one v_dot2_u32_u16 against (1, 1)
// per word.  The words are copied out of the vector before the bit-cast:
// hipcc (ROCm 7.2, gfx950) compiles __builtin_bit_cast(us2, v.y) taken
// straight off an ext-vector ELEMENT as v.x in some contexts (one dword read
// four times; tests/native/dot2_repro.hip reproduces it and
// tests/test_dot2_isa.py checks this helper's code on every build).
__device__ __forceinline__ uint32_t chunk_halves(u32x4 v, uint32_t acc) {
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  const us2 one = {1, 1};
  const uint32_t w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
  acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, w0), one, acc, false);
  acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, w1), one, acc, false);
  acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, w2), one, acc, false);
  return __builtin_amdgcn_udot2(__builtin_bit_cast(us2, w3), one, acc, false);
}
// The same over the bytes a mask keeps.
__device__ __forceinline__ uint32_t chunk_halves_masked(u32x4 v, u32x4 m, uint32_t acc) {
  return chunk_halves(v & m, acc);
}

// 17 x 17 table of chunk masks in LDS: entry s * 17 + e keeps bytes [s, e).
// One ds_read_b128 replaces ~30 VALU instructions of shift/select per chunk.
struct MaskLut {
  u32x4 m[17 * 17];
  __device__ __forceinline__ void init() {
    for (int i = threadIdx.x; i < 17 * 17; i += blockDim.x) m[i] = chunk_mask(i / 17, i % 17);
    __syncthreads();
  }
  __device__ __forceinline__ uint64_t sum(u32x4 v, int s, int e) const {
    return masked_sum(v, m[clampi(s, 0, 16) * 17 + clampi(e, 0, 16)]);
  }
  __device__ static __forceinline__ uint32_t index(int s, int e) {
    return (uint32_t)(clampi(s, 0, 16) * 17 + clampi(e, 0, 16));
  }
  // sum_oc() of a precomputed index()
  __device__ __forceinline__ uint32_t sum_oc_idx(u32x4 v, uint32_t i) const {
    return halves_sum(v, m[i]);
  }
  // The same bytes as the plain sum of the masked 16-bit halves: < 2^19
  // (8 x 0xffff), congruent to sum() mod 65535 (2^16 = 1 mod 65535) and
  // zero only when every kept byte is.
  __device__ __forceinline__ uint32_t sum_oc(u32x4 v, int s, int e) const {
    return halves_sum(v, m[clampi(s, 0, 16) * 17 + clampi(e, 0, 16)]);
  }
  // v_dot2_u32_u16 against (1, 1) adds both halves of a word into the
  // accumulator in one instruction: 4 AND + 4 dot2 per chunk, no carries
  // and no fold (the add-with-carry chain took 4 AND + 4 addc + 3 for the fold).
  __device__ static __forceinline__ uint32_t halves_sum(u32x4 v, u32x4 k) {
    return chunk_halves_masked(v, k, 0u);
  }
};

__device__ __forceinline__ u32x4 load_chunk(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
// kTemporal: an ordinary load (lines stay in L2 for the next reader), else
// load_chunk's non-temporal one.
template <bool kTemporal>
__device__ __forceinline__ u32x4 load_chunk_t(const uint8_t* p) {
  if constexpr (kTemporal) return *reinterpret_cast<const u32x4*>(p);
  return load_chunk(p);
}

// One span [a, a + len) seen by the G lanes of a group, in rounds of G*U
// chunks; chunk k (relative to the 16-B aligned-down start c0) belongs to
// lane k mod G.  In a round's first load, lanes past the last chunk re-load
// the last chunk (the same cache line as a live lane's load) and mask it
// away completely; its later loads are skipped outright there (64-B packets
// +9.6 %, profiles/r01/small/masked_loads/).  An aligned
// 16-B chunk never crosses a page, so the over-read at a span's head and
// tail cannot fault -- the property in_cksumdata relies on (:106-115,165-167).
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
      const uint32_t k = k0 + (uint32_t)(u * G + gl);
      if (u == 0) {
        v[u] = load_chunk(c0 + 16u * min(k, nch - 1));
      } else {
        v[u] = u32x4{0u, 0u, 0u, 0u};
        if (k < nch) v[u] = load_chunk(c0 + 16u * k);
      }
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
  // The same with the LDS mask table and half-word chunk sums: one
  // ds_read_b128 and ~8 VALU per chunk instead of ~25 (each round's sum is
  // < U * 2^19, congruent mod 65535, zero only for zero bytes).
  __device__ __forceinline__ uint32_t sum_lut(const MaskLut& lut, uint32_t k0, int gl) const {
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = 16 * (int)(k0 + (uint32_t)(u * G + gl));
      acc += lut.sum_oc(v[u], head - b, end - b);
    }
    return acc;
  }
  // The first round (k0 = 0) of a packet: rounds u >= 1 are summed only when
  // some lane of the wave holds a chunk there (loads past nch were skipped and
  // left zero), so packets that fit G chunks -- aligned 64-B packets at 4
  // lanes x 2 -- skip that vector work.
  __device__ __forceinline__ uint32_t sum_lut_first(const MaskLut& lut, int gl) const {
    uint32_t acc = lut.sum_oc(v[0], head - 16 * gl, end - 16 * gl);
#pragma unroll
    for (int u = 1; u < U; ++u) {
      const uint32_t k = (uint32_t)(u * G + gl);
      if (__ballot(k < nch)) {  // wave-uniform
        const int b = 16 * (int)k;
        acc += lut.sum_oc(v[u], head - b, end - b);
      }
    }
    return acc;
  }
  __device__ __forceinline__ uint64_t rest_lut(const MaskLut& lut, int gl) {
    uint64_t acc = 0;
    for (uint32_t k0 = G * U; k0 < nch; k0 += G * U) {
      load(k0, gl);
      acc += sum_lut(lut, k0, gl);
    }
    return acc;
  }
};

// Whole-span lane sum (no prefetch interleave).
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

// Inclusive scan over the 64 lanes of a wave with DPP (gfx9 family):
// row_shr:1/2/4/8 inside each 16-lane row, then row_bcast:15 and
// row_bcast:31 across rows -- no LDS round trips.  Op: 0 = add, 1 = max.
// Keyed (add only): a lane takes a partner's partial only if their keys are
// equal, which with keys that never decrease along the lanes is a segmented
// scan.  All 64 lanes must be active.
template <int kOp, bool kKeyed>
__device__ __forceinline__ uint32_t wave_scan(uint32_t x, uint32_t key) {
#define UINET_DPP_STEP(CTRL, RMASK)                                                         \
  {                                                                                         \
    const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, RMASK, 0xf,  \
                                                             true);                         \
    if (kKeyed) {                                                                           \
      const uint32_t ky = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)key, CTRL, RMASK,  \
                                                                0xf, true);                 \
      x += (ky == key) ? y : 0u;                                                            \
    } else if (kOp == 1) {                                                                  \
      x = max(x, y);                                                                        \
    } else {                                                                                \
      x += y;                                                                               \
    }                                                                                       \
  }
  UINET_DPP_STEP(0x111, 0xf)  // row_shr:1
  UINET_DPP_STEP(0x112, 0xf)  // row_shr:2
  UINET_DPP_STEP(0x114, 0xf)  // row_shr:4
  UINET_DPP_STEP(0x118, 0xf)  // row_shr:8
  UINET_DPP_STEP(0x142, 0xa)  // row_bcast:15 -> rows 1, 3
  UINET_DPP_STEP(0x143, 0xc)  // row_bcast:31 -> rows 2, 3
#undef UINET_DPP_STEP
  return x;
}

// kN independent inclusive add-scans over the wave, issued step by step side
// by side so each chain's DPP read-after-write wait fills with the others'
// steps instead of s_nops.  All 64 lanes must be active.
template <int kN>
__device__ __forceinline__ void wave_scan_add_n(uint32_t (&x)[kN]) {
#define UINET_DPP_STEP_N(CTRL, RMASK)                                                     \
  _Pragma("unroll") for (int i = 0; i < kN; ++i) x[i] +=                                 \
      (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x[i], CTRL, RMASK, 0xf, true);
  UINET_DPP_STEP_N(0x111, 0xf)  // row_shr:1
  UINET_DPP_STEP_N(0x112, 0xf)  // row_shr:2
  UINET_DPP_STEP_N(0x114, 0xf)  // row_shr:4
  UINET_DPP_STEP_N(0x118, 0xf)  // row_shr:8
  UINET_DPP_STEP_N(0x142, 0xa)  // row_bcast:15 -> rows 1, 3
  UINET_DPP_STEP_N(0x143, 0xc)  // row_bcast:31 -> rows 2, 3
#undef UINET_DPP_STEP_N
}

// The hardware deals blocks round-robin over the 8 XCDs (block b on XCD
// b % 8), each with its own L2.  With `remap`, block b takes logical id
// (b % 8) * (grid / 8) + b / 8, so an XCD's blocks work on one contiguous band
// of packets (tiles) and the cache line two neighbours share is fetched
// into one L2 instead of two.
__device__ __forceinline__ uint32_t logical_block(uint32_t remap) {
  const uint32_t b = blockIdx.x, per = gridDim.x / 8;
  if (!remap || b >= 8 * per) return b;
  return (b % 8) * per + b / 8;
}

// Lane i gets lane i+1's x (DPP wave_shl:1, a gfx9-family control; lane 63
// gets 0).  Needs all 64 lanes active.
__device__ __forceinline__ uint32_t wave_shl1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, true);
}

}  // namespace uinet
