// k_spans_lean: the span kernel for 32 and 64 lanes per packet (packets of
// 0.7 KB and up; config 2's 1500 B, config 4, config 5's 9000 B), and
// k_spans_quad (below) for 4 lanes per packet (small packets).
//
// Same arithmetic as the other span kernels (cksum_device.h; reference
// /root/reference/sys/amd64/amd64/in_cksum.c:91-170,193-232): every byte at
// logical position p adds byte * 256^(p&1), folded with end-around carry.
//
// What it changes is the vector work per byte.  A streaming read that also
// issues ~64 vector instructions per 16-B chunk and lane makes the platform
// throttle 10-20 launches into a burst, one with ~32 does not
// (profiles/r02/cold_ab/ section 4); round 2's k_spans_pp (removed, see
// profiles/r03/pruned/) issued ~42 per KiB, most of them per packet, not per
// byte.  Here every per-packet quantity is
// wave-uniform scalar work and the per-packet vector work is shared:
//
//  * Descriptors.  A wave folds kP = 64 / G packets per step (one per lane
//    group).  Their offsets, lengths, seeds and parity bytes come in by
//    scalar loads, and the scalar unit derives each packet's first aligned
//    chunk, head, end, last chunk, rotation and folded seed.  A lane takes its
//    group's value with one AND and one add (no v_cndmask pairs).
//  * Loads.  The wave's packets are addressed from one scalar base (the
//    lowest first chunk) plus a 32-bit lane offset: `global_load_dwordx4 v,
//    voff, s[base]`, one v_min per slot for the clamp to the last chunk.  A
//    wave whose packets lie 4 GiB apart takes per-lane 64-bit addresses.
//  * Masks.  A chunk slot's mask comes from a 34-entry LDS table (bytes
//    [0, e) and [s, 16), ANDed for the head lane); a slot that every packet
//    of the wave covers whole (slot 1 of a 1500-B packet) skips the table and
//    the ANDs.  The table is copied from a constant image in global memory.
//  * Sums.  Each chunk is 4 v_dot2_u32_u16 against (1, 1) into a 32-bit
//    lane partial (< 2^21 at 3 loads per lane, < 2^23 at 9; no fold before
//    the reduction).
//  * Reduction, two steps at once.  A group's partials of packet A (step k)
//    and packet B (step k + 1) meet in one v_permlane16_swap (G = 32) or
//    v_permlane32_swap + v_permlane16_swap (G = 64), then 4 DPP row_ror adds:
//    each 16-lane row then holds one packet's total, and the fold, the
//    rotation (a shift by 0 or 8 and one more fold), the seed, the complement
//    and the store run once for 2 (G = 64) or 4 (G = 32) packets.
//  * Pipelining: step k + 1's chunks are loaded before step
//    k is summed, every load unconditional, so the wait for step k leaves step
//    k + 1's loads in flight.  Spans longer than one round (16 G U bytes)
//    finish with serial rounds.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "cksum_device.h"

namespace uinet {
namespace {

// The chunk masks as two 17-entry rows, a constant image that a block copies
// into LDS (instead of computing ~30 VALU per entry): entry e keeps bytes
// [0, e) of a 16-byte chunk, entry 17 + s keeps bytes [s, 16); the mask of
// [s, e) is their AND.  A block copies 544 B; the 17 x 17 table of every
// (s, e) cost 4.6 KB per block, and at 512 blocks per CU ~600 MB of L2 reads
// per launch from the same lines (config 2 3.8 % slower, profiles/r03/r03s/).
struct alignas(16) SplitWords {
  uint32_t w[34 * 4];
};
constexpr SplitWords make_split_words() {
  SplitWords t{};
  for (int i = 0; i < 34; ++i)
    for (int d = 0; d < 4; ++d) {
      uint32_t m = 0;
      for (int b = 0; b < 4; ++b) {
        const int byte = 4 * d + b;
        if (i < 17 ? byte < i : byte >= i - 17) m |= 0xffu << (8 * b);
      }
      t.w[i * 4 + d] = m;
    }
  return t;
}
__device__ const SplitWords g_split_words = make_split_words();

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
// A compiler-only memory barrier placed right after a batch of loads: the
// loads stay where they are issued.  Without it the compiler sinks a step's
// loads past the previous step's sum whenever that sum branches (k_spans_quad's
// ballots) or loops (k_spans_lean at 64 lanes: spans longer than one round),
// which drains the pipeline there.  No instruction is emitted and no wait:
// the barrier names no registers.
__device__ __forceinline__ void issued() { asm volatile("" ::: "memory"); }
// A wave-uniform value the compiler may not reason about (keeps 32-bit
// compares of a 64-bit value's halves from being merged back into a 64-bit
// compare, which only the vector ALU has).
__device__ __forceinline__ uint32_t opaque_s(uint32_t x) {
  asm volatile("" : "+s"(x));
  return x;
}

// Scalar (SMEM) loads: through the constant address space a uniform load of
// memory the kernel never writes becomes an s_load.
__device__ __forceinline__ uint64_t sld64(const uint64_t* p) {
  const uint64_t v = *(const __attribute__((address_space(4))) uint64_t*)(uintptr_t)p;
  return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v);
}
__device__ __forceinline__ uint32_t sld32(const uint32_t* p) {
  return rfl(*(const __attribute__((address_space(4))) uint32_t*)(uintptr_t)p);
}
// The aligned dword that holds the byte at p (never crosses a page); the
// byte is (word >> 8 * (p & 3)) & 0xff.
__device__ __forceinline__ uint32_t sld8w(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  return sld32(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3));
}
// Span descriptors by scalar loads, wide (u64 offset, u32 length:
// uinet_cksum_spans) or packed (u32 offset, u16 length: uinet_cksum_spans32).
// A u16 length comes from the aligned dword that holds it.
__device__ __forceinline__ uint64_t sld_off(const uint64_t* p) { return sld64(p); }
__device__ __forceinline__ uint64_t sld_off(const uint32_t* p) { return sld32(p); }
__device__ __forceinline__ uint32_t sld_len(const uint32_t* p) { return sld32(p); }
__device__ __forceinline__ uint32_t sld_len(const uint16_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  return (sld32(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3)) >> (8 * (a & 2))) & 0xffffu;
}

// Four dot2 against (1, 1): both 16-bit halves of every word added into acc
// (cksum_device.h: the words are copied out before the bit-cast).
__device__ __forceinline__ uint32_t dot_acc(u32x4 v, uint32_t acc) { return chunk_halves(v, acc); }
__device__ __forceinline__ uint32_t dot_acc_masked(u32x4 v, u32x4 m, uint32_t acc) {
  return chunk_halves_masked(v, m, acc);
}

// x + the value of row_ror:n (lanes rotate by n inside each 16-lane row).
template <int kN>
__device__ __forceinline__ uint32_t add_ror(uint32_t x) {
  return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x120 + kN, 0xf, 0xf, false);
}

// One step of a wave: the raw descriptors of its kP packets (one per lane
// group) as its scalar loads return them, in SGPRs.
template <int kP>
struct Step {
  uint64_t o[kP];   // span offsets from `base`
  uint32_t l[kP];   // lengths
  uint32_t sd[kP];  // raw seeds
  uint32_t lp[kP];  // the aligned dword holding the parity byte, and its shift
  uint32_t q0;      // the step's first packet
};
// What a step's sum needs, derived when it is loaded: head (span start inside
// its first chunk) and end (head + len) per packet; whether the pair lies too
// far apart for 32-bit lane offsets from one scalar base; the rotation bits
// (address parity != logical parity, in_cksum.c:222-225) placed at the
// reduction rows of an A step (G = 32: rows 0 / 2; G = 64: rows 0, 1); the
// folded seeds (the in_cksum_pseudo_header sum, in_cksum.c:241-276).
template <int kP>
struct Geo {
  uint32_t h[kP], e[kP];
  bool far;
  uint32_t rot;     // Step::rot
  uint32_t sd[kP];  // Step::sd
};

// kTemporal: ordinary packet-byte loads (the host-resident span path: over
// PCIe a line two packets share is then read once, from L2, 3 % faster),
// else non-temporal (HBM: 12 % faster; profiles/r06/r06labt/).
template <int G, int kU, bool kParity, bool kSeed, bool kStrided, typename OffT, typename LenT,
          bool kTemporal = false>
__global__ __launch_bounds__(kBlock) void k_spans_lean(
    const uint8_t* __restrict__ base, const OffT* __restrict__ off,
    const LenT* __restrict__ len, const uint32_t* __restrict__ seed,
    const uint8_t* __restrict__ parity, uint16_t* __restrict__ out, uint32_t n, uint32_t flags,
    uint32_t remap, uint64_t stride, uint32_t slen) {
  static_assert(G == 32 || G == 64, "one or two packets per wave");
  static_assert(kU == 3 || (G == 64 && kU == 9), "chunk loads per lane and round: 3, or 9 at 64 "
                                                 "lanes (a 9000-B frame in one round)");
  constexpr int kP = 64 / G;
  constexpr uint32_t kGroups = kBlock / G;
  constexpr uint32_t kRound = 16u * G * kU;  // bytes of a span one round covers
  constexpr uint32_t kBias = 0x80000000u;    // lane offsets are biased: pairs may lie either way
  // The split mask table (g_split_words): T[e] keeps bytes [0, e), T[17 + s]
  // bytes [s, 16).  The 17 x 17 table it replaced cost 4 % on config 2 at
  // 512 blocks per CU: every block copied 4.6 KB from the same L2 lines
  // (profiles/r03/r03s/).
  __shared__ u32x4 lut_m[34];
  // the table entry at byte address a (= 16 x entry index)
  auto lut_at = [&](uint32_t a) -> u32x4 {
    return *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(lut_m) + a);
  };
  // bytes [s, e) of a chunk, s and e clamped to [0, 16]
  auto mask_se = [&](int s_, int e_) -> u32x4 {
    return lut_m[clampi(e_, 0, 16)] & lut_m[17 + clampi(s_, 0, 16)];
  };

  const uint32_t lane = threadIdx.x & 63;
  const uint32_t gl = lane & (G - 1);
  const uint32_t pos0 = 16u * gl;             // byte of this lane's slot-0 chunk in its span
  const uint32_t negpos16 = 0u - 16u * pos0;  // the same in mask-table units, negated
  const uint32_t m0 = gl == 0 ? ~0u : 0u;     // the lane that holds a span's head chunk
  // ~0 in the lanes of group 1 (kP = 2): a lane's value of a per-packet
  // quantity is a0 + ((a1 - a0) & gmask).  Opaque, so that the compiler keeps
  // one AND and one add instead of a v_mov / v_mov / v_cndmask select.
  uint32_t gmask = (kP == 2 && lane >= 32) ? ~0u : 0u;
  asm volatile("" : "+v"(gmask));
  auto gsel = [&](const uint32_t (&a)[kP]) -> uint32_t {
    if constexpr (kP == 1) return a[0];
    else return a[0] + ((a[1] - a[0]) & gmask);
  };

  const uint32_t boff = (uint32_t)(reinterpret_cast<uintptr_t>(base) & 15);
  const uint8_t* base_m = base - kBias;  // a step's loads: base_m + o[0] + (biased) lane offset
  // packets per grid step; the host keeps n + 3 S below 2^32
  const uint32_t S = gridDim.x * kGroups;
  const uint32_t wave = rfl(threadIdx.x) / 64;
  uint32_t q = logical_block(remap) * kGroups + wave * kP;  // the wave's first packet (even)

  // Per 16-lane row r after the reduction: which packet of the pair, as an
  // offset from the step's first packet.  G = 32: rows are (A g0, B g0, A g1,
  // B g1); G = 64: (A, A, B, B).
  const uint32_t row = lane >> 4;
  const uint32_t row_b = kP == 2 ? (row & 1) : (row >> 1);  // 1 = packet B (step k + 1)
  const uint32_t row_g = kP == 2 ? (row >> 1) : 0;          // lane group
  const uint32_t row_sh8 = 8 * row;                         // this row's byte in rr
  const uint32_t row_q = row_g + (row_b ? S : 0u);          // its packet - the step's first
  const bool store_lane = kP == 2 ? (lane & 15) == 0 : (lane & 31) == 0;
  // the results as a buffer resource of 2 n bytes (n < 2^31)
  const __amdgpu_buffer_rsrc_t out_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(2u * n), 0x00020000);

  // Descriptors of the step at q0 (< n; q0 even when kP = 2): scalar loads
  // only, no dependent arithmetic and no branch (the second packet's index is
  // clamped to the batch), so issuing them never waits for them; everything
  // derived from them is computed where the step is loaded.
  auto desc = [&](uint32_t q0) {
    Step<kP> s;
#pragma unroll
    for (int g = 0; g < kP; ++g) {
      const uint32_t qg = min(q0 + (uint32_t)g, n - 1);
      if constexpr (kStrided) {
        s.o[g] = (uint64_t)qg * stride;
        s.l[g] = slen;
      } else {
        s.o[g] = sld_off(off + qg);
        s.l[g] = sld_len(len + qg);
      }
      s.sd[g] = kSeed ? sld32(seed + qg) : 0u;
      s.lp[g] = kParity ? sld8w(parity + qg) : 0u;
    }
    s.q0 = q0;
    return s;
  };

  // Where a step's chunks are: one scalar base for the wave, and per packet
  // its first chunk d and last chunk lo as biased 32-bit offsets from it.  A
  // far pair (offsets 1 GiB or more apart, or a span of 1 GiB or more) loads
  // packet 0's chunks in both groups; far_sum folds it again.
  struct Addr {
    const uint8_t* sb;
    uint32_t d[kP], lo[kP];
  };
  // Past-the-end packets get length 0; an empty span borrows its neighbour's
  // offset (or 0), so that its re-read chunk is one the wave reads anyway and
  // its own (unread) offset is never dereferenced.
  auto norm = [&](Step<kP> s) {
#pragma unroll
    for (int g = 0; g < kP; ++g)
      if (s.q0 + (uint32_t)g >= n) s.l[g] = 0;
    if constexpr (kP == 2) {
      if (!s.l[0]) s.o[0] = s.l[1] ? s.o[1] : 0;
      if (!s.l[1]) s.o[1] = s.o[0];
    } else {
      if (!s.l[0]) s.o[0] = 0;
    }
    return s;
  };
  auto addr = [&](const Step<kP>& s0, Geo<kP>& z) {
    Addr w;
    uint32_t b[kP];
#pragma unroll
    for (int g = 0; g < kP; ++g) {
      const uint32_t qg = s0.q0 + (uint32_t)g;
      const uint32_t lp =
          kParity
              ? (s0.lp[g] >> (8u * (((uint32_t)reinterpret_cast<uintptr_t>(parity) + qg) & 3u))) & 1u
              : 0u;
      b[g] = (lp ^ boff ^ (uint32_t)s0.o[g]) & 1u;
      z.sd[g] = kSeed && qg < n ? fold16_32(s0.sd[g]) : 0u;
    }
    z.rot = kP == 2 ? (b[0] | (b[kP - 1] << 2)) : b[0] * 3u;
    const Step<kP> s = norm(s0);
    uint32_t lastb[kP];
#pragma unroll
    for (int g = 0; g < kP; ++g) {
      z.h[g] = ((uint32_t)s.o[g] + boff) & 15u;
      z.e[g] = z.h[g] + s.l[g];
      lastb[g] = (max(z.e[g], 1u) - 1u) & ~15u;  // 16 x the last chunk (0 when empty)
      w.d[g] = kBias - z.h[g];
    }
    w.sb = base_m + s.o[0];
    z.far = false;
    if constexpr (kP == 2) {
      const uint64_t df = s.o[1] - s.o[0];
      const uint32_t dlo = (uint32_t)df, dhi = opaque_s((uint32_t)(df >> 32));
      z.far = dhi != (uint32_t)((int32_t)dlo >> 31) || dlo + 0x40000000u >= kBias ||
              (lastb[0] | lastb[1]) >= 0x40000000u;
      w.d[1] += dlo;
      if (z.far) {
        w.d[1] = w.d[0];
        lastb[1] = lastb[0];
      }
    }
#pragma unroll
    for (int g = 0; g < kP; ++g) w.lo[g] = w.d[g] + lastb[g];
    return w;
  };
  // Chunk slot u of round r (byte rb = r * kRound of the span): lane offsets
  // pos0 + rb + 16 u G from the packet's first chunk, clamped to its last.
  auto load_round = [&](const Addr& w, uint32_t rb, u32x4 (&v)[kU]) {
    const uint32_t b = gsel(w.d) + pos0 + rb, l = gsel(w.lo);
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = load_chunk_t<kTemporal>(w.sb + min(b + 16u * u * G, l));
  };
  auto load_step = [&](const Step<kP>& s, u32x4 (&v)[kU]) {
    Geo<kP> z;
    load_round(addr(s, z), 0, v);
    issued();
    return z;
  };

  // A far step's lane partial, every round with per-lane 64-bit addresses.
  auto far_sum = [&](uint32_t q0, const Geo<kP>& z) -> uint32_t {
    const Step<kP> s = norm(desc(q0));
    uint32_t chi[kP], clo[kP], lb[kP], emax = 0;
#pragma unroll
    for (int g = 0; g < kP; ++g) {
      const uint64_t c0 = s.o[g] - z.h[g];
      chi[g] = (uint32_t)(c0 >> 32);
      clo[g] = (uint32_t)c0;
      lb[g] = (max(z.e[g], 1u) - 1u) & ~15u;
      emax = max(emax, z.e[g]);
    }
    const uint8_t* pb = base + (((uint64_t)gsel(chi) << 32) | gsel(clo));
    const uint32_t l = gsel(lb), e0 = gsel(z.e) - pos0, h0 = gsel(z.h) - pos0;
    uint32_t acc = 0;
    for (uint32_t rb = 0; rb < emax; rb += kRound) {  // wave-uniform
      u32x4 w[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u)
        w[u] = load_chunk_t<kTemporal>(pb + min(pos0 + rb + 16u * u * G, l));
      uint32_t r = 0;
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const uint32_t k = rb + 16u * u * G;
        r = dot_acc_masked(w[u], mask_se((int)(h0 - k), (int)(e0 - k)), r);
      }
      acc = fold16_32(acc) + r;
    }
    return acc;
  };

  // The lane partial of one step: round 0 from registers, later rounds
  // (spans longer than kRound) serially.  Mask-table addresses are 16 x the
  // entry index: 16 x clamp(end - chunk start, 0, 16), and for the head lane
  // 272 + 16 x head.
  auto sum_step = [&](uint32_t q0, const Geo<kP>& z, const u32x4 (&v)[kU]) -> uint32_t {
    if (z.far) return far_sum(q0, z);  // wave-uniform, rare
    uint32_t E[kP], H[kP], emin = z.e[0], emax = z.e[0];
#pragma unroll
    for (int g = 0; g < kP; ++g) {
      E[g] = 16u * min(z.e[g], 1u << 20);  // round 0 cannot tell 2^20 from more
      H[g] = 16u * z.h[g];
      emin = min(emin, z.e[g]);
      emax = max(emax, z.e[g]);
    }
    const uint32_t e16 = gsel(E) + negpos16;
    // head lane: T[e] & T[17 + h]; the others: T[e] & T[17] (all ones)
    const u32x4 m = lut_at(clampi((int)e16, 0, 256)) & lut_at(272u + (gsel(H) & m0));
    uint32_t acc = dot_acc_masked(v[0], m, 0u);
#pragma unroll
    for (int u = 1; u < kU; ++u) {
      if (emin >= 16u * (u + 1) * G)  // wave-uniform: every lane's chunk is whole
        acc = dot_acc(v[u], acc);
      else
        acc = dot_acc_masked(v[u], lut_at(clampi((int)(e16 - 256u * u * G), 0, 256)), acc);
    }
    if (emax > kRound) {  // wave-uniform
      Geo<kP> z2;
      const Addr w = addr(desc(q0), z2);
      const uint32_t e0 = gsel(z.e) - pos0;
      auto round_sum = [&](const u32x4 (&x)[kU], uint32_t rb) {
        uint32_t r = 0;
#pragma unroll
        for (int u = 0; u < kU; ++u)
          r = dot_acc_masked(x[u], lut_m[clampi((int)(e0 - rb - 16u * u * G), 0, 16)], r);
        acc = fold16_32(acc) + r;  // < 2^23: 64 lanes of it still fit 32 bits
      };
      if constexpr (kP == 1 && kU <= 3) {
        // one packet per wave, 3-KB rounds (spans of 1.5-6 KB mean length, or
        // of unknown length; 9000-B frames take kU = 9, one round).  Rounds 1
        // and 2 are straight-line code with both rounds' loads issued before
        // the first sum (a span of one round more re-reads its last chunk in
        // round 2, masked away); spans longer than three rounds finish
        // serially.  (The ping-pong loop this replaces ran its rounds
        // serially: the compiler waited for all loads where the loop's paths
        // met, draining the pipeline at every round.)
        u32x4 x[kU], y[kU];
        load_round(w, kRound, x);
        load_round(w, 2 * kRound, y);
        issued();
        round_sum(x, kRound);
        round_sum(y, 2 * kRound);
        for (uint32_t rb = 3 * kRound; rb < emax; rb += kRound) {
          load_round(w, rb, x);
          round_sum(x, rb);
        }
      } else {  // two packets per wave, or 9-KB rounds: one round at a time
        for (uint32_t rb = kRound; rb < emax; rb += kRound) {
          u32x4 x[kU];
          load_round(w, rb, x);
          round_sum(x, rb);
        }
      }
    }
    return acc;
  };

  // Packets A (step at q0) and B (step at q0 + S): reduce, fold, rotate, seed,
  // complement and store, once for the 2 * kP packets.
  auto finish = [&](uint32_t xA, uint32_t xB, const Geo<kP>& sA, const Geo<kP>& sB,
                    uint32_t q0) {
    uint32_t t;
    if constexpr (kP == 2) {
      const auto r = __builtin_amdgcn_permlane16_swap(xA, xB, false, false);
      t = r[0] + r[1];  // rows: A g0, B g0, A g1, B g1 (16-lane partials)
    } else {
      const auto r = __builtin_amdgcn_permlane32_swap(xA, xB, false, false);
      const uint32_t h = r[0] + r[1];  // lanes 0-31: A, 32-63: B
      const auto r2 = __builtin_amdgcn_permlane16_swap(h, h, false, false);
      t = r2[0] + r2[1];  // rows: A, A, B, B
    }
    t = add_ror<8>(t);
    t = add_ror<4>(t);
    t = add_ror<2>(t);
    t = add_ror<1>(t);  // every lane: its row's total (< 2^27; < 2^29 at kU = 9)
    // row r rotates by 8 when bit r of rowrot is set: rr = 8 in byte r
    const uint32_t rowrot = sA.rot | (sB.rot << (kP == 2 ? 1 : 2));
    const uint32_t rr = ((rowrot * 0x00204081u) & 0x01010101u) << 3;
    uint32_t x = fold16_32(t);
    x = fold16_32(x << __builtin_amdgcn_ubfe(rr, row_sh8, 8));  // x * 256^rot mod 65535
    if constexpr (kSeed) {
      if constexpr (kP == 2) {
        const uint32_t ss0 = sA.sd[0] | (sB.sd[0] << 16);  // rows 0, 1
        const uint32_t ss1 = sA.sd[1] | (sB.sd[1] << 16);  // rows 2, 3
        x = fold16_32(x + __builtin_amdgcn_ubfe(row_g ? ss1 : ss0, 16 * row_b, 16));
      } else {
        x = fold16_32(x + __builtin_amdgcn_ubfe(sA.sd[0] | (sB.sd[0] << 16), 16 * row_b, 16));
      }
    }
    uint32_t res = x;
    if (!(flags & UINET_CKSUM_F_NO_COMPLEMENT)) {
      res = ~x & 0xffffu;
      if ((flags & UINET_CKSUM_F_UDP) && res == 0) res = 0xffff;  // ip_output.c:962-963
    }
    // no branch around the store (a divergent branch here made the whole
    // loop's descriptors divergent): lanes that do not store address past
    // the end of the buffer resource, and the hardware drops the write
    const uint32_t qr = q0 + row_q;
    const uint32_t ob = store_lane && qr < n ? 2u * qr : 0xfffffff0u;
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)res, out_rsrc, (int)ob, 0, 0);
  };

  // Steps run two at a time, A and B; the next A's chunks are loaded while B
  // is summed.  The wave knows how many of its steps are live (K), so the
  // loop body has no exit (an exit that shared code with it made the compiler
  // wait for the loads in flight) and no step past the end is ever loaded:
  // the last one or two steps run after the loop.  Descriptors are fetched
  // two steps ahead (clamped to the batch: a clamped fetch is never loaded).
  const uint32_t qmax = (n - 1) & ~(uint32_t)(kP - 1);  // the last step start
  u32x4 vA[kU], vB[kU];
  Geo<kP> zA;
  // The block's mask table: its words are loaded first (L2 hits), then the
  // first step's chunks, and the table is written to LDS while those are in
  // flight (the wait before the writes covers only the table's loads).
  const uint32_t li = min(threadIdx.x, 33u);
  const u32x4 lw0 = reinterpret_cast<const u32x4*>(g_split_words.w)[li];
  zA = load_step(desc(min(q, qmax)), vA);
  lut_m[li] = lw0;  // unconditional: threads past the table rewrite its last entry
  __syncthreads();  // every thread reaches this barrier: no exit before it
  if (q >= n) return;  // wave-uniform
  const uint32_t K = (n - q + S - 1) / S;  // live steps of this wave, >= 1
  Step<kP> sB = desc(min(q + S, qmax));
  uint32_t k = 0;
  for (; k + 2 < K; k += 2) {  // steps k, k + 1 and k + 2 are live
    const Geo<kP> zB = load_step(sB, vB);  // step k + 1 in flight while step k is summed
    const Step<kP> sC = desc(q + 2 * S);
    const uint32_t xA = sum_step(q, zA, vA);
    const Geo<kP> zC = load_step(sC, vA);  // step k + 2 in flight while k + 1 is summed
    sB = desc(min(q + 3 * S, qmax));
    finish(xA, sum_step(q + S, zB, vB), zA, zB, q);
    zA = zC;
    q += 2 * S;
  }
  if (k + 1 < K) {  // two live steps left
    const Geo<kP> zB = load_step(sB, vB);
    const uint32_t xA = sum_step(q, zA, vA);
    finish(xA, sum_step(q + S, zB, vB), zA, zB, q);
  } else {  // one
    finish(sum_step(q, zA, vA), 0u, zA, zA, q);
  }
}

// k_spans_quad: 4 lanes per packet, for small packets (mean length <= 64 B:
// config 2s shapes).  Round 2 found 64-B packets bound by per-packet vector
// work (~110 VALU instructions per KiB in k_spans<4, 2>, and a wait for all
// loads in flight once per packet: profiles/r02/ab_small/); one lane per
// packet (round 3) made every chunk load touch 64 lines and ran 70 % slower
// (profiles/r03/r03e/ab_span_c2s.log).  Here a wave folds 16 packets per step
// with the pipeline of k_spans_lean:
//  * descriptors come per super-step of 64 packets (4 steps): one coalesced
//    vector load per array, one lane per packet, issued a whole super-step
//    before its first step; a step's quads take their packet's words with
//    ds_bpermute.  (Per-step descriptor loads, issued one step ahead, chained
//    each step's chunk loads to a descriptor round trip.)
//  * a lane's chunk slots are chunks gl and 4 + gl (64-bit addresses,
//    clamped to the packet's last chunk).  Slot 1 is loaded only when some
//    span of the step reaches past 64 B: unconditional, its redundant loads
//    made aligned 64-B packets 13-23 % slower (profiles/r03/r03o/, r03p/).  A
//    slot that every lane holds whole skips the mask table, one that every
//    lane holds empty skips the sum (ballots);
//  * step k + 1's chunks are loaded before step k is summed;
//  * a step with a span longer than one round (ragged batches) is marked and
//    redone whole at the end of its super-step, where few registers are live;
//  * a packet's 4 lane partials meet in 2 DPP quad_perm adds, and the fold,
//    rotation, seed and complement run branch-free in every lane; lane i
//    collects packet i's result of the super-step (one ds_bpermute per step)
//    and the 64 results leave in one 128-B store (through a buffer resource:
//    lanes past the batch address past its end).
template <int U, bool kParity, bool kSeed, bool kStrided, typename OffT, typename LenT>
__global__ __launch_bounds__(kBlock) void k_spans_quad(
    const uint8_t* __restrict__ base, const OffT* __restrict__ off,
    const LenT* __restrict__ len, const uint32_t* __restrict__ seed,
    const uint8_t* __restrict__ parity, uint16_t* __restrict__ out, uint32_t n, uint32_t flags,
    uint32_t remap, uint64_t stride, uint32_t slen) {
  constexpr uint32_t kRoundB = 64u * U;  // bytes of a span one round covers
  constexpr uint32_t kWavesPB = kBlock / 64;
  __shared__ u32x4 lut_m[34];  // the split mask table (see k_spans_lean)
  auto mask_se = [&](int s_, int e_) -> u32x4 {
    return lut_m[clampi(e_, 0, 16)] & lut_m[17 + clampi(s_, 0, 16)];
  };
  const uint32_t lane = threadIdx.x & 63, gi = lane >> 2, gl = lane & 3;
  const __amdgpu_buffer_rsrc_t out_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(2u * n), 0x00020000);

  // A super-step's raw descriptors, lane i = packet p0 + i (index clamped to
  // the batch: loads only, no branch).
  struct B {
    uint32_t olo, ohi, l, sd, lp;
  };
  auto blk = [&](uint32_t p0) {
    B d{};
    if constexpr (!kStrided) {
      const uint32_t qc = min(p0 + lane, n - 1);
      const uint64_t o = (uint64_t)off[qc];
      d.olo = (uint32_t)o;
      d.ohi = (uint32_t)(o >> 32);
      d.l = (uint32_t)len[qc];
      d.sd = kSeed ? seed[qc] : 0u;
      d.lp = kParity ? parity[qc] : 0u;
    } else {
      d.sd = kSeed ? seed[min(p0 + lane, n - 1)] : 0u;
    }
    return d;
  };
  // what a step's sum needs: first aligned chunk, head, end (head + len), 16 x
  // last chunk, rotation (address parity != logical parity), folded seed
  struct Z {
    const uint8_t* c0;
    uint32_t h, e, lb, rot, sd;
  };
  // step j of the super-step at p0 (its packets p0 + 16 j .. + 15)
  auto geo = [&](const B& d, uint32_t p0, uint32_t j) {
    const int src = (int)(16u * j + gi);
    const uint32_t q = p0 + 16u * j + gi;
    uint64_t o;
    uint32_t l, lp = 0, sd = 0;
    if constexpr (kStrided) {
      o = (uint64_t)min(q, n - 1) * stride;
      l = slen;
    } else {
      o = ((uint64_t)(uint32_t)__shfl((int)d.ohi, src) << 32) | (uint32_t)__shfl((int)d.olo, src);
      l = (uint32_t)__shfl((int)d.l, src);
      if constexpr (kParity) lp = (uint32_t)__shfl((int)d.lp, src);
    }
    if constexpr (kSeed) sd = (uint32_t)__shfl((int)d.sd, src);
    Z z;
    l = q < n ? l : 0u;
    // an empty span re-reads the arena's first chunk: its own offset is never
    // dereferenced
    const uint8_t* a = base + (l ? o : 0ull);
    const uint32_t alo = (uint32_t)reinterpret_cast<uintptr_t>(a);
    z.h = alo & 15u;
    z.c0 = a - z.h;
    z.e = z.h + l;
    z.lb = (max(z.e, 1u) - 1u) & ~15u;
    z.rot = (lp ^ alo) & 1u;  // in_cksum.c:222-225
    z.sd = kSeed ? fold16_32(sd) : 0u;
    return z;
  };
  // issued() keeps the loads where they are: with no store before their use,
  // the compiler otherwise sinks them below the previous step's sum (its
  // ballot branches), and the pipeline is gone.
  auto load = [&](const Z& z, u32x4 (&v)[U]) {
    v[0] = load_chunk(z.c0 + min(16u * gl, z.lb));
    // slot 1 only when some span of the step reaches past 64 B (wave-uniform):
    // aligned 64-B packets never need it
    if constexpr (U == 2)
      if (__ballot(z.e > 64u)) v[1] = load_chunk(z.c0 + min(16u * (4u + gl), z.lb));
    issued();
  };
  // Round 0 of a step from registers.  A step with a span longer than one
  // round (ragged batches) is marked pending and redone whole at the end of
  // its super-step (`redo`): inlined at every step, that path's registers
  // were the kernel's count (84 VGPRs against 70 without it).
  auto sum = [&](const Z& z, const u32x4 (&v)[U], uint32_t j, uint32_t& pend) -> uint32_t {
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cb = (int)(16u * (4u * u + gl));
      const int s = (int)z.h - cb, e = (int)z.e - cb;
      if (__ballot(!(s <= 0 && e >= 16)) == 0)  // wave-uniform: every chunk whole
        acc = dot_acc(v[u], acc);
      else if (__ballot(e > 0) != 0)  // some lane holds bytes of this slot
        acc = dot_acc_masked(v[u], mask_se(s, e), acc);
    }
    if (__ballot(z.e > kRoundB)) pend |= 1u << j;  // wave-uniform
    return acc;
  };
  // A pending step's whole sum, one chunk per lane per 64-B round.
  auto full_sum = [&](const Z& y) -> uint32_t {
    uint32_t acc = 0;
#pragma unroll 1
    for (uint32_t rb = 0; __ballot(rb < y.e); rb += 64u) {
      const uint32_t cb = rb + 16u * gl;
      const u32x4 w = load_chunk(y.c0 + min(cb, y.lb));
      acc = fold16_32(acc) +
            dot_acc_masked(w, mask_se((int)(y.h - cb), (int)(y.e - cb)), 0u);
    }
    return acc;
  };
  // Step j's results: reduce, fold, rotate, seed, complement in every lane,
  // then lane 16 j + i takes packet i's result (quad i) into `res`; `flush`
  // stores a super-step's 64 results with one coalesced 128-B store.
  uint32_t res = 0;
  auto finish = [&](uint32_t x, const Z& z, uint32_t j) {
    // quad_perm [1,0,3,2] then [2,3,0,1]: every lane holds its packet's total
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xb1, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4e, 0xf, 0xf, false);
    x = fold16_32(x);
    x = fold16_32(x << (8u * z.rot));  // x * 256^rot mod 65535
    if constexpr (kSeed) x = fold16_32(x + z.sd);
    uint32_t r = x;
    if (!(flags & UINET_CKSUM_F_NO_COMPLEMENT)) {
      r = ~x & 0xffffu;
      if ((flags & UINET_CKSUM_F_UDP) && r == 0) r = 0xffff;  // ip_output.c:962-963
    }
    r = (uint32_t)__shfl((int)r, (int)(4u * (lane & 15u)));
    res = (lane >> 4) == j ? r : res;
  };
  // the pending steps of the super-step at p0 (block c), redone whole
  auto redo = [&](const B& c, uint32_t p0, uint32_t pend) {
#pragma unroll 1
    for (uint32_t j = 0; j < 4; ++j)
      if (pend & (1u << j)) {
        const Z y = geo(c, p0, j);
        finish(full_sum(y), y, j);
      }
  };
  // lanes past the batch address past the end of the buffer resource: the
  // hardware drops their writes
  auto flush = [&](uint32_t p0) {
    const uint32_t q = p0 + lane;
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)res, out_rsrc,
                                          (int)(q < n ? 2u * q : 0xfffffff0u), 0, 0);
  };

  // the mask table: its words first (L2 hits), then the first step
  const u32x4 lw0 = reinterpret_cast<const u32x4*>(g_split_words.w)[min(threadIdx.x, 33u)];
  // super-steps of 64 packets; wave w takes super-steps w, w + NW, ... (the
  // host keeps n + 2 S below 2^32)
  const uint32_t NW = gridDim.x * kWavesPB;
  const uint32_t S = 64u * NW;
  const uint32_t w0 = logical_block(remap) * kWavesPB + rfl(threadIdx.x) / 64;
  uint32_t p = 64u * w0;
  u32x4 vA[U], vB[U];
  Z zA, zB;
  // two descriptor blocks, ping-pong: a block is reloaded only after its last
  // use, so no loaded value is ever copied (a copy of the block loaded last
  // made the compiler wait for every load in flight once per super-step)
  B b0 = blk(min(p, n - 1));
  B b1 = blk(min(p + S, n - 1));
  zA = geo(b0, p, 0);
  load(zA, vA);
  // unconditional (threads past the table rewrite its last entry with the
  // same word): under a branch the compiler sinks the load into it and waits
  // for every load in flight, the first step's chunks included
  lut_m[min(threadIdx.x, 33u)] = lw0;
  __syncthreads();  // every thread reaches this barrier: no exit before it
  if (p >= n) return;  // wave-uniform
  // The four steps of a full super-step at p (step 0 in flight in A), the
  // next super-step's step 0 (block nx) issued under the last sum.
  auto super = [&](const B& c, const B& nx) {
    uint32_t pend = 0;
    zB = geo(c, p, 1);
    load(zB, vB);  // step 1 in flight while step 0 is summed
    finish(sum(zA, vA, 0, pend), zA, 0);
    zA = geo(c, p, 2);
    load(zA, vA);
    finish(sum(zB, vB, 1, pend), zB, 1);
    zB = geo(c, p, 3);
    load(zB, vB);
    finish(sum(zA, vA, 2, pend), zA, 2);
    zA = geo(nx, p + S, 0);
    load(zA, vA);
    finish(sum(zB, vB, 3, pend), zB, 3);
    if (pend) redo(c, p, pend);  // wave-uniform, rare
    flush(p);
    p += S;
  };
  // The last super-step: J live steps (1..4), step 0 in flight in A.
  auto last = [&](const B& c) {
    uint32_t pend = 0;
    const uint32_t J = min((n - p + 15u) / 16u, 4u);
    if (J == 1) {
      finish(sum(zA, vA, 0, pend), zA, 0);
    } else {
      zB = geo(c, p, 1);
      load(zB, vB);
      finish(sum(zA, vA, 0, pend), zA, 0);
      if (J == 2) {
        finish(sum(zB, vB, 1, pend), zB, 1);
      } else {
        zA = geo(c, p, 2);
        load(zA, vA);
        finish(sum(zB, vB, 1, pend), zB, 1);
        if (J == 3) {
          finish(sum(zA, vA, 2, pend), zA, 2);
        } else {
          zB = geo(c, p, 3);
          load(zB, vB);
          finish(sum(zA, vA, 2, pend), zA, 2);
          finish(sum(zB, vB, 3, pend), zB, 3);
        }
      }
    }
    if (pend) redo(c, p, pend);
    flush(p);
  };
  // live super-steps of this wave (>= 1); all but the last have 4 live steps
  const uint32_t K4 = (n - p + S - 1) / S;
  uint32_t i = 0;
  for (; i + 2 < K4; i += 2) {  // super-steps i, i + 1 full, i + 2 live
    super(b0, b1);
    b0 = blk(min(p + S, n - 1));  // super-step i + 2
    super(b1, b0);
    b1 = blk(min(p + S, n - 1));  // super-step i + 3
  }
  if (i + 1 < K4) {  // two live super-steps left
    super(b0, b1);
    last(b1);
  } else {
    last(b0);
  }
}

// k_strided_dense: the strided API for small packets laid (nearly) back to
// back -- 32 <= stride <= 256 and stride - len <= stride / 4, e.g. 64-B
// packets at stride 64 -- off 16-B alignment (launch_strided: aligned ones
// run k_spans_quad<1>, 14 % faster on 2s; this kernel is 5 % faster than
// k_spans<4, 2> on 2su, profiles/r03/r03s2m/).  Instead of lanes per packet
// (k_spans_quad / k_spans, where a packet off 16-B alignment touches one
// chunk more than its 4 and the 4-lane geometry loads a second slot for it),
// a wave reads the arena as one dense run of aligned 16-B chunks, one per
// lane (one 1-KiB load instruction per step), and splits each chunk between
// the two packet slots it can straddle:
//   * a step covers K = floor(1008 / stride) slots; a lane's chunk starts r
//     bytes into the step (r >= -15), in slot j = floor(r / stride) (a
//     multiply by ceil(2^20 / stride), exact for r < 1024);
//   * part A = the bytes of slot j's packet in the chunk, part B = those of
//     slot j + 1 (nonzero only in the chunk that holds the boundary), each
//     one ds_read_b128 from the 17 x 17 mask table and 4 v_dot2;
//   * B moves to the next lane (DPP wave_shr:1), which is always in slot
//     j + 1 (stride >= 32), so lane sums are per slot; a wave prefix sum and
//     one LDS word per run end give every packet its sum as a difference;
//   * lane j folds packet j's sum, rotates it when the packet starts at an
//     odd address (in_cksum.c:222-225), adds its seed and stores it (one
//     coalesced store per step).
// The chunks end at the step's last packet's last byte, so only bytes between
// packets are read beyond what the packets hold (the gaps, <= 1/4).
struct alignas(16) Mask17 {
  uint32_t w[17 * 17 * 4];
};
constexpr Mask17 make_mask17() {
  Mask17 t{};
  for (int i = 0; i < 17 * 17; ++i)
    for (int d = 0; d < 4; ++d) {
      uint32_t m = 0;
      for (int b = 0; b < 4; ++b) {
        const int byte = 4 * d + b;
        if (byte >= i / 17 && byte < i % 17) m |= 0xffu << (8 * b);
      }
      t.w[i * 4 + d] = m;
    }
  return t;
}
__device__ const Mask17 g_mask17 = make_mask17();

template <bool kSeed>
__global__ __launch_bounds__(kBlock) void k_strided_dense(
    const uint8_t* __restrict__ base, const uint32_t* __restrict__ seed,
    uint16_t* __restrict__ out, uint32_t n, uint32_t flags, uint32_t stride, uint32_t slen,
    uint32_t kpk, uint32_t recip) {
  constexpr uint32_t kWavesPB = kBlock / 64;
  __shared__ u32x4 lut[17 * 17];
  __shared__ uint32_t lds_ends[kWavesPB][33];  // per wave: prefix sum at each run end
  {
    const u32x4* img = reinterpret_cast<const u32x4*>(g_mask17.w);
    const uint32_t i1 = 256u + min((uint32_t)threadIdx.x, 17u * 17u - 257u);
    const u32x4 m0 = img[threadIdx.x], m1 = img[i1];
    lut[threadIdx.x] = m0;
    lut[i1] = m1;  // threads past the table rewrite its last entry
    __syncthreads();
  }
  const uint32_t lane = threadIdx.x & 63;
  uint32_t* ends = lds_ends[threadIdx.x >> 6];
  const uint32_t steps = (n + kpk - 1) / kpk;
  const uint32_t W = gridDim.x * kWavesPB;
  const uint64_t ab = reinterpret_cast<uintptr_t>(base);
  // a step's chunk: slot 0's first byte B0, the first aligned chunk c0, the
  // chunk count (to the last packet's last byte, <= 64) and this lane's load
  struct St {
    uint64_t B0, c0;
    uint32_t p0, K, nch;
  };
  auto geo = [&](uint32_t k) {
    St t;
    t.p0 = k * kpk;
    t.K = min(kpk, n - t.p0);
    t.B0 = ab + (uint64_t)t.p0 * stride;
    t.c0 = t.B0 & ~15ull;
    t.nch = (uint32_t)((t.B0 + (uint64_t)(t.K - 1) * stride + slen + 15u - t.c0) >> 4);
    return t;
  };
  auto load = [&](const St& t) {
    return load_chunk(reinterpret_cast<const uint8_t*>(t.c0 + 16ull * min(lane, t.nch - 1u)));
  };
  // Step k's sum, its chunk v already loaded.
  auto step = [&](const St& t, const u32x4& v) {
    const uint32_t p0 = t.p0, K = t.K, nch = t.nch;
    const uint64_t B0 = t.B0, c0 = t.c0;
    const bool valid = lane < nch;
    const int r = (int)(c0 - B0) + 16 * (int)lane;
    const int j = r < 0 ? -1 : (int)(((uint32_t)r * recip) >> 20);
    const int sa = j * (int)stride - r;  // slot j's first byte in the chunk (<= 0)
    const int ea = j >= 0 ? sa + (int)slen : 0;
    const int sb = sa + (int)stride;
    const int eb = j + 1 < (int)K ? sb + (int)slen : sb;
    const uint32_t ia = valid ? (uint32_t)(clampi(sa, 0, 16) * 17 + clampi(ea, 0, 16)) : 0u;
    const uint32_t ib = valid ? (uint32_t)(clampi(sb, 0, 16) * 17 + clampi(eb, 0, 16)) : 0u;
    const uint32_t suma = dot_acc_masked(v, lut[ia], 0u);
    const uint32_t sumb = dot_acc_masked(v, lut[ib], 0u);
    // lane i + 1 takes lane i's part B (wave_shr:1; lane 0 gets 0)
    const uint32_t w =
        suma + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sumb, 0x138, 0xf, 0xf, false);
    const uint32_t P = wave_scan<0, false>(w, 0u);  // < 64 * 2^20
    const uint32_t key = valid ? (uint32_t)(j + 1) : 0xffffu;
    const uint32_t nkey = wave_shl1(key);
    if (lane == 0) ends[0] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (valid && (lane == 63 || nkey != key)) ends[key] = P;  // run end of slot j
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane < K) {
      const uint32_t q = p0 + lane;
      uint32_t x = fold16_32(ends[lane + 1] - ends[lane]);
      if ((((uint32_t)B0 + lane * stride) & 1u) != 0) x = fold16_32(x << 8);  // odd start
      if constexpr (kSeed) x = fold16_32(x + fold16_32(seed[q]));
      uint32_t res = x;
      if (!(flags & UINET_CKSUM_F_NO_COMPLEMENT)) {
        res = ~x & 0xffffu;
        if ((flags & UINET_CKSUM_F_UDP) && res == 0) res = 0xffff;  // ip_output.c:962-963
      }
      out[q] = (uint16_t)res;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  };
  // Steps k, k + W, ... in two register sets: step k + W's chunk is loaded
  // before step k is summed (its index clamped to the last step: a clamped
  // load is never summed), so every load is unconditional and the wait for
  // step k leaves step k + W in flight.
  uint32_t k = blockIdx.x * kWavesPB + rfl(threadIdx.x) / 64;
  if (k >= steps) return;  // wave-uniform, after the block's only barrier
  St ta = geo(k);
  u32x4 va = load(ta);
  for (;;) {
    const St tb = geo(min(k + W, steps - 1));
    const u32x4 vb = load(tb);
    asm volatile("" ::: "memory");
    step(ta, va);
    k += W;
    if (k >= steps) break;
    ta = geo(min(k + W, steps - 1));
    va = load(ta);
    asm volatile("" ::: "memory");
    step(tb, vb);
    k += W;
    if (k >= steps) break;
  }
}

}  // namespace

template <typename OffT, typename LenT>
int launch_spans_quad(const void* base, const OffT* off, const LenT* len,
                      const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                      uint32_t flags, int u, bool strided, uint64_t stride, uint32_t slen,
                      int blocks_cu, hipStream_t stream) {
  constexpr uint32_t kPerBlock = 64u * (kBlock / 64);  // packets per block super-step
  uint64_t blocks = ((uint64_t)n + kPerBlock - 1) / kPerBlock;
  // the kernel's 32-bit packet indices need n + 2 * blocks * kPerBlock < 2^32
  const uint64_t cap = std::min<uint64_t>(256ull * (uint64_t)blocks_cu, (1ull << 26) / kPerBlock);
  blocks = std::max<uint64_t>(1, std::min(blocks, cap));
  const dim3 grid((uint32_t)blocks), blk(kBlock);
  const uint8_t* b = static_cast<const uint8_t*>(base);
  const uint32_t remap = (uint32_t)tuning().xcd_remap;
  constexpr bool kWide = sizeof(OffT) == 8;
#define UINET_QUAD(U, P, SD, ST)                                                             \
  UINET_LAUNCH((k_spans_quad<U, P, SD, ST, OffT, LenT>), grid, blk, 0, stream, b, off, \
                     len, seed, parity, out, n, flags, remap, stride, slen)
#define UINET_QUAD_U(U)                                          \
  if (strided) { /* wide descriptors only: none are read */     \
    if constexpr (kWide) {                                       \
      if (seed) UINET_QUAD(U, false, true, true);                \
      else UINET_QUAD(U, false, false, true);                    \
    }                                                            \
  } else if (parity) {                                           \
    if (seed) UINET_QUAD(U, true, true, false);                  \
    else UINET_QUAD(U, true, false, false);                      \
  } else {                                                       \
    if (seed) UINET_QUAD(U, false, true, false);                 \
    else UINET_QUAD(U, false, false, false);                     \
  }
  if (u == 1) {
    UINET_QUAD_U(1)
  } else {
    UINET_QUAD_U(2)
  }
#undef UINET_QUAD_U
#undef UINET_QUAD
  return check_launch();
}

template <typename OffT, typename LenT>
int launch_spans_lean(const void* base, const OffT* off, const LenT* len,
                      const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                      uint32_t flags, int g, int u, bool strided, uint64_t stride,
                      uint32_t slen, int blocks_cu, hipStream_t stream, bool temporal) {
  const uint32_t groups = kBlock / g;
  // Two steps per wave by default at 32 lanes per packet (2 x 1500 B each):
  // config 2 at 2 steps (256 blocks per CU) is flat through the driver's
  // window and within 4 % of the widest grid warm; 4 steps lost 3-4 % warm
  // (configs 2 and 4), 1 step ramps after an idle gap (profiles/r03/r03t/,
  // r03z/).  At 64 lanes a step is one packet of >= 1.5 KB (9 KB in config
  // 5, where 2 steps per wave lost 1.2 %): one step per wave.  blocks_cu > 0
  // (the knob) caps the grid at blocks_cu per CU instead.
  const uint64_t spw = g == 32 ? 2 : 1;  // steps per wave
  uint64_t blocks = ((uint64_t)n + spw * groups - 1) / (spw * groups);
  const uint64_t lim = blocks_cu > 0 ? 256ull * (uint64_t)blocks_cu : 256ull * 4096ull;
  // the kernel's 32-bit packet indices need n + 3 * blocks * groups < 2^32
  const uint64_t cap = std::min<uint64_t>(lim, (1ull << 26) / groups);
  if (blocks_cu > 0) blocks = ((uint64_t)n + groups - 1) / groups;
  blocks = std::max<uint64_t>(1, std::min(blocks, cap));
  const dim3 grid((uint32_t)blocks), blk(kBlock);
  const uint8_t* b = static_cast<const uint8_t*>(base);
  const uint32_t remap = (uint32_t)tuning().xcd_remap;
  constexpr bool kWide = sizeof(OffT) == 8;
#define UINET_LEAN(G, U, P, SD, ST)                                                   \
  UINET_LAUNCH((k_spans_lean<G, U, P, SD, ST, OffT, LenT>), grid, blk, 0, stream, b, off, \
               len, seed, parity, out, n, flags, remap, stride, slen)
#define UINET_LEAN_T(G, U, SD)                                                              \
  UINET_LAUNCH((k_spans_lean<G, U, false, SD, false, OffT, LenT, true>), grid, blk, 0, stream, \
               b, off, len, seed, parity, out, n, flags, remap, stride, slen)
#define UINET_LEAN_G(G, U)                                       \
  if (temporal && !strided && !parity) {                         \
    if (seed) UINET_LEAN_T(G, U, true);                          \
    else UINET_LEAN_T(G, U, false);                              \
  } else if (strided) { /* wide descriptors only: none are read */ \
    if constexpr (kWide) {                                       \
      if (seed) UINET_LEAN(G, U, false, true, true);             \
      else UINET_LEAN(G, U, false, false, true);                 \
    }                                                            \
  } else if (parity) {                                           \
    if (seed) UINET_LEAN(G, U, true, true, false);               \
    else UINET_LEAN(G, U, true, false, false);                   \
  } else {                                                       \
    if (seed) UINET_LEAN(G, U, false, true, false);              \
    else UINET_LEAN(G, U, false, false, false);                  \
  }
  if (g == 32) {
    UINET_LEAN_G(32, 3)
  } else if (u == 9) {
    UINET_LEAN_G(64, 9)
  } else {
    UINET_LEAN_G(64, 3)
  }
#undef UINET_LEAN_G
#undef UINET_LEAN_T
#undef UINET_LEAN
  return check_launch();
}

// The dense strided kernel when the shape fits (see k_strided_dense), else
// returns 1 and the caller picks another kernel.
int launch_strided_dense(const void* base, uint64_t stride, uint32_t len, const uint32_t* seed,
                         uint16_t* out, uint32_t n, uint32_t flags, int blocks_cu,
                         hipStream_t stream) {
  if (stride < 32 || stride > 256 || len > stride || 4 * (stride - len) > stride) return 1;
  const uint32_t s = (uint32_t)stride;
  const uint32_t kpk = 1008u / s;                         // slots per step
  const uint32_t recip = ((1u << 20) + s - 1) / s;        // ceil(2^20 / stride)
  const uint64_t steps = ((uint64_t)n + kpk - 1) / kpk;
  uint64_t blocks = (steps + 3) / 4;
  const uint64_t cap = std::min<uint64_t>(256ull * (uint64_t)blocks_cu, (1ull << 26) / 4);
  blocks = std::max<uint64_t>(1, std::min(blocks, cap));
  const uint8_t* b = static_cast<const uint8_t*>(base);
  if (seed)
    UINET_LAUNCH((k_strided_dense<true>), dim3((uint32_t)blocks), dim3(kBlock), 0, stream,
                       b, seed, out, n, flags, s, len, kpk, recip);
  else
    UINET_LAUNCH((k_strided_dense<false>), dim3((uint32_t)blocks), dim3(kBlock), 0, stream,
                       b, seed, out, n, flags, s, len, kpk, recip);
  return check_launch();
}

// wide (uinet_cksum_spans, strided) and packed (uinet_cksum_spans32) descriptors
#define UINET_SPANS_INST(OffT, LenT)                                                        \
  template int launch_spans_quad<OffT, LenT>(const void*, const OffT*, const LenT*,         \
                                             const uint32_t*, const uint8_t*, uint16_t*,    \
                                             uint32_t, uint32_t, int, bool, uint64_t,       \
                                             uint32_t, int, hipStream_t);                   \
  template int launch_spans_lean<OffT, LenT>(const void*, const OffT*, const LenT*,         \
                                             const uint32_t*, const uint8_t*, uint16_t*,    \
                                             uint32_t, uint32_t, int, int, bool, uint64_t,  \
                                             uint32_t, int, hipStream_t, bool);
UINET_SPANS_INST(uint64_t, uint32_t)
UINET_SPANS_INST(uint32_t, uint16_t)
#undef UINET_SPANS_INST

}  // namespace uinet
