// MI355X (gfx950) chain kernels: in_cksum_skip(m, len, skip) over
// device-resident mbuf chains given as segment lists.
//
// Packet p is the chain of segments [pkt_seg[p], pkt_seg[p+1]) (one segment
// per mbuf, in m_next order); the chain bytes [skip, len) are summed exactly
// as the reference walk does (/root/reference/sys/amd64/amd64/in_cksum.c
// :203-229 -- len counts from the chain start, zero-length mbufs contribute
// nothing, a short chain sums what it has), with the logical parity counted
// from `skip`.  len == NULL means "the whole chain", skip == NULL means 0.
//
// The kernel gives a wave a tile of 32 consecutive packets (8 when the batch
// is small), i.e. a contiguous range of segments, processed in descriptor
// rounds of 64 segments (one per lane, `describe_round`): packet slot (LDS
// start markers + a DPP max-scan), chain position (a DPP add-scan of the
// lengths minus a max-scan of the packet-start positions, carried across
// rounds), the clip to [skip, len), chunk count, (packet, parity) bin.  Long
// segments (>= long_ch chunks) are streamed by the whole wave, one at a time
// (`stream_long`).  Sums land in the wave's u64 LDS bins per (packet,
// parity); each packet's odd-parity bin is byte-rotated once at the end.
//
// k_chains_pipe -- the chunk list: a round's short segments become
// one concatenated list of 16-byte chunks that the wave sweeps 64 chunks per
// pass, so every load is a dense 1 KiB whatever the segment lengths; a chunk
// finds its segment by LDS start markers + a DPP max-scan, is masked from a
// 17x17 LDS table and binned by a telescoping DPP prefix sum; each batch of
// passes is issued one step before it is summed.
//
// Formulations measured and removed (code under profiles/r03/pruned/ and
// profiles/r04/pruned/): a serial walk (G lanes per packet), a bitmap segment
// lookup, k_chains_lean (LDS segment records), and (round 4) the address
// sweep -- a dense, ordered round read as plain chunks with a running prefix,
// each segment F(end) - F(start): 30 % fewer vector instructions per KiB but
// at best 1.5-2.4 % faster on config 3 inside this kernel (its LDS staging
// held every round to 5 waves per SIMD: 3tx 4 % slower), and 17-27 % slower
// as a kernel of its own (profiles/r04/NOTES.md).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "cksum_device.h"

namespace uinet {
namespace {

constexpr int kWaves = kBlock / 64;
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short us16x2 __attribute__((ext_vector_type(2)));
#ifndef UINET_CHAINS_LONGU  // build-time A/B knob (profiles/r01/ab/chains_occ/longu)
#define UINET_CHAINS_LONGU 2
#endif
constexpr int kLongU = UINET_CHAINS_LONGU;  // chunks in flight per lane on a long segment
constexpr uint32_t kListMax = 1024;  // longest segment (chunks) the chunk list takes
// Mean segment bytes (len_hint) for which k_chains_wide runs: a segment that
// fits one of its 9-KiB rounds (a jumbo frame, a TSO payload slice).  Longer
// segments take serial rounds, and 1-2 KiB ones leave it per-packet bound,
// where the tile kernel is faster (tools/chains_cross.py, profiles/r05/r05cross*).
constexpr uint32_t kWideHintLo = 4096, kWideHintHi = 64 * 9 * 16;

// 16-B raw buffer load, non-temporal (aux bit 1), from a resource spanning
// 4 GiB: one VGPR of offset instead of a 64-bit address per chunk.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t window_rsrc(const uint8_t* sbase) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sbase), 0, (int)0xffffffffu,
                                           0x00020000);
}
__device__ __forceinline__ u32x4 load_chunk_buf(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 2);
}

// One descriptor round's per-segment work, one segment per lane (segment
// r0 + lane: offset so, length l): the packet slot from the LDS start markers
// of the tile's packets (`ps` = lane's packet's first segment, np packets),
// the chain position, the clip to [skip, len) (lane's packet's k_skip /
// k_len, read by slot), the chunk count and the (slot, rotation) bin.  It
// reads the previous round's carries and returns the new ones.
struct RoundDesc {
  uint32_t slot, pos, eff, head, nch, rot, meta, carry_slot1, carry_pos;
  uint64_t ao, c0;
};
__device__ __forceinline__ RoundDesc describe_round(uint32_t* pkmark, int lane, int np, uint32_t ps,
                                                    uint32_t r0, uint64_t so, uint32_t l,
                                                    uint32_t k_skip, uint32_t k_len,
                                                    uint32_t carry_slot1, uint32_t carry_pos,
                                                    const uint8_t* base) {
  RoundDesc D;
  const bool pk_in = lane < np && ps >= r0 && ps < r0 + 64;
  if (pk_in) atomicMax(&pkmark[ps - r0], (uint32_t)lane + 1);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint32_t pk = pkmark[lane];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (pk_in) pkmark[ps - r0] = 0;
  const uint32_t slot1 = max(wave_scan<1, false>(pk, 0u), carry_slot1);
  D.slot = slot1 - 1;
  // chain position: T = carry_pos + exclusive prefix of the lengths never
  // decreases along the lanes, so the max-scan of T at packet starts is T at
  // this segment's packet start (0 while the packet of the previous round
  // continues: its position is T itself)
  const uint32_t T = carry_pos + wave_scan<0, false>(l, 0u) - l;
  D.pos = T - wave_scan<1, false>(pk ? T : 0u, 0u);
  D.carry_slot1 = __builtin_amdgcn_readlane(slot1, 63);
  D.carry_pos = __builtin_amdgcn_readlane(D.pos + l, 63);
  const uint32_t sk = __shfl(k_skip, (int)D.slot);
  const uint32_t ln = __shfl(k_len, (int)D.slot);
  const uint32_t lo = sk > D.pos ? min(sk - D.pos, l) : 0u;
  const uint32_t hi = ln > D.pos ? min(ln - D.pos, l) : 0u;
  D.eff = hi > lo ? hi - lo : 0u;
  D.ao = so + lo;
  D.head = D.eff ? (uint32_t)(reinterpret_cast<uintptr_t>(base + D.ao) & 15) : 0u;
  // chunks touched, without forming head + eff (a u32 segment may be 4 GiB)
  D.nch = D.eff ? (D.eff >> 4) + ((D.head + (D.eff & 15u) + 15u) >> 4) : 0u;
  D.c0 = D.ao - D.head;
  D.rot = ((D.pos + lo - sk) ^ (uint32_t)reinterpret_cast<uintptr_t>(base + D.ao)) & 1u;
  D.meta = (D.slot << 1) | D.rot;
  return D;
}

// The round's long segments (lanes set in lm), one wave-wide span each:
// kLongU chunks per lane in flight, one wave-reduced sum added to the
// segment's bin.  sum(v, lo, hi) folds bytes [lo, hi) of a chunk (u64).
template <typename SumFn>
__device__ __forceinline__ void stream_long(uint64_t lm, const RoundDesc& D, const uint8_t* base,
                                            int lane, unsigned long long* acc, SumFn sum) {
  const uint32_t c0_lo = (uint32_t)D.c0, c0_hi = (uint32_t)(D.c0 >> 32);
  for (; lm; lm &= lm - 1) {
    const int s = (int)__builtin_ctzll(lm);
    // head and length read separately: a segment may hold up to 4 GiB, more
    // than one packed 32-bit word (eff << 4 | head) keeps
    const uint32_t h = __builtin_amdgcn_readlane(D.head, s);
    const uint32_t el = __builtin_amdgcn_readlane(D.eff, s);
    const uint32_t mts = __builtin_amdgcn_readlane(D.meta, s);
    const uint8_t* cb = base + (readlane_u64(c0_lo, c0_hi, s));
    const uint32_t nc = __builtin_amdgcn_readlane(D.nch, s);
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
          lsum += sum(v[u], lo_b, hi_b);
        }
      }
    }
    const uint32_t x = __builtin_amdgcn_readlane(wave_scan<0, false>(fold16(lsum), 0u), 63);
    if (lane == 0) atomicAdd(&acc[mts], (unsigned long long)x);
  }
}

// k_chains_pipe: the pipelining and addressing details.
//   * A batch is ISSUED (segment lookup, mask index and bin, loads) one step
//     before it is CONSUMED (chunk sums, binning), so batch k+1's loads are in
//     flight while batch k is summed.  The pipeline drains at the end of each
//     round: carrying it across rounds (round r+1's descriptor work under
//     round r's last loads) needed 104 VGPRs and ran 20 % slower at
//     occupancy 4 (profiles/r01/ab/chains_pipe/).
//   * What a consumed chunk needs besides its bytes is one packed word
//     (mask-table index | bin << 16).
//   * Chunks within the round's 4 GiB window load through a raw buffer
//     resource: one 32-bit VGPR offset per chunk; otherwise 64-bit addresses.
// Against the same scheme without pipelining (k_chains_flat, removed after
// this A/B; interleaved, same process): config 3 +2.4-2.7 %, 3tx +1-2 %, 5tso
// equal.  Things that did NOT help: an LDS rank lookup of the segment records
// (VALU -14 %, but a second dependent LDS round trip before each load: -13 %),
// temporal instead of non-temporal loads (HBM bytes -1.1 %, time +8 %), an
// XCD-banded tile order, smaller tiles at the end of the launch, a pipelined
// long-segment stream (profiles/r01/ab/).
// Build-time occupancy override for A/B (-DUINET_CHAINS_WAVES=N forces that
// many waves per SIMD, spilling what does not fit).
// The default holds the kPass = 2 kernel at 7 waves per SIMD (72 VGPRs, no
// spills): left alone the compiler takes 88 for the interleaved consume and
// drops to 5.  7 fits because a long segment keeps 2 chunks per lane in flight
// (kLongU), not 4: the long-segment loads were the round-level pressure point
// that spilled 36 B at 7 waves (profiles/r03/r03s2d/).  7 waves with kLongU 2
// against 6 with 4: config 3 -1.0 %, 3tx -0.2 %, 5tso -0.7 % time
// (profiles/r03/r03s2u/); 8 waves (64 VGPRs) still spills, +21 %.
#ifdef UINET_CHAINS_WAVES
#define UINET_CHAINS_OCC __attribute__((amdgpu_waves_per_eu(UINET_CHAINS_WAVES)))
#else
#define UINET_CHAINS_OCC __attribute__((amdgpu_waves_per_eu(kPass == 2 ? 7 : 1)))
#endif

template <int kPass, int kTile, typename OffT, typename LenT>
__global__ __launch_bounds__(kBlock) UINET_CHAINS_OCC void k_chains_pipe(const uint8_t* __restrict__ base,
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
  // segment-start markers per batch, (lane + 1) << 8 | meta, and one spare slot
  // per lane that lanes without a start in the batch write (no exec mask)
  __shared__ uint16_t lds_mark[kWaves][kWin + 64];
  lut.init();
  for (int i = threadIdx.x; i < kWaves * 64; i += blockDim.x) (&lds_pkmark[0][0])[i] = 0;
  for (int i = threadIdx.x; i < kWaves * (kWin + 64); i += blockDim.x) (&lds_mark[0][0])[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned long long* acc = lds_acc[wid];
  uint32_t* pkmark = lds_pkmark[wid];
  uint16_t* mark = lds_mark[wid];
  // 16 x (chunk - batch start) of this lane's chunk in pass q, in both halves
  s16x2 lane16[kPass];
#pragma unroll
  for (int q = 0; q < kPass; ++q) {
    const short x = (short)(16 * (q * 64 + lane));
    lane16[q] = s16x2{x, x};
  }
  const uint32_t tiles = (n + kTile - 1) / kTile;
  const uint32_t wstride = gridDim.x * kWaves;

  // the pipeline's register sets: the pending batch (issued, not yet
  // consumed; `pend` wave-uniform) in a, the one being issued in b
  u32x4 va[kPass], vb[kPass];
  uint32_t ka[kPass], kb[kPass];
  uint32_t pend = 0;
  // The passes' chunk sums first, then their prefix sums side by side (the
  // DPP chains interleave: +1.3-3 % on config 3, profiles/r02/ab_lab/), then
  // the bin updates.
  auto consume = [&](const u32x4 (&v)[kPass], const uint32_t (&key)[kPass]) {
    uint32_t P[kPass], sl[kPass], nx[kPass];
#pragma unroll
    for (int q = 0; q < kPass; ++q) P[q] = lut.sum_oc_idx(v[q], key[q] & 0xffffu);  // < 2^19
#pragma unroll
    for (int q = 0; q < kPass; ++q) {
      sl[q] = key[q] >> 16;
      nx[q] = wave_shl1(sl[q]);
    }
    wave_scan_add_n<kPass>(P);  // < 2^25
#pragma unroll
    for (int q = 0; q < kPass; ++q) {
      if (lane == 63 || nx[q] != sl[q]) {
        atomicAdd(&acc[sl[q]], (unsigned long long)P[q]);
        if (lane != 63) __atomic_fetch_sub(&acc[nx[q]], (unsigned long long)P[q], __ATOMIC_RELAXED);
      }
    }
  };

  for (uint32_t t = blockIdx.x * kWaves + wid; t < tiles; t += wstride) {
    const uint32_t P0 = t * kTile;
    const int np = (int)min((uint32_t)kTile, n - P0);
    const uint32_t ps = pkt_seg[P0 + (uint32_t)min(lane, np)];
    const uint32_t k_skip = (lane < np && pskip) ? pskip[P0 + lane] : 0u;
    const uint32_t k_len = (lane < np) ? (plen ? plen[P0 + lane] : 0xffffffffu) : 0u;
    const uint32_t S0 = __builtin_amdgcn_readfirstlane(ps);
    const uint32_t S1 = __builtin_amdgcn_readlane(ps, np);
    if (lane < 2 * kTile) acc[lane] = 0;
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
      const RoundDesc D = describe_round(pkmark, lane, np, ps, r0, so, l, k_skip, k_len,
                                         carry_slot1, carry_pos, base);
      carry_slot1 = D.carry_slot1;
      carry_pos = D.carry_pos;
      const uint32_t eff = D.eff, head = D.head, nch = D.nch, meta = D.meta;
      const uint64_t c0 = D.c0;
      const uint32_t c0_lo = (uint32_t)c0, c0_hi = (uint32_t)(c0 >> 32);
      // --- long segments: one wave-wide span each -------------------------
      const bool is_long =
          nch >= kListMax || (long_ch != 0 && nch >= long_ch);
      stream_long(__ballot(is_long), D, base, lane, acc,
                  [&](u32x4 v, int lo_b, int hi_b) { return lut.sum(v, lo_b, hi_b); });
      // --- the round's chunk list -----------------------------------------
      const uint32_t nch_l = is_long ? 0u : nch;
      const uint32_t ci = wave_scan<0, false>(nch_l, 0u);
      const uint32_t cst = ci - nch_l;
      const uint32_t C = __builtin_amdgcn_readlane(ci, 63);  // < 64 * kListMax
      const uint64_t lm_list = __ballot(nch_l != 0);
      if (lm_list == 0) continue;
      const int lf = (int)__builtin_ctzll(lm_list);
      const uint64_t R0 = readlane_u64(c0_lo, c0_hi, lf);
      const uint64_t rel = c0 - R0 + (1ull << 31);  // R0 - 2 GiB .. R0 + 2 GiB
      const bool window = __ballot(nch_l != 0 && rel >= (1ull << 32) - (1ull << 16)) == 0;
      // The segment's kept bytes [q0, q0 + eff) in list bytes (q0 < 2^20),
      // as a pair of 16-bit halves: a chunk's mask bounds are this pair minus
      // 16 x its list chunk, exact in 16 bits for the chunk's own segment
      // (|q0 - 16 c| < 16 kListMax + 2 KiB) and computed modulo 2^16 per half.
      const uint32_t q0 = head + 16u * cst;
      const uint32_t r16 = (q0 & 0xffffu) | ((q0 + eff) << 16);
      const uint16_t mval = (uint16_t)(((uint32_t)lane + 1u) << 8 | meta);
      const uint64_t dk = c0 - 16ull * cst;
      const uint32_t dkr = (uint32_t)rel - 16u * cst;  // mod 2^32; + 16 c lands in range
      const __amdgpu_buffer_rsrc_t rsrc = window_rsrc(base + (R0 - (1ull << 31)));
      uint32_t carry_seg1 = 0;  // segment + 1 of the chunk before the batch
      // Issue the batch at list chunk b into (v, key): segment lookup, mask
      // index and bin, loads.  Nothing here waits for packet bytes.
      //   * lookup: the batch's segment starts are marked in LDS with
      //     (lane + 1) << 8 | meta; a max-scan gives every chunk its segment
      //     and its bin (meta = slot << 1 | rot) in one value, carried across
      //     passes as a scalar max;
      //   * key: the segment's 16-bit pair (kept bytes relative to the batch)
      //     minus the chunk's 16 x position, clamped to [0, 16] by two packed
      //     16-bit ops, becomes the mask-table index lo * 17 + hi and the bin
      //     in one v_dot2 (a chunk past the list end clamps to the empty mask);
      //   * two ds_bpermutes per chunk: the pair and the window offset.
      auto issue = [&](uint32_t b, u32x4 (&v)[kPass], uint32_t (&key)[kPass], auto kWindow) {
        const bool mk = nch_l != 0 && cst >= b && cst < b + kWin;
        const uint32_t mslot = mk ? cst - b : (uint32_t)(kWin + lane);
        mark[mslot] = mval;
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
        const short b16 = (short)(16u * b);
        const s16x2 rb = __builtin_bit_cast(s16x2, r16) - s16x2{b16, b16};
        const uint32_t rbw = __builtin_bit_cast(uint32_t, rb);
#pragma unroll
        for (int q = 0; q < kPass; ++q) {
          const uint32_t c = b + (uint32_t)(q * 64 + lane);
          const uint32_t cc = min(c, C - 1);  // past the end: the last chunk, masked
          // byte address of the segment's lane for ds_bpermute; cross-lane
          // reads stay outside any condition (a ds_bpermute under a partial
          // exec mask reads 0 from the inactive source lanes)
          const int src = (int)(sc1[q] >> 6) - 4;  // meta < 64 shifts out
          const s16x2 pr =
              __builtin_bit_cast(s16x2, (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)rbw)) -
              lane16[q];
          const s16x2 cl = __builtin_elementwise_min(__builtin_elementwise_max(pr, s16x2{0, 0}),
                                                     s16x2{16, 16});
          // meta (byte 0 of the mark) into byte 2: one v_perm
          key[q] = __builtin_amdgcn_udot2(__builtin_bit_cast(us16x2, cl), us16x2{17, 1},
                                          __builtin_amdgcn_perm(0u, sc1[q], 0x0c000c0cu), false);
          if constexpr (decltype(kWindow)::value) {
            const uint32_t d = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)dkr);
            v[q] = load_chunk_buf(rsrc, d + 16u * cc);
          } else {
            const uint32_t lo32 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)dk);
            const uint32_t hi32 =
                (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(dk >> 32));
            v[q] = load_chunk(base + ((((uint64_t)hi32 << 32) | lo32) + 16ull * cc));
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        mark[mslot] = 0;
      };
      auto run = [&](auto kWindow) {
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
      out[p] = finish(acc[2 * lane] + rot8(odd) + (seed ? seed[p] : 0u), flags);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}


// A segment length read by a wave-uniform (scalar) load.  A packed u16 length
// is taken out of its aligned 32-bit word: s_load has no 16-bit form, and a
// vector load of it would share the vector memory counter with the packet
// bytes in flight (a wait for it waits for them).  The word lies in the page
// that holds the length.
template <typename LenT>
__device__ __forceinline__ uint32_t seg_len_at(const LenT* __restrict__ p, uint32_t s) {
  if constexpr (sizeof(LenT) == 2) {
    // the word pointer stays derived from the argument (no integer round
    // trip), which is what lets the compiler keep the load scalar
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(p) >> 1) & 1u;
    const uint32_t i = s + mis;
    const uint32_t w = reinterpret_cast<const uint32_t*>(p - mis)[i >> 1];
    return (i & 1u) ? w >> 16 : w & 0xffffu;
  } else {
    return (uint32_t)p[s];
  }
}

// k_chains_wide: one wave per packet, for chains of few long segments (a TSO
// engine's 40-B header mbuf + 9 KB payload slice, config 5tso).  The tile
// kernel above streams such a segment with 2 chunks per lane in flight (its
// 72-VGPR budget) and serialises a tile's 32 packets in one wave; here every
// packet is a wave of its own and each segment goes out as kWideU chunks per
// lane at once -- the span kernel's 64 x 9 shape, 9 KiB per load round.  The
// segments of a packet are walked in order with wave-uniform (scalar)
// descriptor reads, clipped to [skip, len) exactly as describe_round does,
// summed into (even, odd) logical-parity accumulators, and the odd one is
// byte-rotated once at the end (in_cksum.c:222-225).
constexpr int kWideU = 9;
template <typename OffT, typename LenT>
__global__ __launch_bounds__(kBlock) void k_chains_wide(const uint8_t* __restrict__ base,
                                                       const OffT* __restrict__ seg_off,
                                                       const LenT* __restrict__ seg_len,
                                                       const uint32_t* __restrict__ pkt_seg,
                                                       const uint32_t* __restrict__ plen,
                                                       const uint32_t* __restrict__ pskip,
                                                       const uint32_t* __restrict__ seed,
                                                       uint16_t* __restrict__ out, uint32_t n,
                                                       uint32_t flags, uint32_t remap) {
  __shared__ MaskLut lut;
  lut.init();
  const int lane = threadIdx.x & 63;
  const uint32_t wstride = gridDim.x * kWaves;
  // XCD-banded packet order (knob xcd_remap): neighbouring packets share
  // descriptor and header lines, fetched once into one XCD's L2
  for (uint32_t p = __builtin_amdgcn_readfirstlane(logical_block(remap) * kWaves + (threadIdx.x >> 6));
       p < n; p += wstride) {
    const uint32_t S0 = pkt_seg[p], S1 = pkt_seg[p + 1];
    const uint32_t sk = pskip ? pskip[p] : 0u;
    const uint32_t ln = plen ? plen[p] : 0xffffffffu;
    uint64_t ev = 0, od = 0;  // this lane's chunk sums by logical parity
    struct Seg {
      const uint8_t* cb;
      uint32_t head, nch, last_end;
      bool rot;
    };
    // Segment s at chain offset pos, clipped to [sk, ln): nch 0 when empty.
    // Descriptors are read by scalar loads (wave-uniform), so a read never
    // waits behind packet-byte loads in the vector memory counter.
    auto desc = [&](uint32_t s, uint32_t pos, uint32_t l) {
      Seg g{nullptr, 0u, 0u, 0u, false};
      const uint32_t lo = sk > pos ? min(sk - pos, l) : 0u;
      const uint32_t hi = ln > pos ? min(ln - pos, l) : 0u;
      if (hi > lo) {
        const uint32_t eff = hi - lo;
        const uint8_t* a = base + (uint64_t)seg_off[s] + lo;
        g.head = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15);
        g.nch = (eff >> 4) + ((g.head + (eff & 15u) + 15u) >> 4);
        g.last_end = ((g.head + (eff & 15u) + 15u) & 15u) + 1u;
        g.cb = a - g.head;
        g.rot = ((pos + lo - sk) ^ (uint32_t)reinterpret_cast<uintptr_t>(a)) & 1u;
      }
      return g;
    };
    // chunk k's kept byte range [lo_b, hi_b) within segment g
    auto lo_of = [](const Seg& g, uint32_t k) { return k == 0 ? (int)g.head : (k < g.nch ? 0 : 16); };
    auto hi_of = [](const Seg& g, uint32_t k) {
      return k + 1 < g.nch ? 16 : (k + 1 == g.nch ? (int)g.last_end : 0);
    };
    auto add = [&](bool rot, uint64_t x) {
      if (rot) od += x; else ev += x;
    };
    // One round of a long segment from chunk k0: kWideU chunks per lane.
    // `pre` runs between the loads and their sums (a short segment summed
    // while these loads are in flight).
    auto round = [&](const Seg& g, uint32_t k0, auto pre) {
      u32x4 v[kWideU];
#pragma unroll
      for (int u = 0; u < kWideU; ++u)
        if (u == 0 || k0 + 64u * u < g.nch)
          v[u] = load_chunk(g.cb + 16ull * min(k0 + (uint32_t)(u * 64 + lane), g.nch - 1));
      pre();
      uint32_t part = 0;  // < kWideU * 2^19
#pragma unroll
      for (int u = 0; u < kWideU; ++u) {
        if (u == 0 || k0 + 64u * u < g.nch) {
          const uint32_t k = k0 + (uint32_t)(u * 64 + lane);
          part += lut.sum_oc(v[u], lo_of(g, k), hi_of(g, k));
        }
      }
      add(g.rot, part);
    };
    auto rest = [&](const Seg& g) {
      for (uint32_t k0 = 64 * kWideU; k0 < g.nch; k0 += 64 * kWideU) round(g, k0, [] {});
    };
    uint32_t pos = 0;  // chain offset of segment s
    for (uint32_t s = S0; s < S1; ++s) {
      const uint32_t l = seg_len_at(seg_len, s);
      const Seg g = desc(s, pos, l);
      pos += l;
      if (g.nch == 0) continue;
      if (g.nch > 64) {  // long: rounds of kWideU chunks per lane
        round(g, 0, [] {});
        rest(g);
        continue;
      }
      // short (one chunk per lane).  Followed by a long segment (a TSO
      // header and its payload slice), the long one's descriptor is read
      // while the short one's bytes are in flight, and its sum is added under
      // the long one's first round.
      const uint32_t k = (uint32_t)lane;
      const u32x4 hv = load_chunk(g.cb + 16ull * min(k, g.nch - 1));
      const uint32_t hs = lut.sum_oc(hv, lo_of(g, k), hi_of(g, k));
      if (s + 1 < S1) {
        const uint32_t l2 = seg_len_at(seg_len, s + 1);
        const Seg g2 = desc(s + 1, pos, l2);
        if (g2.nch > 64) {
          pos += l2;
          ++s;
          round(g2, 0, [&] { add(g.rot, hs); });
          rest(g2);
          continue;
        }
      }
      add(g.rot, hs);
    }
    const uint32_t e = __builtin_amdgcn_readlane(wave_scan<0, false>(fold16(ev), 0u), 63);
    const uint32_t o = __builtin_amdgcn_readlane(wave_scan<0, false>(fold16(od), 0u), 63);
    if (lane == 0) out[p] = finish((uint64_t)e + rot8(fold16(o)) + (seed ? seed[p] : 0u), flags);
  }
}

template <typename OffT, typename LenT>
int launch_chains_t(const void* base, const OffT* seg_off, const LenT* seg_len,
                    const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                    const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                    uint32_t len_hint, hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  const Tuning& tn = tuning();
  const uint8_t* b = static_cast<const uint8_t*>(base);
  // Segments of 4-9 KiB on average (len_hint = mean segment bytes): a wave per packet.
  if (tn.chains_wide == 2 ||
      (tn.chains_wide == 0 && len_hint >= kWideHintLo && len_hint <= kWideHintHi)) {
    uint64_t blocks = ((uint64_t)n + kWaves - 1) / kWaves;
    const uint64_t cap = 256ull * (uint64_t)blocks_per_cu(64);
    blocks = blocks > cap ? cap : blocks;
    UINET_LAUNCH((k_chains_wide<OffT, LenT>), dim3((int)blocks), dim3(kBlock), 0, stream, b,
                 seg_off, seg_len, pkt_seg, len, skip, seed, out, n, flags, (uint32_t)tn.xcd_remap);
    return check_launch();
  }
  // Tile of 32 packets, or 8 when 32 would give fewer than 16 tiles per CU
  // (5tso, 131 K packets, runs 0.8 % faster at 32: profiles/r01/ab/bpc_s6/tile;
  // the 128 K switch rechecked on mid-size config-3 batches, profiles/r05/r05tile/).
  // Two 64-chunk passes per batch: four lost on every config
  // (profiles/r01/ab/chains_pipe/); the chains_pass / chains_tile knobs that
  // forced other shapes were removed in round 6 (profiles/r06/pruned/).
  const int tile = n >= 32u * 4096u ? 32 : 8;
  const uint32_t tiles = (n + (uint32_t)tile - 1) / (uint32_t)tile;
  uint64_t blocks = (tiles + kWaves - 1) / kWaves;
  const uint64_t cap = 256ull * (uint64_t)blocks_per_cu(64);
  blocks = blocks > cap ? cap : blocks;
  const uint32_t long_ch = (uint32_t)tn.chains_long;
#define LF(P, T)                                                                           \
  UINET_LAUNCH((k_chains_pipe<P, T, OffT, LenT>), dim3((int)blocks), dim3(kBlock), 0,   \
               stream, b, seg_off, seg_len, pkt_seg, len, skip, seed, out, n, flags, long_ch)
  if (tile == 8)
    LF(2, 8);
  else
    LF(2, 32);
#undef LF
  return check_launch();
}

}  // namespace

int launch_chains(const void* base, const uint64_t* seg_off, const uint32_t* seg_len,
                  const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                  const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                  uint32_t len_hint, hipStream_t stream) {
  return launch_chains_t(base, seg_off, seg_len, pkt_seg, len, skip, seed, out, n, flags,
                         len_hint, stream);
}

int launch_chains32(const void* base, const uint32_t* seg_off, const uint16_t* seg_len,
                    const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                    const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                    uint32_t len_hint, hipStream_t stream) {
  return launch_chains_t(base, seg_off, seg_len, pkt_seg, len, skip, seed, out, n, flags,
                         len_hint, stream);
}

}  // namespace uinet
