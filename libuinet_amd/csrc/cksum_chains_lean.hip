// k_chains_lean: in_cksum_skip(m, len, skip) over device-resident mbuf
// chains given as segment lists -- the same job and the same per-round chunk
// list as k_chains_pipe (cksum_chains.hip), with the pass-level work cut so
// that the kernel fits a copy-free two-batch pipeline at 8 waves per SIMD.
//
// Semantics: /root/reference/sys/amd64/amd64/in_cksum.c:203-229 (len counts
// from the chain start, zero-length mbufs contribute nothing, a short chain
// sums what it has), logical parity counted from `skip`.
//
// A wave owns a tile of kTile packets (a contiguous segment range) and works
// through it in descriptor rounds of 64 segments, one per lane:
//   * round setup (as k_chains_pipe): packet slot by LDS start markers and a
//     DPP max-scan, chain position by add/max scans, the clip to [skip, len),
//     head / chunk count; segments of 128 chunks and more are streamed by the
//     whole wave (one wave-reduced sum each);
//   * the other ("list") segments' chunks form one concatenated list of
//     16-byte chunks.  Each list segment writes its record (list start,
//     end, bin, load base) into an LDS table at its rank among the list
//     segments, and sets its start bit in a bitmap of the list (one 64-bit
//     word per 64 chunks, <= 128 words: list segments hold < 128 chunks);
//   * a pass of 64 list chunks finds each chunk's segment with two readlanes
//     of the pass's bitmap word and an mbcnt (no LDS round trip, no scan),
//     then reads the segment's record with ONE ds_read_b128 (k_chains_pipe:
//     an LDS marker write / read, a 6-step DPP max-scan and three
//     ds_bpermutes per pass);
//   * masks from the 17 x 17 LDS table, chunk sums by 4 v_dot2_u32_u16, the
//     per-(packet, parity) binning by one DPP prefix sum with +P / -P at run
//     ends (telescoping) into the wave's u64 LDS bins, as k_chains_pipe;
//   * batches of kPass passes run through two register sets, A and B, with
//     no copy between them: batch k + 1 is issued (lookup + loads) before
//     batch k is consumed, and the wave knows the round's batch count, so the
//     loop body has no exit and the wait for batch k leaves batch k + 1's
//     loads in flight.  (k_chains_pipe copies the issued set at the loop's
//     back edge, which waits for it: its loads are in flight only while the
//     previous batch is consumed.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "cksum_device.h"

namespace uinet {
namespace {

constexpr int kLWaves = kBlock / 64;
constexpr uint32_t kLongMin = 128;  // segments of >= this many chunks stream wave-wide
constexpr int kBmW = 128;           // bitmap words: a list holds < 64 * 128 chunks

__device__ __forceinline__ __amdgpu_buffer_rsrc_t lean_window(const uint8_t* sbase) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sbase), 0, (int)0xffffffffu,
                                           0x00020000);
}

template <int kPass, int kTile, typename OffT, typename LenT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void k_chains_lean(
    const uint8_t* __restrict__ base, const OffT* __restrict__ seg_off,
    const LenT* __restrict__ seg_len, const uint32_t* __restrict__ pkt_seg,
    const uint32_t* __restrict__ plen, const uint32_t* __restrict__ pskip,
    const uint32_t* __restrict__ seed, uint16_t* __restrict__ out, uint32_t n, uint32_t flags,
    uint32_t long_ch) {
  static_assert(kTile >= 1 && kTile <= 32, "a tile's packets are one per lane, 2 bins each");
  constexpr int kWin = 64 * kPass;  // list chunks per batch
  __shared__ MaskLut lut;
  __shared__ unsigned long long lds_acc[kLWaves][2 * kTile];  // (slot, rot) bins
  __shared__ uint32_t lds_pkmark[kLWaves][64];                 // packet-start markers
  __shared__ unsigned long long lds_bm[kLWaves][kBmW];         // list segment starts
  __shared__ u32x4 lds_rec[kLWaves][64];                       // list segment records
  lut.init();
  for (int i = threadIdx.x; i < kLWaves * 64; i += blockDim.x) (&lds_pkmark[0][0])[i] = 0;
  for (int i = threadIdx.x; i < kLWaves * kBmW; i += blockDim.x) (&lds_bm[0][0])[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned long long* acc = lds_acc[wid];
  uint32_t* pkmark = lds_pkmark[wid];
  unsigned long long* bm = lds_bm[wid];
  u32x4* rec = lds_rec[wid];
  const uint32_t tiles = (n + kTile - 1) / kTile;
  const uint32_t wstride = gridDim.x * kLWaves;
  const uint32_t long_min = long_ch ? min(long_ch, kLongMin) : kLongMin;

  u32x4 va[kPass], vb[kPass];
  uint32_t ka[kPass], kb[kPass];
  // The batch's chunk sums, their prefix sums side by side, the bin updates.
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
        if (lane != 63) atomicAdd(&acc[nx[q]], (unsigned long long)(-(long long)P[q]));
      }
    }
  };

  for (uint32_t t = blockIdx.x * kLWaves + wid; t < tiles; t += wstride) {
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
      // T at this segment's packet start
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
      const bool is_long = nch >= long_min;
      for (uint64_t lm = __ballot(is_long); lm; lm &= lm - 1) {
        const int s = (int)__builtin_ctzll(lm);
        const uint32_t h = __builtin_amdgcn_readlane(head, s);
        const uint32_t el = __builtin_amdgcn_readlane(eff, s);
        const uint32_t mts = __builtin_amdgcn_readlane(meta, s);
        const uint8_t* cb = base + (readlane_u64(c0_lo, c0_hi, s));
        const uint32_t nc = __builtin_amdgcn_readlane(nch, s);
        // chunk k keeps bytes [k ? 0 : h, k < nc - 1 ? 16 : last_end)
        const uint32_t last_end = ((h + (el & 15u) + 15u) & 15u) + 1u;
        constexpr int kLongU = 4;
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
      const uint32_t nch_l = is_long ? 0u : nch;
      const uint32_t ci = wave_scan<0, false>(nch_l, 0u);
      const uint32_t cst = ci - nch_l;
      const uint32_t C = __builtin_amdgcn_readlane(ci, 63);  // < 64 * kLongMin
      const uint64_t lm_list = __ballot(nch_l != 0);
      if (lm_list == 0) continue;
      const int lf = (int)__builtin_ctzll(lm_list);
      const uint64_t R0 = readlane_u64(c0_lo, c0_hi, lf);
      const uint64_t rel = c0 - R0 + (1ull << 31);  // R0 - 2 GiB .. R0 + 2 GiB
      const bool window = __ballot(nch_l != 0 && rel >= (1ull << 32) - (1ull << 16)) == 0;
      const __amdgpu_buffer_rsrc_t rsrc = lean_window(base + (R0 - (1ull << 31)));
      // record of a list segment, at its rank among the list segments:
      // (list start byte | bin << 20, list end byte, load base lo, hi)
      if (nch_l != 0) {
        const uint32_t q0 = head + 16u * cst;  // < 2^17
        const uint64_t dk = c0 - 16ull * cst;
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
            (uint32_t)(lm_list >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm_list, 0u));
        u32x4 rr;
        rr.x = q0 | (meta << 20);
        rr.y = q0 + eff;
        rr.z = window ? (uint32_t)rel - 16u * cst : (uint32_t)dk;
        rr.w = (uint32_t)(dk >> 32);
        rec[rank] = rr;
        atomicOr(&bm[cst >> 6], 1ull << (cst & 63u));
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      // the bitmap, one word per lane (words 64.. only for lists of more
      // than 4096 chunks), cleared behind the read for the next round
      const uint64_t bw0 = bm[lane];
      const bool two_words = C > 64u * 64u;  // wave-uniform
      uint64_t bw1 = 0;
      if (two_words) bw1 = bm[64 + lane];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      bm[lane] = 0;
      if (two_words) bm[64 + lane] = 0;
      uint32_t segc = 0;  // list segments started before the pass
      // the round's last list segment: a lookup is clamped to it, so that no
      // slip in the lookup can read a stale record and load from its address
      const uint32_t seg_last = (uint32_t)__builtin_popcountll(lm_list) - 1u;
      // Issue batch `b` (its first list chunk) into (v, key): segment lookup,
      // mask index and bin, loads.  Nothing here waits for packet bytes.
      auto issue = [&](uint32_t b, u32x4 (&v)[kPass], uint32_t (&key)[kPass], auto kWindow) {
#pragma unroll
        for (int q = 0; q < kPass; ++q) {
          const uint32_t w = (b >> 6) + (uint32_t)q;  // this pass's bitmap word (< 128)
          uint64_t M;
          if (w < 64) {
            M = readlane_u64((uint32_t)bw0, (uint32_t)(bw0 >> 32), (int)w);
          } else {
            M = readlane_u64((uint32_t)bw1, (uint32_t)(bw1 >> 32), (int)(w - 64));
          }
          // starts at or before the lane: bit 0 plus the bits of M >> 1 below
          // the lane (mbcnt counts the bits below the lane); chunk 0 of the
          // list always starts a segment, so seg >= 0
          const uint64_t Mr = M >> 1;
          const uint32_t seg = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(Mr >> 32),
              __builtin_amdgcn_mbcnt_lo((uint32_t)Mr, segc + (uint32_t)(M & 1u) - 1u));
          segc += (uint32_t)__builtin_popcountll(M);
          const uint32_t c = b + (uint32_t)(q * 64 + lane);
          const bool in = c < C;
          const uint32_t cc = in ? c : C - 1;  // past the end: the last chunk, masked
          const u32x4 r = rec[min(seg, seg_last)];
          const int base16 = 16 * (int)c;
          const int s_lo = (int)(r.x & 0xfffffu) - base16;
          const int s_hi = in ? (int)r.y - base16 : s_lo;
          key[q] = MaskLut::index(s_lo, s_hi) | ((r.x >> 20) << 16);
          if constexpr (decltype(kWindow)::value) {
            v[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(r.z + 16u * cc), 0, 2);
          } else {
            v[q] = load_chunk(base + ((((uint64_t)r.w << 32) | r.z) + 16ull * cc));
          }
        }
      };
      // Batches k (set A) and k + 1 (set B) alternate with no copy; the last
      // one or two batches of the round run after the loop.
      auto run = [&](auto kWindow) {
        const uint32_t nb = (C + kWin - 1) / kWin;  // >= 1
        issue(0, va, ka, kWindow);
        uint32_t k = 0;
        for (; k + 2 < nb; k += 2) {  // batches k, k + 1 and k + 2 exist
          issue((k + 1) * kWin, vb, kb, kWindow);
          consume(va, ka);
          issue((k + 2) * kWin, va, ka, kWindow);
          consume(vb, kb);
        }
        if (k + 1 < nb) {
          issue((k + 1) * kWin, vb, kb, kWindow);
          consume(va, ka);
          consume(vb, kb);
        } else {
          consume(va, ka);
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
      out[p] = finish(acc[2 * lane] + rot8(odd) + (seed ? seed[p] : 0u), flags);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

}  // namespace

template <typename OffT, typename LenT>
int launch_chains_lean_t(const void* base, const OffT* seg_off, const LenT* seg_len,
                         const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                         const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                         int tile, int bpc, uint32_t long_ch, hipStream_t stream) {
  const uint32_t tiles = (n + (uint32_t)tile - 1) / (uint32_t)tile;
  uint64_t blocks = (tiles + kLWaves - 1) / kLWaves;
  const uint64_t cap = 256ull * (uint64_t)bpc;
  blocks = std::max<uint64_t>(1, std::min(blocks, cap));
  const uint8_t* b = static_cast<const uint8_t*>(base);
#define UINET_LC(T)                                                                          \
  hipLaunchKernelGGL((k_chains_lean<2, T, OffT, LenT>), dim3((uint32_t)blocks), dim3(kBlock), \
                     0, stream, b, seg_off, seg_len, pkt_seg, len, skip, seed, out, n, flags,  \
                     long_ch)
  if (tile == 8)
    UINET_LC(8);
  else
    UINET_LC(32);
#undef UINET_LC
  return check_launch();
}

template int launch_chains_lean_t<uint64_t, uint32_t>(const void*, const uint64_t*,
                                                      const uint32_t*, const uint32_t*,
                                                      const uint32_t*, const uint32_t*,
                                                      const uint32_t*, uint16_t*, uint32_t,
                                                      uint32_t, int, int, uint32_t, hipStream_t);
template int launch_chains_lean_t<uint32_t, uint16_t>(const void*, const uint32_t*,
                                                      const uint16_t*, const uint32_t*,
                                                      const uint32_t*, const uint32_t*,
                                                      const uint32_t*, uint16_t*, uint32_t,
                                                      uint32_t, int, int, uint32_t, hipStream_t);

}  // namespace uinet
