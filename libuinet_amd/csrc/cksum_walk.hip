// MI355X (gfx950) device-side mbuf chain walk for host-mbuf batches whose
// mbufs and packet bytes all lie in registered host memory
// (uinet_cksum_register_host: the UMA slabs of uinet_vm_kern.c:48-51, the
// netmap rings of uinet_if_netmap_host.c:153).
//
// The host hands over only the batch's jobs -- head mbuf pointer, len, skip,
// seed per packet -- and the small table of registered regions.  A pair of
// lanes per packet chases m_next / m_data / m_len (struct m_hdr offsets 0 / 16 /
// 24, /root/reference/sys/sys/mbuf.h:90-98) over PCIe through the regions'
// device aliases, exactly as far as in_cksum_skip reads the chain
// (/root/reference/sys/amd64/amd64/in_cksum.c:203-229: until `len` bytes
// from the chain start are covered or m_next is NULL), and writes one
// segment per mbuf into the packet's K-slot row of an HBM segment list
// (zero-length slots pad the row).  k_chains_pipe then folds that list with
// the packets' own len / skip -- the [skip, len) clip, zero-length mbufs and
// the logical parity are the chain kernel's, which is parity-tested against
// the oracle -- reading the packet bytes in place over PCIe.
//
// Anything the walk cannot take the way the host walk would is reported in
// the status word and the host runs that batch through its own walk instead:
// a pointer outside the registered regions, a negative m_len or skip, and (in
// the in_cksum_pseudo_header form) a first mbuf shorter than off0, where the
// reference's sum is not the skip form's (in_cksum.c:254-256).  status[1] is
// the longest chain: when it exceeds K the batch is walked again with room
// for it, and the next batch starts from it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cksum_internal.h"
#include "walk_xlate.h"

namespace uinet {
namespace {

using WalkRegion = WalkRegionHost;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 GlobalU32x4;

// The partner lane's value (lanes 2k and 2k + 1 swap): DPP quad_perm [1,0,3,2].
__device__ __forceinline__ uint32_t pair_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

// Two lanes per packet: lanes 2k and 2k + 1 load the two 16-B halves of the
// header's first 32 bytes in ONE instruction, which the coalescer issues as
// one request for the line (one lane loading both halves issues two), then
// swap halves over DPP.  Both lanes of a pair follow the same chain, so their
// control flow is identical.  What bounds the walk is the host link, not the
// requests: every hop costs L2 a 128-B line read over PCIe for 32 useful
// bytes, and the walk moves those lines at ~40 GB/s, the rate the fold reads
// packet bytes at (k_walk_mbufs; profiles/r05/r05p-r05r).
__global__ __launch_bounds__(256) void k_walk_mbufs(
    const uint64_t* __restrict__ heads, const int32_t* __restrict__ jlen,
    const int32_t* __restrict__ jskip, const uint32_t* __restrict__ jseed,
    const WalkRegion* __restrict__ regions, int nreg, uint32_t n, uint32_t K, uint32_t seg_base,
    uint64_t lo_dev, int pseudo, uint64_t* __restrict__ seg_off, uint32_t* __restrict__ seg_len,
    uint32_t* __restrict__ pkt_seg, uint32_t* __restrict__ len_out,
    uint32_t* __restrict__ skip_out, uint32_t* __restrict__ seed_out,
    uint32_t* __restrict__ status) {
  __shared__ WalkRegion R[kWalkRegionsMax];
  for (int k = (int)threadIdx.x; k < nreg; k += (int)blockDim.x) R[k] = regions[k];
  __syncthreads();
  const uint32_t half = threadIdx.x & 1;  // which 16 B of the header this lane loads
  const uint32_t stride = (gridDim.x * blockDim.x) >> 1;
  uint32_t any_bad = 0, longest = 0;  // this lane's, over its packets
  for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 1; i < n; i += stride) {
    const uint64_t head = heads[i];
    const int32_t L = jlen[i], S = jskip[i];
    const uint32_t lim = L < 0 ? 0u : (uint32_t)L;  // len < 0: nothing is summed
    uint32_t bad = S < 0 ? kWalkFallback : 0u;
    uint32_t cnt = 0;
    uint64_t cum = 0;
    const size_t row = (size_t)i * K;
    for (uint64_t m = head; !bad && m && cum < lim;) {
      // a chain no row can hold goes to the host walk: the walk stops here, so
      // a cyclic or corrupt m_next list cannot keep the kernel running
      if (cnt >= kWalkKMax) {
        bad = kWalkFallback;
        break;
      }
      uint64_t dm;
      if (!walk_xlate(R, nreg, m, 32, &dm)) {
        bad = kWalkUnmapped;
        break;
      }
      // lane 0 of the pair: m_next, m_nextpkt; lane 1: m_data, m_len, m_flags
      const u32x4 v = reinterpret_cast<const GlobalU32x4*>(dm)[half];
      const uint32_t w0 = pair_swap(v.x), w1 = pair_swap(v.y), w2 = pair_swap(v.z);
      const uint64_t next = half ? ((uint64_t)w0 | (uint64_t)w1 << 32)
                                 : ((uint64_t)v.x | (uint64_t)v.y << 32);
      const uint64_t data = half ? ((uint64_t)v.x | (uint64_t)v.y << 32)
                                 : ((uint64_t)w0 | (uint64_t)w1 << 32);
      const int32_t ml = (int32_t)(half ? v.z : w2);
      if (ml < 0 || (pseudo && cnt == 0 && ml < S)) {
        bad = kWalkFallback;
        break;
      }
      uint64_t off = 0;
      if (ml > 0) {
        uint64_t dd;
        if (!walk_xlate(R, nreg, data, (uint64_t)ml, &dd)) {
          bad = kWalkUnmapped;
          break;
        }
        off = dd - lo_dev;
      }
      if (cnt < K) {  // one store each
        if (half) seg_len[row + cnt] = (uint32_t)ml;
        else seg_off[row + cnt] = off;
      }
      cnt++;
      cum += (uint64_t)ml;
      m = next;
    }
    for (uint32_t k = cnt; k < K; k++) {
      if (half) seg_len[row + k] = 0;
      else seg_off[row + k] = 0;
    }
    any_bad |= bad;
    longest = max(longest, cnt);
    if (!half) {
      pkt_seg[i] = seg_base + i * K;
      if (i == n - 1) pkt_seg[n] = seg_base + n * K;
      len_out[i] = lim;
      skip_out[i] = (uint32_t)S;
    } else {
      seed_out[i] = jseed ? jseed[i] : 0u;
    }
  }
  // one atomic per wave: the status bits and the longest chain (the host
  // sizes the next batch's rows by it)
  for (int d = 32; d; d >>= 1) {
    any_bad |= (uint32_t)__shfl_xor((int)any_bad, d);
    longest = max(longest, (uint32_t)__shfl_xor((int)longest, d));
  }
  if ((threadIdx.x & 63) == 0) {
    if (any_bad) atomicOr(&status[0], any_bad);
    if (longest) atomicMax(&status[1], longest);
  }
}

// One lane per packet: a batch whose every sum lies in its packet's first
// mbuf (the single-mbuf span path with the mbufs registered too), read by the
// GPU instead of the host.  Packet i's head mbuf (its first 32 bytes) gives the
// span [m_data + skip, m_data + min(len, m_len)) exactly as the host span path
// takes it (in_cksum.c:203-229, :254-272; cksum_api.hip span_fast_batch):
// its device address and length go to off / len (0 / 0 when nothing is
// summed), the seed to seed_out.  A sum that needs a second mbuf, a negative
// skip or m_len, or a byte outside the regions sets status bits and the host
// takes the batch another way.  stats (6 u64, initialised by the caller to
// {~0, 0, 0, 0, ~0, 0}): the lowest span address, the highest span end, the
// summed bytes, the status bits, the lowest and highest region index -- what
// the host needs to copy a dense group to HBM in one run.
__global__ __launch_bounds__(256) void k_span_walk(
    const uint64_t* __restrict__ heads, const int32_t* __restrict__ jlen,
    const int32_t* __restrict__ jskip, const uint32_t* __restrict__ jseed,
    const WalkRegion* __restrict__ regions, int nreg, uint32_t n, int pseudo,
    uint64_t* __restrict__ off_out, uint32_t* __restrict__ len_out,
    uint32_t* __restrict__ seed_out, unsigned long long* __restrict__ stats) {
  __shared__ WalkRegion R[kWalkRegionsMax];
  for (int k = (int)threadIdx.x; k < nreg; k += (int)blockDim.x) R[k] = regions[k];
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t lo = ~0ull, hi = 0, bytes = 0;
  uint32_t bad = 0, rmin = ~0u, rmax = 0;
  if (i < n) {
    const uint64_t m = heads[i];
    const int32_t L = jlen[i], S = jskip[i];
    uint64_t off = 0;
    uint32_t len = 0;
    if (S < 0) {
      bad = kWalkFallback;
    } else if (m && L > S) {
      uint64_t dm;
      if (!walk_xlate(R, nreg, m, 32, &dm)) {
        bad = kWalkUnmapped;
      } else {
        // m_next, m_nextpkt | m_data, m_len, m_flags (sys/sys/mbuf.h:90-98)
        const u32x4 a = reinterpret_cast<const GlobalU32x4*>(dm)[0];
        const u32x4 b = reinterpret_cast<const GlobalU32x4*>(dm)[1];
        const uint64_t next = (uint64_t)a.x | (uint64_t)a.y << 32;
        const uint64_t data = (uint64_t)b.x | (uint64_t)b.y << 32;
        const int32_t ml = (int32_t)b.z;
        const bool more = next != 0;
        const bool second = S < ml ? (L > ml && more) : (more || (pseudo && S > ml));
        if (ml < 0 || second) {
          bad = kWalkFallback;
        } else if (S < ml) {
          const uint32_t span = (uint32_t)(min(L, ml) - S);
          uint64_t dd;
          if (!walk_xlate(R, nreg, data + (uint64_t)S, span, &dd)) {
            bad = kWalkUnmapped;
          } else {
            int r = 0;  // the region (walk_xlate's search, for its index)
            for (int lo_i = 0, hi_i = nreg; lo_i < hi_i;) {
              const int mid = (lo_i + hi_i) >> 1;
              if (R[mid].base <= data + (uint64_t)S) {
                lo_i = mid + 1;
                r = mid;
              } else {
                hi_i = mid;
              }
            }
            off = dd;
            len = span;
            lo = dd;
            hi = dd + span;
            bytes = span;
            rmin = rmax = (uint32_t)r;
          }
        }
      }
    }
    off_out[i] = off;
    len_out[i] = len;
    if (seed_out) seed_out[i] = jseed ? jseed[i] : 0u;
  }
  for (int d = 32; d; d >>= 1) {
    const uint64_t olo = (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)lo, d) |
                         (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(lo >> 32), d) << 32;
    const uint64_t ohi = (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)hi, d) |
                         (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(hi >> 32), d) << 32;
    const uint64_t ob = (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)bytes, d) |
                        (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(bytes >> 32), d) << 32;
    lo = min(lo, olo);
    hi = max(hi, ohi);
    bytes += ob;
    bad |= (uint32_t)__shfl_xor((int)bad, d);
    rmin = min(rmin, (uint32_t)__shfl_xor((int)rmin, d));
    rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, d));
  }
  if ((threadIdx.x & 63) == 0) {
    if (bytes) {
      atomicMin(&stats[0], (unsigned long long)lo);
      atomicMax(&stats[1], (unsigned long long)hi);
      atomicAdd(&stats[2], (unsigned long long)bytes);
      atomicMin(&stats[4], (unsigned long long)rmin);
      atomicMax(&stats[5], (unsigned long long)rmax);
    }
    if (bad) atomicOr(&stats[3], (unsigned long long)bad);
  }
}

// off[i] := its offset from gbase (0 for an empty span: the span kernel may
// read its base, which the caller keeps readable).
__global__ __launch_bounds__(256) void k_span_rebase(uint64_t* __restrict__ off,
                                                     const uint32_t* __restrict__ len, uint32_t n,
                                                     uint64_t gbase) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) off[i] = len[i] ? off[i] - gbase : 0ull;
}

}  // namespace

int launch_span_walk(const uint64_t* heads, const int32_t* len, const int32_t* skip,
                     const uint32_t* seed, const WalkRegionHost* regions, int nreg, uint32_t n,
                     bool pseudo, uint64_t* off_out, uint32_t* len_out, uint32_t* seed_out,
                     unsigned long long* stats, hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (nreg < 1 || nreg > kWalkRegionsMax) return UINET_CKSUM_EINVAL;
  UINET_LAUNCH(k_span_walk, dim3((n + 255) / 256), dim3(256), 0, stream, heads, len, skip, seed,
               regions, nreg, n, pseudo ? 1 : 0, off_out, len_out, seed_out, stats);
  return check_launch();
}

int launch_span_rebase(uint64_t* off, const uint32_t* len, uint32_t n, uint64_t gbase,
                       hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  UINET_LAUNCH(k_span_rebase, dim3((n + 255) / 256), dim3(256), 0, stream, off, len, n, gbase);
  return check_launch();
}

int launch_walk_mbufs(const uint64_t* heads, const int32_t* len, const int32_t* skip,
                      const uint32_t* seed, const WalkRegionHost* regions, int nreg, uint32_t n,
                      uint32_t K, uint32_t seg_base, uint64_t lo_dev, bool pseudo, uint64_t* seg_off,
                      uint32_t* seg_len, uint32_t* pkt_seg, uint32_t* len_out, uint32_t* skip_out,
                      uint32_t* seed_out, uint32_t* status, hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (nreg < 1 || nreg > kWalkRegionsMax || K == 0 ||
      (uint64_t)seg_base + (uint64_t)n * K > 0xffffffffull)
    return UINET_CKSUM_EINVAL;
  // two lanes per packet, every chain in flight at once (up to 1 M packets
  // per pass of the grid)
  const uint64_t blocks64 = (2 * (uint64_t)n + 255) / 256;
  const int blocks = (int)(blocks64 < 8192 ? blocks64 : 8192);
  UINET_LAUNCH(k_walk_mbufs, dim3(blocks), dim3(256), 0, stream, heads, len, skip, seed,
               regions, nreg, n, K, seg_base, lo_dev, pseudo ? 1 : 0,
               seg_off, seg_len, pkt_seg, len_out, skip_out, seed_out, status);
  return check_launch();
}

}  // namespace uinet
