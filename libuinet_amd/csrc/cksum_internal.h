// Internal interfaces between the HIP kernels (cksum_kernels.hip) and the
// host side of the engine (cksum_api.hip).  Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "uinet_cksum.h"
#include "walk_xlate.h"

namespace uinet {

// Process-wide performance knobs (uinet_cksum_set_tuning); seeded from the
// environment on first use.  0 = "use the kernel's default".  tuning() returns
// a snapshot of the live values (relaxed atomics in cksum_api.hip).
struct Tuning {
  int blocks_per_cu;   // grid-stride width
  int host_threads;    // host-mbuf batch walk/pack threads, 1..64
  int chains_long;     // flat chains: segments of >= this many 16-B chunks stream
                       // wave-wide (0 = never)
  int chains_wide;     // chains: 0 = a wave per packet (k_chains_wide) when the mean
                       // segment is 4-9 KiB, 1 = never, 2 = always
  int xcd_remap;       // span kernels: XCD-banded block order (0/1)
  int multi_gather;    // uinet_cksum_spans_multi: 0 RCCL gather when it applies, 1 peer copies
  int span_fast;       // host-mbuf batches whose sums lie in the first mbuf: 1 the host
                       // reads the heads and writes span descriptors, 2 the GPU reads
                       // the heads when the mbufs are registered, 0 off
  int walk_device;     // host-mbuf batches in registered memory, 0 the host walks them,
                       // else the GPU: 3 walks and folds in one launch (cksum_mbufs.hip),
                       // 2 walks into a segment list first (cksum_walk.hip), 1 = 2 for
                       // the chain batches and 3 for the offload hooks
};
Tuning tuning();

// Records the HIP error (if any) of the last launch on this thread and maps
// it to a UINET_CKSUM_* code.
int check_launch();
int record_hip(hipError_t e);

// Every kernel launch goes through UINET_LAUNCH, which notes the kernel's
// host stub for uinet_cksum_last_kernel() (the instantiation a launch on this
// thread last started: bench.py matches its profiler traffic by that name).
void note_kernel(const void* host_stub);
#define UINET_LAUNCH(K, ...)                               \
  do {                                                     \
    ::uinet::note_kernel(reinterpret_cast<const void*>(&K)); \
    hipLaunchKernelGGL(K, __VA_ARGS__);                    \
  } while (0)

int launch_spans(const void* base, const uint64_t* off, const uint32_t* len,
                 const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                 uint32_t flags, uint32_t len_hint, hipStream_t stream);
int launch_strided(const void* base, uint64_t pkt_stride, uint32_t len, const uint32_t* seed,
                   uint16_t* out, uint32_t n, uint32_t flags, hipStream_t stream);
// Packed span descriptors (uinet_cksum_spans32): u32 offsets, u16 lengths.
int launch_spans32(const void* base, const uint32_t* off, const uint16_t* len,
                   const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                   uint32_t flags, uint32_t len_hint, hipStream_t stream);
// k_spans_lean (cksum_spans.hip): G = 32 or 64 lanes per packet; strided
// takes packet i at base + i * stride, slen bytes (off / len unused, wide
// descriptor types only); blocks_cu 0 = two steps per wave, else at most
// blocks_cu blocks per CU; temporal: ordinary packet loads (no parity
// array, not strided), for bytes read over PCIe.  Instantiated for
// (uint64_t, uint32_t) and (uint32_t, uint16_t) descriptors.
template <typename OffT, typename LenT>
int launch_spans_lean(const void* base, const OffT* off, const LenT* len,
                      const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                      uint32_t flags, int g, int u, bool strided, uint64_t stride, uint32_t slen,
                      int blocks_cu, hipStream_t stream, bool temporal = false);
// Internal flag bit for launch_spans / launch_spans32 (never a UINET_CKSUM_F_*
// value; the public entry points clear it): the packet bytes lie in
// registered host memory, read over PCIe.
constexpr uint32_t kFlagHostBytes = 0x80000000u;
// k_spans_quad (cksum_spans.hip): 4 lanes per packet, U = 1 or 2 chunk
// slots per lane, for small packets.  Same instantiations.
template <typename OffT, typename LenT>
int launch_spans_quad(const void* base, const OffT* off, const LenT* len,
                      const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                      uint32_t flags, int u, bool strided, uint64_t stride, uint32_t slen,
                      int blocks_cu, hipStream_t stream);
// k_strided_dense (cksum_spans.hip): small strided packets laid nearly back
// to back (32 <= stride <= 256, stride - len <= stride / 4); returns 1 without
// launching when the shape does not fit.
int launch_strided_dense(const void* base, uint64_t stride, uint32_t len, const uint32_t* seed,
                         uint16_t* out, uint32_t n, uint32_t flags, int blocks_cu,
                         hipStream_t stream);
int launch_chains(const void* base, const uint64_t* seg_off, const uint32_t* seg_len,
                  const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                  const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                  uint32_t len_hint, hipStream_t stream);
int launch_chains32(const void* base, const uint32_t* seg_off, const uint16_t* seg_len,
                    const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                    const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                    uint32_t len_hint, hipStream_t stream);

// Device-side chain walk (cksum_walk.hip) for host-mbuf batches whose mbufs
// and bytes lie in registered host memory.  Host range [base, end) is read by
// the device at host address + delta; regions sorted by base.
constexpr int kWalkRegionsMax = 256;
constexpr uint32_t kWalkFallback = 1;  // status[0]: a job the host walk must take
constexpr uint32_t kWalkUnmapped = 2;  // status[0]: a pointer outside the regions
constexpr uint32_t kWalkKMax = 4096;   // segment-list rows: longer chains take the host walk
// Packet i's chain (heads[i], len[i], skip[i], seed[i]; seed may be NULL) into
// row i of a K-slot segment list in HBM (seg_off relative to lo_dev; pkt_seg
// [i] = seg_base + i * K, the row's index in a list of which seg_off / seg_len
// are row 0), plus u32 len / skip / seed arrays for launch_chains.  status (2 u32
// in device memory, zeroed by the caller): [0] kWalk* bits, [1] the longest
// chain when one exceeds K.  `pseudo`: the in_cksum_pseudo_header form (skip
// = off0 must lie within the first mbuf).
int launch_walk_mbufs(const uint64_t* heads, const int32_t* len, const int32_t* skip,
                      const uint32_t* seed, const WalkRegionHost* regions, int nreg, uint32_t n,
                      uint32_t K, uint32_t seg_base, uint64_t lo_dev, bool pseudo, uint64_t* seg_off,
                      uint32_t* seg_len, uint32_t* pkt_seg, uint32_t* len_out, uint32_t* skip_out,
                      uint32_t* seed_out, uint32_t* status, hipStream_t stream);

// The single-mbuf span walk (cksum_walk.hip, k_span_walk): packet i's span
// from its head mbuf, as a device address (off_out) and length, or status
// bits in stats[3] when the batch is not that shape; stats (6 u64, set by the
// caller to {~0, 0, 0, 0, ~0, 0}): lowest span address, highest span end,
// summed bytes, status, lowest and highest region index.  launch_span_rebase:
// off[i] -= gbase where len[i] != 0, else 0.
int launch_span_walk(const uint64_t* heads, const int32_t* len, const int32_t* skip,
                     const uint32_t* seed, const WalkRegionHost* regions, int nreg, uint32_t n,
                     bool pseudo, uint64_t* off_out, uint32_t* len_out, uint32_t* seed_out,
                     unsigned long long* stats, hipStream_t stream);
int launch_span_rebase(uint64_t* off, const uint32_t* len, uint32_t n, uint64_t gbase,
                       hipStream_t stream);

// The fused mbuf walk + fold (cksum_mbufs.hip).  launch_mbufs: chains in
// device memory (uinet_cksum_mbufs; status: UINET_CKSUM_MBUF_* bits).
// launch_mbufs_xlate: chains and bytes in registered host memory read through
// the region table (status[0]: kWalkUnmapped / kWalkFallback -- the host then
// redoes the batch; `pseudo`: the first mbuf must hold skip).
int launch_mbufs(const uint64_t* heads, const int32_t* len, const int32_t* skip,
                 const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                 uint32_t seg_hint, uint32_t* status, hipStream_t stream);
int launch_mbufs_xlate(const uint64_t* heads, const int32_t* len, const int32_t* skip,
                       const uint32_t* seed, const WalkRegionHost* regions, int nreg, bool pseudo,
                       uint16_t* out, uint32_t n, uint32_t flags, uint32_t* status,
                       hipStream_t stream);

// Driver hooks on the device (cksum_hookdev.hip): k_hook_parse writes two jobs
// per frame (jm / jl / js / jd: 2n entries) and its plan / frame records
// (hook_plan_bytes / hook_frame_bytes each); k_hook_apply writes the verdicts
// into the mbufs and st_out[n], unless status[0] is set or status[1] > K.
size_t hook_plan_bytes(bool rx);
size_t hook_frame_bytes();
int launch_hook_parse(bool rx, const uint64_t* mv, uint32_t n, int l2len,
                      const WalkRegionHost* regions, int nreg, uint64_t* jm, int32_t* jl,
                      int32_t* js, uint32_t* jd, void* plans, void* frames, uint32_t* status,
                      hipStream_t stream);
int launch_hook_apply(bool rx, const void* plans, const void* frames, const uint16_t* res,
                      uint32_t n, uint32_t K, const uint32_t* status, uint8_t* st_out,
                      hipStream_t stream);

}  // namespace uinet
