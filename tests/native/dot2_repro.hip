// Minimal reproducer of the hipcc (ROCm 7.2, gfx950) bit-cast miscompile the
// chunk sums once hit (profiles/r03/NOTES.md, r03s3a), and the same loop on
// the engine's shipped helper.  Compiled to ISA (never run) by
// tests/test_dot2_isa.py, which reads the v_dot2_u32_u16 operands.
//
// k_elem:   __builtin_bit_cast(us2, v.y) taken straight off an ext-vector
//           element.  In this context hipcc reads element x four times.
// k_helper: chunk_halves() from libuinet_amd/csrc/cksum_device.h (the words
//           copied out first), used by every span and chain kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cksum_device.h"

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t elem_sum(uinet::u32x4 v, uint32_t acc) {
  const us2 one = {1, 1};
  acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, v.x), one, acc, false);
  acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, v.y), one, acc, false);
  acc = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, v.z), one, acc, false);
  return __builtin_amdgcn_udot2(__builtin_bit_cast(us2, v.w), one, acc, false);
}

// The long-segment stream's shape: two chunks per lane in flight, a clamped
// first load, a wave-uniform whole-step branch.
template <bool kHelper>
__device__ __forceinline__ void stream(const uint8_t* cb, uint32_t nc, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  uint64_t lsum = 0;
  for (uint32_t k0 = 0; k0 < nc; k0 += 128) {
    uinet::u32x4 v[2];
    for (int u = 0; u < 2; ++u)
      if (u == 0 || k0 + 64u * u < nc)
        v[u] = uinet::load_chunk(cb + 16ull * min(k0 + (uint32_t)(u * 64 + lane), nc - 1));
    uint32_t t = 0;
    if (k0 != 0 && k0 + 128 < nc) {
      for (int u = 0; u < 2; ++u) t = kHelper ? uinet::chunk_halves(v[u], t) : elem_sum(v[u], t);
    } else {
      for (int u = 0; u < 2; ++u)
        if (u == 0 || k0 + 64u * u < nc) t += v[u].x & 0xff;
    }
    lsum += t;
  }
  out[threadIdx.x] = (uint32_t)lsum;
}

extern "C" __global__ void k_elem(const uint8_t* cb, uint32_t nc, uint32_t* out) {
  stream<false>(cb, nc, out);
}
extern "C" __global__ void k_helper(const uint8_t* cb, uint32_t nc, uint32_t* out) {
  stream<true>(cb, nc, out);
}
