// Host-address -> device-address translation of the device chain walk
// (cksum_walk.hip), in a header of its own so the host test
// tests/native/walk_xlate_test.cpp runs the very same code on the CPU: an
// address this accepts is read by the GPU, so a wrong answer here is a GPU
// memory fault, not a wrong checksum.
#pragma once

#include <stdint.h>

#ifdef __HIPCC__
#define UINET_HD __host__ __device__
#else
#define UINET_HD
#endif

namespace uinet {

// Host range [base, end) is readable by the device at host address + delta.
struct WalkRegionHost {
  uint64_t base, end;
  int64_t delta;
};

// Device address of host bytes [a, a + n), n > 0, if one region holds them
// all.  R: nreg regions sorted by base, non-overlapping.
UINET_HD inline bool walk_xlate(const WalkRegionHost* R, int nreg, uint64_t a, uint64_t n,
                                uint64_t* dev) {
  int lo = 0, hi = nreg;
  while (lo < hi) {  // the last region with base <= a
    const int mid = (lo + hi) >> 1;
    if (R[mid].base <= a) lo = mid + 1; else hi = mid;
  }
  if (lo == 0) return false;
  const WalkRegionHost& r = R[lo - 1];
  if (a >= r.end || n > r.end - a) return false;  // r.base <= a by the search
  *dev = a + (uint64_t)r.delta;
  return true;
}

}  // namespace uinet
