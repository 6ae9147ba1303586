// Host run of walk_xlate (libuinet_amd/csrc/walk_xlate.h), the translation the
// device chain walk applies to every mbuf and data pointer before the GPU
// reads it: random sorted, non-overlapping region tables (adjacent ones
// included) and queries around every boundary, against a linear scan.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#include "walk_xlate.h"

using uinet::WalkRegionHost;

static bool brute(const std::vector<WalkRegionHost>& R, uint64_t a, uint64_t n, uint64_t* dev) {
  for (const WalkRegionHost& r : R)
    if (a >= r.base && a < r.end && n <= r.end - a) {
      *dev = a + (uint64_t)r.delta;
      return true;
    }
  return false;
}

int main() {
  std::mt19937_64 rng(12345);
  long checks = 0, bad = 0, hits = 0;
  for (int t = 0; t < 4000; t++) {
    const int nreg = (int)(rng() % 9);  // 0..8 regions
    std::vector<WalkRegionHost> R;
    uint64_t cur = (rng() % 4) ? (rng() % (1ull << 40)) : (~0ull - (1ull << 20));
    for (int k = 0; k < nreg; k++) {
      cur += (rng() % 3 == 0) ? 0 : 1 + rng() % 5000;  // adjacent or a gap
      const uint64_t len = 1 + rng() % 8192;
      if (cur + len < cur) break;  // top of the address space
      R.push_back({cur, cur + len, (int64_t)(rng() % (1ull << 44)) - (1ll << 43)});
      cur += len;
    }
    std::vector<uint64_t> probes;
    for (const WalkRegionHost& r : R)
      for (uint64_t p : {r.base, r.end, r.base - 1, r.end - 1, r.base + 1, r.end + 1,
                         r.end + 4096, r.base + (r.end - r.base) / 2})
        probes.push_back(p);
    for (int k = 0; k < 16; k++) probes.push_back(rng());
    probes.push_back(0);
    probes.push_back(~0ull);
    for (uint64_t a : probes)
      for (uint64_t n : {1ull, 15ull, 32ull, 1500ull, 9000ull, 1ull << 62, ~0ull}) {
        uint64_t d1 = 0, d2 = 0;
        const bool g = uinet::walk_xlate(R.data(), (int)R.size(), a, n, &d1);
        const bool w = brute(R, a, n, &d2);
        checks++;
        hits += w;
        if (g != w || (g && d1 != d2)) {
          if (bad++ < 5)
            printf("mismatch: a=%llx n=%llx got %d want %d\n", (unsigned long long)a,
                   (unsigned long long)n, g, w);
        }
      }
  }
  printf("checks=%ld hits=%ld bad=%ld\n", checks, hits, bad);
  return bad ? 1 : 0;
}
