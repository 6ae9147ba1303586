// Stress test of libuinet_amd/csrc/host_pool.h (host-only, no HIP): several
// caller threads run batches concurrently with varying job and thread
// counts; every job must run exactly once per batch.
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "../../libuinet_amd/csrc/host_pool.h"

int main() {
  std::atomic<long> bad{0};
  auto caller = [&](int t) {
    for (int it = 0; it < 2000; it++) {
      const int jobs = 1 + (it * 7 + t) % 37, threads = 1 + (it + t) % 9;
      std::vector<std::atomic<int>> hit(jobs);
      for (auto& h : hit) h = 0;
      uinet::host_pool().run(jobs, threads, [&](int j) { hit[j]++; });
      for (auto& h : hit) bad += h.load() != 1;
    }
  };
  std::vector<std::thread> ts;
  for (int t = 0; t < 4; t++) ts.emplace_back(caller, t);
  for (auto& t : ts) t.join();
  printf("bad=%ld\n", bad.load());
  return bad.load() != 0;
}
