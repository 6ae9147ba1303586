// Read-bandwidth microbenchmark for MI355X (measurement tool, not product):
// what a pure streaming read of a >= 1.5 GB buffer achieves with 16-byte
// loads, by grid size, loads in flight per lane and cache policy.  Sets the
// "achievable" ceiling the checksum kernel is compared against.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ p, uint64_t n16,
                                              uint32_t* __restrict__ sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  uint64_t i = tid;
  for (; i + (U - 1) * nthr < n16; i += U * nthr) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + i + u * nthr));
        v[u] = make_uint4(t.x, t.y, t.z, t.w);
      } else {
        v[u] = p[i + u * nthr];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  for (; i < n16; i += nthr) { uint4 v = p[i]; acc += v.x + v.y + v.z + v.w; }
  if (acc == 0x12345678u) sink[0] = acc;  // keep the loads live
}

// Contiguous-chunk variant: each block streams its own contiguous slice
// (locality per CU) instead of a grid-wide stride.
template <int U>
__global__ __launch_bounds__(256) void k_read_chunk(const uint4* __restrict__ p, uint64_t n16,
                                                    uint32_t* __restrict__ sink) {
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t b0 = blockIdx.x * per, b1 = min(n16, b0 + per);
  uint32_t acc = 0;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += U * 256) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = min(i + u * 256, b1 - 1);
      v[u] = p[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}


// Tile variant (the span kernel's access shape): logical tile t is 256 x U
// consecutive 16-B chunks, one-shot or grid-stride over tiles; nt loads; with
// `remap` block b takes logical id (b % 8) * (grid / 8) + b / 8 so each XCD
// streams one contiguous band.
template <int U, bool REMAP>
__global__ __launch_bounds__(256) void k_read_tile(const uint4* __restrict__ p, uint64_t n16,
                                                   uint32_t* __restrict__ sink) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t g = gridDim.x, per = g / 8;
  uint32_t b = blockIdx.x;
  if (REMAP && b < 8 * per) b = (b % 8) * per + b / 8;
  const uint64_t tiles = (n16 + 256 * U - 1) / (256 * U);
  uint32_t acc = 0;
  for (uint64_t t = b; t < tiles; t += g) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = min(t * 256 * U + (uint64_t)u * 256 + threadIdx.x, n16 - 1);
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + i));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
  }
  return best;
}

// Tile read with K dependent-free integer multiply-adds per 16-B chunk and
// lane: the arithmetic load of a checksum kernel without its memory shape.
template <int K>
__global__ __launch_bounds__(256) void k_read_valu(const uint4* __restrict__ p, uint64_t n16,
                                                   uint32_t* __restrict__ sink) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t tiles = (n16 + 1023) / 1024;
  uint32_t acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3;
  for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t i = min(t * 1024 + (uint64_t)u * 256 + threadIdx.x, n16 - 1);
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + i));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int k = 0; k < K; k += 4) {
        acc0 = acc0 * 3u + v[u].x;
        acc1 = acc1 * 5u + v[u].y;
        acc2 = acc2 * 7u + v[u].z;
        acc3 = acc3 * 9u + v[u].w;
      }
      if (K == 0) acc0 += v[u].x + v[u].y + v[u].z + v[u].w;
    }
  }
  if ((acc0 ^ acc1 ^ acc2 ^ acc3) == 0x12345678u) sink[0] = acc0;
}

template <int K>
static int cold_valu(int n) {
  const uint64_t bytes = 1572864000ull, n16 = bytes / 16;
  uint4* p;
  uint32_t* sink;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(p, 0x5a, bytes));
  const int grid = (int)((n16 + 1023) / 1024);
  k_read_valu<K><<<grid, 256>>>(p, n16, sink);
  CK(hipDeviceSynchronize());
  usleep(2000000);
  hipEvent_t* ev = (hipEvent_t*)malloc(sizeof(hipEvent_t) * (n + 1));
  for (int i = 0; i <= n; ++i) CK(hipEventCreate(&ev[i]));
  CK(hipEventRecord(ev[0]));
  for (int i = 0; i < n; ++i) {
    k_read_valu<K><<<grid, 256>>>(p, n16, sink);
    CK(hipEventRecord(ev[i + 1]));
  }
  CK(hipEventSynchronize(ev[n]));
  printf("{\"kernel\": \"read_valu%d\", \"ms\": [", K);
  for (int i = 0; i < n; ++i) {
    float ms;
    CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
    printf("%s%.5f", i ? ", " : "", ms);
  }
  printf("]}\n");
  CK(hipFree(p));
  CK(hipFree(sink));
  return 0;
}

// `hbm_read cold N`: after 2 s idle, N back-to-back launches of the best
// pure-read shape (tile_u4, one tile per block) over config 2's 1.5 GB, each
// bracketed by events -- the cold-start profile of a kernel with next to no
// arithmetic, beside tools/cold_start.py's for the checksum kernels.
static int cold(int n) {
  const uint64_t bytes = 1572864000ull, n16 = bytes / 16;
  uint4* p;
  uint32_t* sink;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(p, 0x5a, bytes));
  CK(hipDeviceSynchronize());
  const int grid = (int)((n16 + 1023) / 1024);
  k_read_tile<4, false><<<grid, 256>>>(p, n16, sink);  // first touch, untimed
  CK(hipDeviceSynchronize());
  usleep(2000000);
  hipEvent_t* ev = (hipEvent_t*)malloc(sizeof(hipEvent_t) * (n + 1));
  for (int i = 0; i <= n; ++i) CK(hipEventCreate(&ev[i]));
  CK(hipEventRecord(ev[0]));
  for (int i = 0; i < n; ++i) {
    k_read_tile<4, false><<<grid, 256>>>(p, n16, sink);
    CK(hipEventRecord(ev[i + 1]));
  }
  CK(hipEventSynchronize(ev[n]));
  printf("{\"kernel\": \"tile_u4\", \"grid\": %d, \"bytes\": %llu, \"ms\": [", grid,
         (unsigned long long)bytes);
  for (int i = 0; i < n; ++i) {
    float ms;
    CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
    printf("%s%.5f", i ? ", " : "", ms);
  }
  printf("]}\n");
  return 0;
}

// Independent (not chained) 32-B reads at random 256-B slots: lanes 2k and
// 2k + 1 read the two 16-B halves of slot hash(k), the device walk's access
// shape without its dependency -- the link's rate for scattered line reads.
__global__ __launch_bounds__(256) void k_read_slots(const uint4* __restrict__ p, uint64_t nslot,
                                                    uint64_t reads, uint32_t* __restrict__ sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = tid; i < 2 * reads; i += nthr) {
    uint64_t h = (i >> 1) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    const uint64_t slot = h % nslot;
    const uint4 v = p[slot * 16 + (i & 1)];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// One lane per random 256-B slot, loading C consecutive 16-B chunks of its
// first 128-B line with C independent loads issued back to back (the hook
// parse's window copy): do concurrent misses to one line of host memory
// merge in L2, or does each become a read over the link?
template <int C>
__global__ __launch_bounds__(256) void k_read_line_chunks(const uint4* __restrict__ p,
                                                          uint64_t nslot, uint64_t lines,
                                                          uint32_t* __restrict__ sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = tid; i < lines; i += nthr) {
    uint64_t h = i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    const uint4* q = p + (h % nslot) * 16;
    uint4 v[C];
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = q[c];
#pragma unroll
    for (int c = 0; c < C; ++c) acc += v[c].x + v[c].y + v[c].z + v[c].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// `hbm_read host BYTES`: the same reads over registered host memory (the
// zero-copy and device-walk paths' source), through its device alias, beside
// a hipMemcpy of the buffer to HBM: the PCIe ceiling the host-resident paths
// are measured against.
static int host(uint64_t bytes) {
  const uint64_t n16 = bytes / 16;
  void* h = nullptr;
  if (posix_memalign(&h, 4096, bytes)) return 1;
  memset(h, 0x5a, bytes);
  CK(hipHostRegister(h, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  uint4* p;
  CK(hipHostGetDevicePointer((void**)&p, h, 0));
  uint4* d;
  uint32_t* sink;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&sink, 64));
  printf("{\"bytes\": %llu, \"memory\": \"registered host\", \"results\": [\n",
         (unsigned long long)bytes);
  bool first = true;
  auto report = [&](const char* name, int grid, float ms, double moved, double n_reads) {
    printf("%s {\"kernel\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.2f, \"Mreads_per_s\": %.1f}\n",
           first ? "" : ",", name, grid, ms, moved / (ms * 1e-3) / 1e9,
           n_reads / (ms * 1e-3) / 1e6);
    first = false;
    fflush(stdout);
  };
  report("hipMemcpy_h2d", 0, time_it([&] { CK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice)); }, 5),
         (double)bytes, 0);
  const int grids[] = {1024, 4096, 16384};
  for (int g : grids) {
    report("stride_u4", g, time_it([&] { k_read<4, false><<<g, 256>>>(p, n16, sink); }, 5),
           (double)bytes, (double)bytes / 64);
    report("stride_u8", g, time_it([&] { k_read<8, false><<<g, 256>>>(p, n16, sink); }, 5),
           (double)bytes, (double)bytes / 64);
  }
  const uint64_t tiles = (n16 + 1023) / 1024;
  report("tile_u4", (int)tiles,
         time_it([&] { k_read_tile<4, false><<<(int)tiles, 256>>>(p, n16, sink); }, 5),
         (double)bytes, (double)bytes / 64);
  const uint64_t nslot = bytes / 256, reads = 4u << 20;
  for (int g : grids)
    report("slots_32B", g,
           time_it([&] { k_read_slots<<<g, 256>>>(p, nslot, reads, sink); }, 5),
           (double)reads * 32, (double)reads);
  // the last column is lines per second here
  const uint64_t lines = 2u << 20;
  const int gl = (int)(lines / 256);
  report("line_chunks_1", gl,
         time_it([&] { k_read_line_chunks<1><<<gl, 256>>>(p, nslot, lines, sink); }, 5),
         (double)lines * 128, (double)lines);
  report("line_chunks_2", gl,
         time_it([&] { k_read_line_chunks<2><<<gl, 256>>>(p, nslot, lines, sink); }, 5),
         (double)lines * 128, (double)lines);
  report("line_chunks_4", gl,
         time_it([&] { k_read_line_chunks<4><<<gl, 256>>>(p, nslot, lines, sink); }, 5),
         (double)lines * 128, (double)lines);
  report("line_chunks_8", gl,
         time_it([&] { k_read_line_chunks<8><<<gl, 256>>>(p, nslot, lines, sink); }, 5),
         (double)lines * 128, (double)lines);
  printf("]}\n");
  CK(hipHostUnregister(h));
  free(h);
  return 0;
}

// 32-B reads at 256-B slots of an HBM buffer: the mbuf header access of the
// HBM chain walk (uinet_cksum_mbufs) without its dependency.  Sequential
// slots (mbufs in chain order, one 32-B header per 256-B record) and random
// slots; run under rocprofv3 --pmc FETCH_SIZE it calibrates what one such
// read costs in fetched bytes.
__global__ __launch_bounds__(256) void k_read_slots_seq(const uint4* __restrict__ p,
                                                        uint64_t reads,
                                                        uint32_t* __restrict__ sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = tid; i < 2 * reads; i += nthr) {
    const uint4 v = p[(i >> 1) * 16 + (i & 1)];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

static int hbm_slots(uint64_t bytes) {
  uint4* p;
  uint32_t* sink;
  CK(hipMalloc(&p, bytes));
  CK(hipMemset(p, 0x5a, bytes));
  CK(hipMalloc(&sink, 64));
  const uint64_t nslot = bytes / 256, reads = nslot;
  printf("{\"bytes\": %llu, \"memory\": \"HBM\", \"slots\": %llu, \"results\": [\n",
         (unsigned long long)bytes, (unsigned long long)nslot);
  bool first = true;
  for (int g : {4096, 16384, 65536}) {
    const float ms_seq = time_it([&] { k_read_slots_seq<<<g, 256>>>(p, reads, sink); }, 5);
    const float ms_rnd = time_it([&] { k_read_slots<<<g, 256>>>(p, nslot, reads, sink); }, 5);
    printf("%s {\"grid\": %d, \"seq_ms\": %.4f, \"seq_Mreads_per_s\": %.1f, \"rnd_ms\": %.4f, "
           "\"rnd_Mreads_per_s\": %.1f}\n", first ? "" : ",", g, ms_seq,
           reads / (ms_seq * 1e-3) / 1e6, ms_rnd, reads / (ms_rnd * 1e-3) / 1e6);
    first = false;
  }
  printf("]}\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 2 && !strcmp(argv[1], "host")) return host(strtoull(argv[2], 0, 0));
  if (argc > 2 && !strcmp(argv[1], "slots")) return hbm_slots(strtoull(argv[2], 0, 0));
  if (argc > 2 && !strcmp(argv[1], "cold")) return cold(atoi(argv[2]));
  if (argc > 3 && !strcmp(argv[1], "cold_valu")) {
    const int k = atoi(argv[3]), n = atoi(argv[2]);
    return k >= 64 ? cold_valu<64>(n) : k >= 32 ? cold_valu<32>(n) : k >= 16 ? cold_valu<16>(n)
                                                                            : cold_valu<0>(n);
  }
  const uint64_t bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : (1572864000ull));
  const uint64_t n16 = bytes / 16;
  uint4* p; uint32_t* sink;
  CK(hipMalloc(&p, bytes)); CK(hipMalloc(&sink, 64));
  CK(hipMemset(p, 0x5a, bytes));
  printf("{\"bytes\": %llu, \"results\": [\n", (unsigned long long)bytes);
  bool first = true;
  auto report = [&](const char* name, int grid, float ms) {
    printf("%s {\"kernel\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", first ? "" : ",",
           name, grid, ms, bytes / (ms * 1e-3) / 1e9);
    first = false;
  };
  const int grids[] = {1024, 2048, 4096, 8192, 16384, 65536};
  for (int g : grids) {
    report("stride_u1", g, time_it([&] { k_read<1, false><<<g, 256>>>(p, n16, sink); }, 20));
    report("stride_u2", g, time_it([&] { k_read<2, false><<<g, 256>>>(p, n16, sink); }, 20));
    report("stride_u4", g, time_it([&] { k_read<4, false><<<g, 256>>>(p, n16, sink); }, 20));
    report("stride_u8", g, time_it([&] { k_read<8, false><<<g, 256>>>(p, n16, sink); }, 20));
    report("stride_u4_nt", g, time_it([&] { k_read<4, true><<<g, 256>>>(p, n16, sink); }, 20));
    report("chunk_u4", g, time_it([&] { k_read_chunk<4><<<g, 256>>>(p, n16, sink); }, 20));
    report("chunk_u8", g, time_it([&] { k_read_chunk<8><<<g, 256>>>(p, n16, sink); }, 20));
  }
  {
    const uint64_t t4 = (n16 + 1023) / 1024, t8 = (n16 + 2047) / 2048, t2 = (n16 + 511) / 512;
    const int caps[] = {0, 256 * 64, 256 * 128, 256 * 256};
    for (int cap : caps) {
      auto G = [&](uint64_t t) { return (int)(cap && t > (uint64_t)cap ? cap : t); };
      report(cap ? "tile_u2_gs" : "tile_u2", G(t2), time_it([&] { k_read_tile<2, false><<<G(t2), 256>>>(p, n16, sink); }, 20));
      report(cap ? "tile_u4_gs" : "tile_u4", G(t4), time_it([&] { k_read_tile<4, false><<<G(t4), 256>>>(p, n16, sink); }, 20));
      report(cap ? "tile_u8_gs" : "tile_u8", G(t8), time_it([&] { k_read_tile<8, false><<<G(t8), 256>>>(p, n16, sink); }, 20));
      report(cap ? "tile_u2_xcd_gs" : "tile_u2_xcd", G(t2), time_it([&] { k_read_tile<2, true><<<G(t2), 256>>>(p, n16, sink); }, 20));
      report(cap ? "tile_u4_xcd_gs" : "tile_u4_xcd", G(t4), time_it([&] { k_read_tile<4, true><<<G(t4), 256>>>(p, n16, sink); }, 20));
      report(cap ? "tile_u8_xcd_gs" : "tile_u8_xcd", G(t8), time_it([&] { k_read_tile<8, true><<<G(t8), 256>>>(p, n16, sink); }, 20));
    }
  }
  printf("]}\n");
  return 0;
}
