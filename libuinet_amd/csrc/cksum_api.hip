// Host side of the engine: the C ABI of include/uinet_cksum.h.
//
//  * Device-resident descriptor API: argument checks + one launch.
//  * Host-mbuf batch API: walks each chain exactly like the reference
//    (/root/reference/sys/amd64/amd64/in_cksum.c:193-232 for in_cksum_skip,
//    :241-276 for in_cksum_pseudo_header, :278-285 for in_cksum_hdr), packs
//    the bytes each packet contributes into pinned staging (one contiguous
//    run per packet, logical order, 16-byte aligned starts), ships staging
//    to HBM with one copy, folds it with one launch of the span kernel and
//    copies the 16-bit results back.
//  * Per-call drop-in ABI: a batch of one.  The reference functions have no
//    error channel, so a HIP failure here is reported on stderr and aborts
//    rather than returning a made-up checksum.
//
// Threading: the reference checksum is fully reentrant; here
// every calling thread gets its own stream and staging buffers (thread_local),
// so concurrent RX/TX threads never share state and take no locks.
#include <hip/hip_runtime.h>

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "cksum_internal.h"

namespace uinet {

// The three fields of struct m_hdr the checksum reads
// (sys/sys/mbuf.h:90-98): m_next@0, m_data@16, m_len@24.
struct MbufHdr {
  MbufHdr* m_next;
  void* m_nextpkt;
  const uint8_t* m_data;
  int m_len;
};
static_assert(offsetof(MbufHdr, m_next) == 0, "m_next offset");
static_assert(offsetof(MbufHdr, m_data) == 16, "m_data offset");
static_assert(offsetof(MbufHdr, m_len) == 24, "m_len offset");

static thread_local int t_last_hip = 0;

int record_hip(hipError_t e) {
  if (e == hipSuccess) return UINET_CKSUM_OK;
  t_last_hip = (int)e;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return UINET_CKSUM_ENODEV;
  if (e == hipErrorOutOfMemory) return UINET_CKSUM_ENOMEM;
  return UINET_CKSUM_EHIP;
}

int check_launch() { return record_hip(hipGetLastError()); }

static Tuning& tuning_rw() {
  static Tuning t = [] {
    Tuning x{0, 0, 2};
    if (const char* e = getenv("UINET_CKSUM_BLOCKS_PER_CU")) {
      const int v = atoi(e);
      x.blocks_per_cu = (v > 0 && v <= 4096) ? v : 0;
    }
    if (const char* e = getenv("UINET_CKSUM_CHAINS")) x.chains_variant = e[0] == 's' ? 1 : 0;
    if (const char* e = getenv("UINET_CKSUM_CHAINS_PASS")) {
      const int v = atoi(e);
      if (v == 2 || v == 4 || v == 8) x.chains_pass = v;
    }
    return x;
  }();
  return t;
}

const Tuning& tuning() { return tuning_rw(); }

namespace {

uint32_t fold16_host(uint64_t s) {
  while (s >> 16) s = (s & 0xffff) + (s >> 16);
  return (uint32_t)s;
}

uint16_t bswap16(uint16_t x) { return (uint16_t)((x << 8) | (x >> 8)); }

// ---- per-thread engine context --------------------------------------------

struct Ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* h_buf = nullptr;  // pinned: descriptors, then packet bytes
  size_t h_cap = 0;
  uint8_t* d_buf = nullptr;  // device mirror of h_buf
  size_t d_cap = 0;
  uint16_t* h_out = nullptr;  // pinned results
  uint16_t* d_out = nullptr;
  size_t out_cap = 0;
};

// Staging is intentionally not released at thread exit: HIP may already be
// torn down when the main thread's thread_local destructors run.
thread_local Ctx t_ctx;

int ctx_ready(Ctx& c) {
  int dev = 0;
  int rc = record_hip(hipGetDevice(&dev));
  if (rc) return rc;
  if (c.device == dev && c.stream) return UINET_CKSUM_OK;
  if (c.device != dev && c.stream) {  // thread switched devices: start over
    c = Ctx();
  }
  rc = record_hip(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
  if (rc) return rc;
  c.device = dev;
  return UINET_CKSUM_OK;
}

int ctx_reserve(Ctx& c, size_t bytes, size_t nout) {
  if (bytes > c.h_cap) {
    size_t cap = c.h_cap ? c.h_cap : (1u << 20);
    while (cap < bytes) cap *= 2;
    if (c.h_buf) (void)hipHostFree(c.h_buf);
    if (c.d_buf) (void)hipFree(c.d_buf);
    c.h_buf = nullptr;
    c.d_buf = nullptr;
    c.h_cap = c.d_cap = 0;
    int rc = record_hip(hipHostMalloc((void**)&c.h_buf, cap, hipHostMallocDefault));
    if (rc) return rc;
    rc = record_hip(hipMalloc((void**)&c.d_buf, cap));
    if (rc) return rc;
    c.h_cap = c.d_cap = cap;
  }
  if (nout > c.out_cap) {
    size_t cap = c.out_cap ? c.out_cap : 4096;
    while (cap < nout) cap *= 2;
    if (c.h_out) (void)hipHostFree(c.h_out);
    if (c.d_out) (void)hipFree(c.d_out);
    c.h_out = nullptr;
    c.d_out = nullptr;
    c.out_cap = 0;
    int rc = record_hip(hipHostMalloc((void**)&c.h_out, cap * 2, hipHostMallocDefault));
    if (rc) return rc;
    rc = record_hip(hipMalloc((void**)&c.d_out, cap * 2));
    if (rc) return rc;
    c.out_cap = cap;
  }
  return UINET_CKSUM_OK;
}

// ---- the reference chain walk, emitting the bytes each packet sums --------

struct Piece {
  const uint8_t* p;
  uint32_t n;
};

// One packet as the reference walks it: the in-order pieces whose bytes are
// summed, the logical parity of the first summed byte, and the seed.
struct PacketWalk {
  std::vector<Piece> pieces;
  uint64_t bytes = 0;
  long clen = 0;    // logical bytes consumed (may go negative, see below)
  long remain = 0;  // bytes still wanted
  long first_clen = 0;
  bool have_first = false;

  void reset(long want) {
    pieces.clear();
    bytes = 0;
    clen = 0;
    remain = want;
    have_first = false;
    first_clen = 0;
  }
  // The `skip_start:` block (in_cksum.c:219-228, :263-272).  A negative
  // mlen (len < skip, or m_len < off0) is outside the reference's contract:
  // it then indexes in_masks[] negatively for unaligned addresses; for
  // aligned ones it sums nothing, which is what happens here, while the
  // length/parity bookkeeping follows the reference.
  void take(const uint8_t* addr, long mlen) {
    if (remain < mlen) mlen = remain;
    if (mlen > 0) {
      if (!have_first) {
        have_first = true;
        first_clen = clen;
      }
      pieces.push_back({addr, (uint32_t)mlen});
      bytes += (uint64_t)mlen;
    }
    clen += mlen;
    remain -= mlen;
  }
  void take_rest(const MbufHdr* m) {  // in_cksum.c:214-229
    for (; m && remain; m = m->m_next) {
      if (m->m_len == 0) continue;
      take(m->m_data, m->m_len);
    }
  }
  void walk_skip(const MbufHdr* m, int len, int skip) {  // in_cksum.c:193-232
    reset((long)len - skip);
    while (skip && m) {
      if (m->m_len > skip) {
        take(m->m_data + skip, (long)m->m_len - skip);
        m = m->m_next;
        skip = 0;
        break;
      }
      skip -= m->m_len;
      m = m->m_next;
    }
    if (skip == 0) take_rest(m);
  }
  void walk_pseudo(const MbufHdr* m, int plen, int off0) {  // in_cksum.c:241-276
    reset(plen);
    take(m->m_data + off0, (long)m->m_len - off0);
    take_rest(m->m_next);
  }
};

// Staging image: [off u64 x n][len u32 x n][seed u32 x n][parity u8 x n] pad16
// then the packed packet bytes.
struct Layout {
  size_t off_o, len_o, seed_o, par_o, data_o;
};

Layout layout_for(size_t n) {
  Layout L;
  L.off_o = 0;
  L.len_o = L.off_o + 8 * n;
  L.seed_o = L.len_o + 4 * n;
  L.par_o = L.seed_o + 4 * n;
  L.data_o = (L.par_o + n + 15) & ~size_t(15);
  return L;
}

// Pack the walked packets, run the span kernel, copy results back.
// `walk(i, pw)` fills pw for packet i and returns its seed.
template <typename WalkFn>
int run_host_batch(int n, uint32_t flags, uint16_t* out16, unsigned* out32, WalkFn walk) {
  if (n < 0) return UINET_CKSUM_EINVAL;
  if (n == 0) return UINET_CKSUM_OK;
  Ctx& c = t_ctx;
  int rc = ctx_ready(c);
  if (rc) return rc;

  // Pass 1: walk, remember pieces (pointer chasing happens once).
  std::vector<PacketWalk> walks((size_t)n);
  std::vector<uint32_t> seeds((size_t)n);
  uint64_t total = 0;
  for (int i = 0; i < n; i++) {
    seeds[(size_t)i] = walk(i, walks[(size_t)i]);
    total += (walks[(size_t)i].bytes + 15) & ~uint64_t(15);
  }
  const Layout L = layout_for((size_t)n);
  rc = ctx_reserve(c, L.data_o + total + 16, (size_t)n);
  if (rc) return rc;

  // Pass 2: pack descriptors and bytes into pinned staging.
  uint64_t* off = reinterpret_cast<uint64_t*>(c.h_buf + L.off_o);
  uint32_t* len = reinterpret_cast<uint32_t*>(c.h_buf + L.len_o);
  uint32_t* seed = reinterpret_cast<uint32_t*>(c.h_buf + L.seed_o);
  uint8_t* par = c.h_buf + L.par_o;
  uint64_t cur = 0;
  uint32_t max_len = 0;
  for (int i = 0; i < n; i++) {
    const PacketWalk& w = walks[(size_t)i];
    if (w.bytes > 0xffffffffull) return UINET_CKSUM_EINVAL;
    off[i] = cur;
    len[i] = (uint32_t)w.bytes;
    seed[i] = seeds[(size_t)i];
    par[i] = (uint8_t)(w.first_clen & 1);
    uint8_t* dst = c.h_buf + L.data_o + cur;
    for (const Piece& p : w.pieces) {
      memcpy(dst, p.p, p.n);
      dst += p.n;
    }
    cur += (w.bytes + 15) & ~uint64_t(15);
    if (len[i] > max_len) max_len = len[i];
  }
  const size_t image = L.data_o + cur;

  rc = record_hip(hipMemcpyAsync(c.d_buf, c.h_buf, image, hipMemcpyHostToDevice, c.stream));
  if (rc) return rc;
  const uint32_t mean = (uint32_t)(total / (uint64_t)n);
  rc = launch_spans(c.d_buf + L.data_o, reinterpret_cast<const uint64_t*>(c.d_buf + L.off_o),
                    reinterpret_cast<const uint32_t*>(c.d_buf + L.len_o),
                    reinterpret_cast<const uint32_t*>(c.d_buf + L.seed_o), c.d_buf + L.par_o,
                    c.d_out, (uint32_t)n, flags, mean ? mean : 1, c.stream);
  if (rc) return rc;
  rc = record_hip(hipMemcpyAsync(c.h_out, c.d_out, (size_t)n * 2, hipMemcpyDeviceToHost,
                                 c.stream));
  if (rc) return rc;
  rc = record_hip(hipStreamSynchronize(c.stream));
  if (rc) return rc;
  for (int i = 0; i < n; i++) {
    if (out16) out16[i] = c.h_out[i];
    if (out32) out32[i] = c.h_out[i];
  }
  return UINET_CKSUM_OK;
}

[[noreturn]] void die(const char* fn, int rc) {
  fprintf(stderr, "libuinet_cksum: %s failed: %s (hip error %d: %s)\n", fn,
          uinet_cksum_strerror(rc), t_last_hip, hipGetErrorString((hipError_t)t_last_hip));
  abort();
}

}  // namespace
}  // namespace uinet

using namespace uinet;

extern "C" {

const char* uinet_cksum_version(void) { return "libuinet_cksum 0.1 (gfx950)"; }

const char* uinet_cksum_strerror(int code) {
  switch (code) {
    case UINET_CKSUM_OK: return "ok";
    case UINET_CKSUM_EINVAL: return "invalid argument";
    case UINET_CKSUM_ENODEV: return "no usable gfx950 device";
    case UINET_CKSUM_ENOMEM: return "out of memory";
    case UINET_CKSUM_EHIP: return "HIP runtime error";
    default: return "unknown error";
  }
}

int uinet_cksum_last_hip_error(void) { return t_last_hip; }

int uinet_cksum_set_tuning(const char* key, int value) {
  if (!key) return UINET_CKSUM_EINVAL;
  Tuning& t = tuning_rw();
  if (!strcmp(key, "blocks_per_cu") && value >= 0 && value <= 4096) {
    t.blocks_per_cu = value;
  } else if (!strcmp(key, "chains_variant") && (value == 0 || value == 1)) {
    t.chains_variant = value;
  } else if (!strcmp(key, "chains_pass") && (value == 2 || value == 4 || value == 8)) {
    t.chains_pass = value;
  } else {
    return UINET_CKSUM_EINVAL;
  }
  return UINET_CKSUM_OK;
}

int uinet_cksum_device_ok(void) {
  int dev = 0, count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

// ---- device-resident API ----------------------------------------------------

int uinet_cksum_spans(const void* base, const uint64_t* off, const uint32_t* len,
                      const uint32_t* seed, const uint8_t* parity, uint16_t* out, uint32_t n,
                      uint32_t flags, uint32_t len_hint, void* stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (!base || !off || !len || !out) return UINET_CKSUM_EINVAL;
  return launch_spans(base, off, len, seed, parity, out, n, flags, len_hint,
                      static_cast<hipStream_t>(stream));
}

int uinet_cksum_strided(const void* base, uint64_t stride, uint32_t len, const uint32_t* seed,
                        uint16_t* out, uint32_t n, uint32_t flags, void* stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (!base || !out) return UINET_CKSUM_EINVAL;
  return launch_strided(base, stride, len, seed, out, n, flags,
                        static_cast<hipStream_t>(stream));
}

int uinet_cksum_chains(const void* base, const uint64_t* seg_off, const uint32_t* seg_len,
                       const uint32_t* pkt_seg, const uint32_t* len, const uint32_t* skip,
                       const uint32_t* seed, uint16_t* out, uint32_t n, uint32_t flags,
                       uint32_t len_hint, void* stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (!base || !seg_off || !seg_len || !pkt_seg || !out) return UINET_CKSUM_EINVAL;
  return launch_chains(base, seg_off, seg_len, pkt_seg, len, skip, seed, out, n, flags,
                       len_hint, static_cast<hipStream_t>(stream));
}

// ---- host-mbuf batch API ------------------------------------------------------

int in_cksum_skip_batch(struct mbuf* const* m, const int* len, const int* skip,
                        unsigned short* out, int n) {
  if (n > 0 && (!m || !len || !skip || !out)) return UINET_CKSUM_EINVAL;
  return run_host_batch(n, 0, out, nullptr, [&](int i, PacketWalk& w) -> uint32_t {
    w.walk_skip(reinterpret_cast<const MbufHdr*>(m[i]), len[i], skip[i]);
    return 0u;
  });
}

int in_cksum_pseudo_header_batch(struct mbuf* const* m, const int* plen, const int* off0,
                                 const uint32_t* src, const uint32_t* dst,
                                 const uint8_t* protonum, uint16_t* out, int n) {
  if (n > 0 && (!m || !plen || !off0 || !src || !dst || !protonum || !out))
    return UINET_CKSUM_EINVAL;
  return run_host_batch(n, 0, out, nullptr, [&](int i, PacketWalk& w) -> uint32_t {
    w.walk_pseudo(reinterpret_cast<const MbufHdr*>(m[i]), plen[i], off0[i]);
    // in_cksum.c:252-253; folded on the host so it fits the u32 seed slot
    // (folding keeps both the value mod 65535 and "is zero").
    const uint64_t s = (uint64_t)src[i] + dst[i] + bswap16(protonum[i]) +
                       bswap16((uint16_t)plen[i]);
    return fold16_host(s);
  });
}

int in_cksum_hdr_batch(const struct ip* const* ip, unsigned int* out, int n) {
  if (n > 0 && (!ip || !out)) return UINET_CKSUM_EINVAL;
  return run_host_batch(n, 0, nullptr, out, [&](int i, PacketWalk& w) -> uint32_t {
    // in_cksum.c:278-285: in_cksumdata(ip, 20) weights by ADDRESS parity and
    // never re-aligns, so the header's logical start parity is its address
    // parity.
    w.reset(20);
    w.clen = (long)(reinterpret_cast<uintptr_t>(ip[i]) & 1);
    w.take(reinterpret_cast<const uint8_t*>(ip[i]), 20);
    return 0u;
  });
}

// ---- drop-in per-call ABI (sys/amd64/include/in_cksum.h:76-83) --------------

unsigned short in_cksum_skip(struct mbuf* m, int len, int skip) {
  unsigned short r = 0;
  const int rc = in_cksum_skip_batch(&m, &len, &skip, &r, 1);
  if (rc) die("in_cksum_skip", rc);
  return r;
}

uint16_t in_cksum_pseudo_header(struct mbuf* m, int plen, int off0, uint32_t src, uint32_t dst,
                                uint8_t protonum) {
  uint16_t r = 0;
  const int rc = in_cksum_pseudo_header_batch(&m, &plen, &off0, &src, &dst, &protonum, &r, 1);
  if (rc) die("in_cksum_pseudo_header", rc);
  return r;
}

unsigned int in_cksum_hdr(const struct ip* ip) {
  unsigned int r = 0;
  const int rc = in_cksum_hdr_batch(&ip, &r, 1);
  if (rc) die("in_cksum_hdr", rc);
  return r;
}

// in_pseudo / in_addword fold three or two register values -- no packet
// bytes, O(1): they stay scalar (in_cksum.c:172-191).
unsigned short in_pseudo(unsigned int a, unsigned int b, unsigned int c) {
  return (unsigned short)fold16_host((uint64_t)a + b + c);
}

unsigned short in_addword(unsigned short a, unsigned short b) {
  return (unsigned short)fold16_host((uint64_t)a + b);
}

}  // extern "C"
