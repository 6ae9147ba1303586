// MI355X (gfx950) driver hooks on the device: the RX / TX offload of a batch
// whose mbufs and frames all lie in registered host memory (SURVEY.md 8f
// items 1-2).  The host copies the batch's mbuf pointers; the GPU
//   1. parses every frame's headers (k_hook_parse: offload_parse.h, the same
//      code the host hook runs, over a view that reads the mbufs through the
//      regions' device aliases) into two checksum jobs per frame,
//   2. walks and folds the jobs (k_walk_mbufs + k_chains_pipe, cksum_walk.hip),
//   3. writes the verdicts into the mbufs (k_hook_apply): RX marks
//      m_pkthdr.csum_flags / csum_data, TX stores ip_sum / th_sum / uh_sum in
//      the packet and clears the csum_flags bits it took over.
// The parse only reads host memory.  Anything the device view cannot take
// (a pointer outside the regions, a frame whose first mbuf's data does not lie
// in one region) sets a status bit, and then k_hook_apply writes nothing and
// the host runs the batch through its own hook, with the same results.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cksum_internal.h"
#include "offload_parse.h"
#include "walk_xlate.h"

namespace uinet {
namespace {

using namespace hook;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 GlobalU32x4;

// struct m_hdr / pkthdr offsets (sys/sys/mbuf.h:90-98,116-133; host_batch.h):
// m_next at 0; m_data, m_len, m_flags at 16, 24, 28 (one 16-B load at kOffData);
// csum_flags, csum_data at 64, 68.
constexpr uint64_t kOffData = 16, kOffCsumFlags = 64, kOffCsumData = 68;
constexpr int kWin = 128;  // bytes of the first mbuf's data kept in the lane

__device__ __forceinline__ u32x4 load16(uint64_t dev) {
  return *reinterpret_cast<const GlobalU32x4*>(dev);
}

// Bytes [dev, dev + k) of host memory (device alias) into dst, through
// aligned 16-B loads (one request each).
__device__ void copy_host(uint64_t dev, uint8_t* dst, int k) {
  uint64_t a = dev & ~15ull;
  int s = (int)(dev - a), got = 0;
  while (got < k) {
    union {
      u32x4 v;
      uint8_t b[16];
    } u;
    u.v = load16(a);
    for (int i = s; i < 16 && got < k; i++) dst[got++] = u.b[i];
    a += 16;
    s = 0;
  }
}

// The parse's view of a packet in registered host memory (offload_parse.h).
// The first mbuf's header fields and the first kWin bytes of its data are
// loaded once (one round trip); other bytes and mbufs are read on demand.
struct DevView {
  uint64_t m = 0;  // the head mbuf's host address
  const WalkRegionHost* R;
  int nreg;
  uint32_t bad = 0;  // kWalkUnmapped: something the view could not translate
  uint64_t dm = 0, dd = 0;  // device addresses of the head mbuf and of its data
  uint64_t next0 = 0;
  int len0 = 0, flags0 = 0, cflags = 0, cdata = 0, win_n = 0;
  uint8_t win[kWin];

  __device__ void init(uint64_t head, const WalkRegionHost* regs, int n) {
    m = head;
    R = regs;
    nreg = n;
    if (!m) return;
    // the three 16-B loads below read bytes [0, kOffCsumFlags + 16) of the mbuf
    if (!walk_xlate(R, nreg, m, kOffCsumFlags + 16, &dm)) {
      bad = kWalkUnmapped;
      m = 0;
      return;
    }
    const u32x4 a = load16(dm), b = load16(dm + kOffData), c = load16(dm + kOffCsumFlags);
    next0 = (uint64_t)a.x | (uint64_t)a.y << 32;
    const uint64_t data = (uint64_t)b.x | (uint64_t)b.y << 32;
    len0 = (int)b.z;
    flags0 = (int)b.w;
    cflags = (int)c.x;
    cdata = (int)c.y;
    if (len0 > 0) {
      // the whole first mbuf's data must be in a region: the apply step
      // writes into it
      if (!walk_xlate(R, nreg, data, (uint64_t)len0, &dd)) {
        bad = kWalkUnmapped;
        m = 0;
        return;
      }
      win_n = len0 < kWin ? len0 : kWin;
      copy_host(dd, win, win_n);
    }
  }
  __device__ uint64_t addr() const { return m; }
  __device__ int m_flags() const { return flags0; }
  __device__ int m_len() const { return len0; }
  __device__ int csum_flags() const { return cflags; }
  __device__ int csum_data() const { return cdata; }
  // chain_read: n bytes at chain offset off, across mbufs
  __device__ int read(int off, uint8_t* dst, int n) const {
    if (off >= 0 && off + n <= win_n) {
      for (int i = 0; i < n; i++) dst[i] = win[off + i];
      return n;
    }
    return read_slow(off, dst, n);
  }
  __device__ const uint8_t* bytes(int off, uint8_t* tmp, int n, int* got) const {
    if (off >= 0 && off + n <= win_n) {
      *got = n;
      return win + off;
    }
    *got = read_slow(off, tmp, n);
    return tmp;
  }
  __device__ int read_slow(int off, uint8_t* dst, int n) const {
    int got = 0;
    uint64_t cur = m, dcur = dm, data = 0;
    int l = len0;
    bool first = true;
    uint64_t nxt = next0;
    while (cur && got < n) {
      if (!first) {
        if (!walk_xlate(R, nreg, cur, 32, &dcur)) {
          const_cast<DevView*>(this)->bad = kWalkUnmapped;
          return got;
        }
        const u32x4 a = load16(dcur), b = load16(dcur + kOffData);
        nxt = (uint64_t)a.x | (uint64_t)a.y << 32;
        data = (uint64_t)b.x | (uint64_t)b.y << 32;
        l = (int)b.z;
      }
      if (l > 0) {
        if (off >= l) {
          off -= l;
        } else {
          const int k = (l - off < n - got) ? l - off : n - got;
          uint64_t src;
          if (first) {
            src = dd + (uint64_t)off;
          } else if (!walk_xlate(R, nreg, data + (uint64_t)off, (uint64_t)k, &src)) {
            const_cast<DevView*>(this)->bad = kWalkUnmapped;
            return got;
          }
          copy_host(src, dst + got, k);
          got += k;
          off = 0;
        }
      }
      first = false;
      cur = nxt;
    }
    return got;
  }
  // chain_len
  __device__ long length() const {
    long t = len0 > 0 ? len0 : 0;
    for (uint64_t cur = next0; cur;) {
      uint64_t d;
      if (!walk_xlate(R, nreg, cur, 32, &d)) {
        const_cast<DevView*>(this)->bad = kWalkUnmapped;
        return t;
      }
      const u32x4 a = load16(d), b = load16(d + kOffData);
      const int l = (int)b.z;
      t += l > 0 ? l : 0;
      cur = (uint64_t)a.x | (uint64_t)a.y << 32;
    }
    return t;
  }
  // ip_sum stays in the packet; the seed ~ip_sum cancels it in the header
  // sum.  The header's sum without the field is positive (its first byte is
  // 0x4X), so fold(sum + ~ip_sum) == fold(sum - ip_sum): the same 16 bits as
  // the host's zero-then-sum.  take_ip_sum is called for ip_sum inside the
  // first mbuf only (tx_parse checks l3 + 12 <= m_len).
  __device__ uint32_t take_ip_sum(int off) {
    uint8_t b[2];
    if (read(off, b, 2) < 2) return 0u;
    const uint32_t w = (uint32_t)b[0] | (uint32_t)b[1] << 8;
    return ~w & 0xffffu;
  }
};

// What the apply step needs of a frame besides its plan.
struct DevFrame {
  uint64_t dm, dd;  // device addresses of the head mbuf and of its data (0: none)
  int cflags, mlen, mflags;
};

template <bool kRx>
struct PlanOf;
template <>
struct PlanOf<true> {
  typedef RxPlan type;
};
template <>
struct PlanOf<false> {
  typedef TxPlan type;
};

template <bool kRx>
__global__ __launch_bounds__(256) void k_hook_parse(
    const uint64_t* __restrict__ mv, uint32_t n, int l2len,
    const WalkRegionHost* __restrict__ regions, int nreg, uint64_t* __restrict__ jm,
    int32_t* __restrict__ jl, int32_t* __restrict__ js, uint32_t* __restrict__ jd,
    typename PlanOf<kRx>::type* __restrict__ plans, DevFrame* __restrict__ frames,
    uint32_t* __restrict__ status) {
  __shared__ WalkRegionHost R[kWalkRegionsMax];
  for (int k = (int)threadIdx.x; k < nreg; k += (int)blockDim.x) R[k] = regions[k];
  __syncthreads();
  uint32_t any_bad = 0;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    DevView v;
    v.init(mv[k], R, nreg);
    typename PlanOf<kRx>::type p;
    PJob j0, j1;
    if constexpr (kRx) {
      j0 = rx_parse(v, l2len, p, &j1);
    } else {
      j0 = tx_parse(v, l2len, p, &j1);
      // a th_sum / uh_sum offset before m_data (csum_data out of range): the
      // host hook writes where ip_output.c would; the device writes nothing
      if (p.l4_job && p.l4_store < 0) v.bad |= kWalkFallback;
    }
    any_bad |= v.bad;
    plans[k] = p;
    frames[k] = DevFrame{v.m ? v.dm : 0, v.dd, v.cflags, v.len0, v.flags0};
    jm[2 * k] = j0.m;
    jl[2 * k] = j0.len;
    js[2 * k] = j0.skip;
    jd[2 * k] = j0.seed;
    jm[2 * k + 1] = j1.m;
    jl[2 * k + 1] = j1.len;
    js[2 * k + 1] = j1.skip;
    jd[2 * k + 1] = j1.seed;
  }
  for (int d = 32; d; d >>= 1) any_bad |= (uint32_t)__shfl_xor((int)any_bad, d);
  if ((threadIdx.x & 63) == 0 && any_bad) atomicOr(&status[0], any_bad);
}

// Little-endian u16 store into host memory, byte by byte (the field may sit
// at any alignment; ip_output.c stores it with the same byte order).
__device__ __forceinline__ void put16(uint64_t dev, uint16_t c) {
  uint8_t* p = reinterpret_cast<uint8_t*>(dev);
  p[0] = (uint8_t)c;
  p[1] = (uint8_t)(c >> 8);
}

template <bool kRx>
__global__ __launch_bounds__(256) void k_hook_apply(
    const typename PlanOf<kRx>::type* __restrict__ plans, const DevFrame* __restrict__ frames,
    const uint16_t* __restrict__ res, uint32_t n, uint32_t K, const uint32_t* __restrict__ status,
    uint8_t* __restrict__ st_out) {
  // all or nothing: a batch the host has to redo must find its mbufs as they were
  if (status[0] != 0 || status[1] > K) return;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    typename PlanOf<kRx>::type p = plans[k];
    const DevFrame f = frames[k];
    if constexpr (kRx) {
      // cksum_offload.hip's RX apply: ip_input.c:460-471, tcp_input.c:697-718
      const bool hdr = f.dm && (f.mflags & kMPktHdr);
      int fl = f.cflags;
      if (p.ip_job) {
        const bool ok = res[2 * k] == 0;
        p.st |= ok ? UINET_RX_IP_OK : 0;
        fl |= kCsumIpChecked | (ok ? kCsumIpValid : 0);
      }
      if (p.l4_job) {
        const uint16_t r = res[2 * k + 1];
        p.st |= UINET_RX_L4 | (r == 0 ? UINET_RX_L4_OK : 0);
        fl |= kCsumDataValid | kCsumPseudoHdr;
        if (hdr) *reinterpret_cast<int*>(f.dm + kOffCsumData) = r ^ 0xffff;
      }
      if (hdr && (p.ip_job || p.l4_job)) *reinterpret_cast<int*>(f.dm + kOffCsumFlags) = fl;
    } else {
      // TX apply: ip_output.c:665-667,953-976; ip6_output.c:188-209
      int fl = f.cflags;
      if (p.l4_job) {
        uint16_t c = res[2 * k + 1];
        if (p.udp && c == 0) c = 0xffff;  // ip_output.c:962-963, ip6_output.c:193-194
        if (p.l4_store + 2 > f.mlen) {
          p.st |= UINET_TX_L4_LOST;  // ip_output.c:966-974: the reference gives up too
        } else {
          put16(f.dd + (uint64_t)p.l4_store, c);
          p.st |= UINET_TX_L4;
        }
        fl &= ~p.clear;
      }
      if (p.ip_job) {
        put16(f.dd + (uint64_t)p.ip_l3 + 10, res[2 * k]);
        p.st |= UINET_TX_IP;
        fl &= ~kCsumIp;
      }
      if (p.l4_job || p.ip_job) *reinterpret_cast<int*>(f.dm + kOffCsumFlags) = fl;
    }
    st_out[k] = p.st;
  }
}

}  // namespace

size_t hook_plan_bytes(bool rx) { return rx ? sizeof(RxPlan) : sizeof(TxPlan); }
size_t hook_frame_bytes() { return sizeof(DevFrame); }

int launch_hook_parse(bool rx, const uint64_t* mv, uint32_t n, int l2len,
                      const WalkRegionHost* regions, int nreg, uint64_t* jm, int32_t* jl,
                      int32_t* js, uint32_t* jd, void* plans, void* frames, uint32_t* status,
                      hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  if (nreg < 1 || nreg > kWalkRegionsMax) return UINET_CKSUM_EINVAL;
  const uint64_t b64 = ((uint64_t)n + 255) / 256;
  const int blocks = (int)(b64 < 8192 ? b64 : 8192);
  if (rx)
    UINET_LAUNCH(k_hook_parse<true>, dim3(blocks), dim3(256), 0, stream, mv, n, l2len, regions,
                 nreg, jm, jl, js, jd, static_cast<RxPlan*>(plans),
                 static_cast<DevFrame*>(frames), status);
  else
    UINET_LAUNCH(k_hook_parse<false>, dim3(blocks), dim3(256), 0, stream, mv, n, l2len, regions,
                 nreg, jm, jl, js, jd, static_cast<TxPlan*>(plans),
                 static_cast<DevFrame*>(frames), status);
  return check_launch();
}

int launch_hook_apply(bool rx, const void* plans, const void* frames, const uint16_t* res,
                      uint32_t n, uint32_t K, const uint32_t* status, uint8_t* st_out,
                      hipStream_t stream) {
  if (n == 0) return UINET_CKSUM_OK;
  const uint64_t b64 = ((uint64_t)n + 255) / 256;
  const int blocks = (int)(b64 < 8192 ? b64 : 8192);
  if (rx)
    UINET_LAUNCH(k_hook_apply<true>, dim3(blocks), dim3(256), 0, stream,
                 static_cast<const RxPlan*>(plans), static_cast<const DevFrame*>(frames), res, n,
                 K, status, st_out);
  else
    UINET_LAUNCH(k_hook_apply<false>, dim3(blocks), dim3(256), 0, stream,
                 static_cast<const TxPlan*>(plans), static_cast<const DevFrame*>(frames), res, n,
                 K, status, st_out);
  return check_launch();
}

}  // namespace uinet
