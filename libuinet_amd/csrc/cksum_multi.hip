// Multi-device batches (include/uinet_cksum.h section 2e).
//
// The checksum has no cross-packet term, so a batch shards across GPUs with
// no data-path exchange, and the only traffic between devices is the 2-B
// result per packet.  For device-resident shards those results meet on the
// root device in ONE RCCL gather over xGMI: an in-process communicator over
// the shards' devices (ncclCommInitAll, cached per device list), every
// shard's kernel on its device's stream, then one grouped ncclGather (in
// place on the root when the shards are equal-sized).  RCCL is loaded with
// dlopen on first use, so the drop-in library has no hard dependency on it;
// when it cannot be loaded, when a device appears twice in the list, or when
// the root device holds no shard, the results are gathered by peer copies
// (hipMemcpyPeerAsync over xGMI, one host thread and stream per shard).  For
// host-mbuf batches every shard writes its own slice of the caller's host
// array.  This is the C-ABI form of the bench's torch.distributed layout (one
// process per GPU, RCCL gather): it serves a libuinet process whose RX/TX
// kthreads (/root/reference/lib/libuinet/uinet_if_netmap.c:1652-1665) call
// into one library on a multi-GPU host, without torch or a launcher.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <vector>

#include "cksum_internal.h"
#include "host_batch.h"
#include "host_pool.h"

namespace uinet {
namespace {

constexpr int kMaxDev = 64;

// Per (worker thread, device): a stream and a result buffer for shards that
// do not live on the root device.
struct ShardCtx {
  hipStream_t stream = nullptr;
  uint16_t* d_out = nullptr;
  size_t cap = 0;
};
thread_local ShardCtx t_shard[kMaxDev];

// Workers that run one shard each; separate from the walk pool so a shard's
// own host batch can still use that (host_pool.h: one batch at a time, the
// others walk on their own thread).
HostPool& shard_pool() {
  static HostPool* p = new HostPool;  // never destroyed, like host_pool()
  return *p;
}

// Peer access from `dev` to `root`'s memory, enabled once per pair.  Without
// it (no P2P path) hipMemcpyPeerAsync still works, staged by the runtime.
void enable_peer(int dev, int root) {
  static std::atomic<uint8_t> done[kMaxDev][kMaxDev];
  if (dev == root || done[dev][root].exchange(1)) return;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, dev, root) == hipSuccess && can) {
    const hipError_t e = hipDeviceEnablePeerAccess(root, 0);
    if (e != hipSuccess) (void)hipGetLastError();  // e.g. already enabled
  }
}

int shard_spans(const uinet_cksum_shard& sh, uint32_t flags, uint32_t len_hint, int root,
                uint16_t* dst) {
  if (sh.n == 0) return UINET_CKSUM_OK;
  int rc = record_hip(hipSetDevice(sh.device));
  if (rc) return rc;
  ShardCtx& c = t_shard[sh.device];
  if (!c.stream) {
    rc = record_hip(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    if (rc) return rc;
  }
  uint16_t* out = dst;  // a shard on the root device writes its slice directly
  if (sh.device != root) {
    enable_peer(sh.device, root);
    if (sh.n > c.cap) {
      if (c.d_out) (void)hipFree(c.d_out);
      c.d_out = nullptr;
      c.cap = 0;
      rc = record_hip(hipMalloc((void**)&c.d_out, 2 * (size_t)sh.n));
      if (rc) return rc;
      c.cap = sh.n;
    }
    out = c.d_out;
  }
  rc = launch_spans(sh.base, sh.off, sh.len, sh.seed, sh.parity, out, sh.n, flags, len_hint,
                    c.stream);
  if (rc) return rc;
  if (sh.device != root) {
    rc = record_hip(hipMemcpyPeerAsync(dst, root, out, sh.device, 2 * (size_t)sh.n, c.stream));
    if (rc) return rc;
  }
  return record_hip(hipStreamSynchronize(c.stream));
}

// --- RCCL, loaded at first use ------------------------------------------
struct Rccl {
  bool ok = false;
  decltype(&ncclCommInitAll) init = nullptr;
  decltype(&ncclGather) gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
};
const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.init = reinterpret_cast<decltype(x.init)>(dlsym(h, "ncclCommInitAll"));
    x.gather = reinterpret_cast<decltype(x.gather)>(dlsym(h, "ncclGather"));
    x.group_start = reinterpret_cast<decltype(x.group_start)>(dlsym(h, "ncclGroupStart"));
    x.group_end = reinterpret_cast<decltype(x.group_end)>(dlsym(h, "ncclGroupEnd"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(h, "ncclCommDestroy"));
    x.ok = x.init && x.gather && x.group_start && x.group_end && x.destroy;
    return x;
  }();
  return r;
}

// One communicator per distinct device list (rank k = list entry k), with a
// stream and a result buffer per rank and the root's padding buffer.  Built
// once (ncclCommInitAll costs ~100 ms) and kept for the process; calls that
// use the same list serialise on its mutex.
struct CommSet {
  std::mutex mu;
  std::vector<int> dev;
  std::vector<ncclComm_t> comm;
  std::vector<hipStream_t> stream;
  std::vector<uint16_t*> buf;  // rank k's results (capacity cap each)
  uint64_t cap = 0;
  uint16_t* pad = nullptr;     // root: ranks x cap, for unequal shards
  uint64_t pad_cap = 0;
};
// A failed build releases what it made (communicators, streams) and is not
// remembered, so a transient failure (a HIP error while another process holds
// a device, a busy xGMI link) does not disable RCCL for the process: the next
// call retries.  A device list that fails kMaxTries times, or whose failure
// can only recur (RCCL rejects the arguments), falls back to peer copies at
// once from then on.
constexpr int kMaxTries = 3;
CommSet* comm_set(const std::vector<int>& dev) {
  static std::mutex mu;
  static std::map<std::vector<int>, CommSet*>* sets = new std::map<std::vector<int>, CommSet*>;
  static std::map<std::vector<int>, int>* fails = new std::map<std::vector<int>, int>;
  std::lock_guard<std::mutex> g(mu);
  auto it = sets->find(dev);
  if (it != sets->end()) return it->second;
  int& nfail = (*fails)[dev];
  if (nfail >= kMaxTries) return nullptr;
  auto* cs = new CommSet;
  cs->dev = dev;
  cs->comm.assign(dev.size(), nullptr);
  cs->stream.assign(dev.size(), nullptr);
  cs->buf.assign(dev.size(), nullptr);
  const ncclResult_t r = rccl().init(cs->comm.data(), (int)dev.size(), dev.data());
  bool ok = r == ncclSuccess;
  for (size_t k = 0; ok && k < dev.size(); k++)
    ok = hipSetDevice(dev[k]) == hipSuccess &&
         hipStreamCreateWithFlags(&cs->stream[k], hipStreamNonBlocking) == hipSuccess;
  if (ok) {
    sets->emplace(dev, cs);
    return cs;
  }
  (void)hipGetLastError();
  for (size_t k = 0; k < dev.size(); k++) {
    if (cs->stream[k]) {
      (void)hipSetDevice(dev[k]);
      (void)hipStreamDestroy(cs->stream[k]);
    }
    if (cs->comm[k]) (void)rccl().destroy(cs->comm[k]);
  }
  delete cs;
  nfail = (r == ncclInvalidArgument || r == ncclInvalidUsage) ? kMaxTries : nfail + 1;
  return nullptr;
}

thread_local int t_last_gather = -1;  // 1 RCCL, 0 peer copies (uinet_cksum_multi_last_gather)

// The RCCL path; returns 1 when it does not apply (the caller falls back).
int spans_multi_rccl(const uinet_cksum_shard* shards, int ns, uint32_t flags, uint32_t len_hint,
                     int root_device, uint16_t* root_out, const std::vector<uint64_t>& at) {
  if (!rccl().ok || tuning().multi_gather != 0) return 1;
  std::vector<int> dev((size_t)ns);
  int root = -1;
  uint64_t nmax = 0;
  bool equal = true;
  for (int k = 0; k < ns; k++) {
    dev[(size_t)k] = shards[k].device;
    if (shards[k].device == root_device) root = k;
    nmax = std::max<uint64_t>(nmax, shards[k].n);
    equal = equal && shards[k].n == shards[0].n;
  }
  std::vector<int> sorted = dev;
  std::sort(sorted.begin(), sorted.end());
  if (root < 0 || std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end() || nmax == 0)
    return 1;
  CommSet* cs = comm_set(dev);
  if (!cs) return 1;
  std::lock_guard<std::mutex> g(cs->mu);
  t_last_gather = 1;  // this call is RCCL's from here, whatever it returns
  // On an error after the first launch, wait for the streams that may still
  // be writing root_out before returning it.
  int launched = 0;
  auto fail = [&](int rc) {
    for (int k = 0; k < launched; k++)
      if (hipSetDevice(dev[(size_t)k]) == hipSuccess)
        (void)hipStreamSynchronize(cs->stream[(size_t)k]);
    return rc;
  };
  int rc = 0;
  if (nmax > cs->cap) {
    cs->cap = 0;  // reset first: a failed (re)allocation leaves no stale capacity
    for (int k = 0; k < ns; k++) {
      if ((rc = record_hip(hipSetDevice(dev[(size_t)k])))) return rc;
      if (cs->buf[(size_t)k]) (void)hipFree(cs->buf[(size_t)k]);
      cs->buf[(size_t)k] = nullptr;
      if ((rc = record_hip(hipMalloc((void**)&cs->buf[(size_t)k], 2 * nmax)))) return rc;
    }
    cs->cap = nmax;
  }
  const uint64_t need = equal ? 0 : (uint64_t)ns * nmax;
  if (need > cs->pad_cap) {
    if ((rc = record_hip(hipSetDevice(root_device)))) return rc;
    if (cs->pad) (void)hipFree(cs->pad);
    cs->pad = nullptr;
    cs->pad_cap = 0;
    if ((rc = record_hip(hipMalloc((void**)&cs->pad, 2 * need)))) return rc;
    cs->pad_cap = need;
  }
  // every shard's kernel on its device's stream; with equal shards the root
  // folds straight into its slice of root_out and gathers in place there
  for (int k = 0; k < ns; k++) {
    const uinet_cksum_shard& sh = shards[k];
    if ((rc = record_hip(hipSetDevice(sh.device)))) return fail(rc);
    uint16_t* o = (equal && k == root) ? root_out + at[(size_t)k] : cs->buf[(size_t)k];
    launched = k + 1;
    if (sh.n &&
        (rc = launch_spans(sh.base, sh.off, sh.len, sh.seed, sh.parity, o, sh.n, flags, len_hint,
                           cs->stream[(size_t)k])))
      return fail(rc);
  }
  uint16_t* recv = equal ? root_out : cs->pad;
  if (rccl().group_start() != ncclSuccess) return fail(UINET_CKSUM_EHIP);
  for (int k = 0; k < ns; k++) {
    const void* send = (equal && k == root) ? (const void*)(root_out + at[(size_t)k])
                                            : (const void*)cs->buf[(size_t)k];
    if (rccl().gather(send, k == root ? (void*)recv : nullptr, 2 * nmax, ncclUint8, root,
                      cs->comm[(size_t)k], cs->stream[(size_t)k]) != ncclSuccess) {
      (void)rccl().group_end();
      return fail(UINET_CKSUM_EHIP);
    }
  }
  if (rccl().group_end() != ncclSuccess) return fail(UINET_CKSUM_EHIP);
  if (!equal) {  // unequal shards: compact the padded slots on the root
    if ((rc = record_hip(hipSetDevice(root_device)))) return fail(rc);
    for (int k = 0; k < ns; k++)
      if (shards[k].n &&
          (rc = record_hip(hipMemcpyAsync(root_out + at[(size_t)k], cs->pad + (uint64_t)k * nmax,
                                          2 * (size_t)shards[k].n, hipMemcpyDeviceToDevice,
                                          cs->stream[(size_t)root]))))
        return fail(rc);
  }
  int first = 0;
  for (int k = 0; k < ns; k++) {
    rc = record_hip(hipSetDevice(dev[(size_t)k]));
    if (!rc) rc = record_hip(hipStreamSynchronize(cs->stream[(size_t)k]));
    if (rc && !first) first = rc;  // still wait for every other stream
  }
  return first;
}

int first_error(const std::vector<int>& rc) {
  for (int r : rc)
    if (r) return r;
  return UINET_CKSUM_OK;
}

}  // namespace
}  // namespace uinet

using namespace uinet;

extern "C" {

int uinet_cksum_spans_multi(const struct uinet_cksum_shard* shards, int nshards, uint32_t flags,
                            uint32_t len_hint, int root_device, uint16_t* root_out) {
  t_last_gather = -1;  // until a gather runs in this call
  if (nshards < 0 || (nshards > 0 && (!shards || !root_out))) return UINET_CKSUM_EINVAL;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return UINET_CKSUM_ENODEV;
  if (root_device < 0 || root_device >= count || root_device >= kMaxDev)
    return UINET_CKSUM_EINVAL;
  std::vector<uint64_t> at((size_t)nshards + 1, 0);
  for (int k = 0; k < nshards; k++) {
    const uinet_cksum_shard& sh = shards[k];
    if (sh.device < 0 || sh.device >= count || sh.device >= kMaxDev) return UINET_CKSUM_EINVAL;
    if (sh.n > UINET_CKSUM_MAX_PACKETS) return UINET_CKSUM_EINVAL;
    if (sh.n && (!sh.base || !sh.off || !sh.len)) return UINET_CKSUM_EINVAL;
    at[(size_t)k + 1] = at[(size_t)k] + sh.n;
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (nshards > 0) {
    const int r = spans_multi_rccl(shards, nshards, flags, len_hint, root_device, root_out, at);
    if (r != 1) {
      (void)hipSetDevice(prev);
      return r;
    }
  }
  t_last_gather = 0;
  std::vector<int> rc((size_t)nshards, 0);
  shard_pool().run(nshards, nshards, [&](int k) {
    int keep = 0;
    (void)hipGetDevice(&keep);
    rc[(size_t)k] = shard_spans(shards[k], flags, len_hint, root_device, root_out + at[(size_t)k]);
    (void)hipSetDevice(keep);
  });
  (void)hipSetDevice(prev);
  return first_error(rc);
}

int uinet_cksum_multi_last_gather(void) { return t_last_gather; }

int in_cksum_skip_batch_multi(const int* devices, int ndev, struct mbuf* const* m, const int* len,
                              const int* skip, unsigned short* out, int n) {
  if (ndev <= 0 || !devices || n < 0) return UINET_CKSUM_EINVAL;
  if (n > 0 && (!m || !len || !skip || !out)) return UINET_CKSUM_EINVAL;
  CpuScope cpu(n);
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return UINET_CKSUM_ENODEV;
  for (int j = 0; j < ndev; j++)
    if (devices[j] < 0 || devices[j] >= count || devices[j] >= kMaxDev) return UINET_CKSUM_EINVAL;
  // contiguous ranges of about equal summed bytes (len - skip, as the walk takes them)
  std::vector<uint64_t> cum((size_t)n + 1, 0);
  for (int i = 0; i < n; i++) {
    const long b = (long)len[i] - skip[i];
    cum[(size_t)i + 1] = cum[(size_t)i] + (uint64_t)(b > 0 ? b : 0);
  }
  std::vector<int> lo((size_t)ndev + 1, 0);
  for (int j = 1; j < ndev; j++) {
    const uint64_t target = cum[(size_t)n] * (uint64_t)j / (uint64_t)ndev;
    int a = lo[(size_t)j - 1], b = n;  // first i with cum[i] >= target
    while (a < b) {
      const int mid = a + (b - a) / 2;
      if (cum[(size_t)mid] < target) a = mid + 1; else b = mid;
    }
    lo[(size_t)j] = a;
  }
  lo[(size_t)ndev] = n;
  int prev = 0;
  (void)hipGetDevice(&prev);
  std::vector<int> rc((size_t)ndev, 0);
  shard_pool().run(ndev, ndev, [&](int j) {
    const int a = lo[(size_t)j], b = lo[(size_t)j + 1];
    if (b <= a) return;
    int keep = 0;
    (void)hipGetDevice(&keep);
    rc[(size_t)j] = record_hip(hipSetDevice(devices[j]));
    if (!rc[(size_t)j]) rc[(size_t)j] = in_cksum_skip_batch(m + a, len + a, skip + a, out + a, b - a);
    (void)hipSetDevice(keep);
  });
  (void)hipSetDevice(prev);
  return first_error(rc);
}

}  // extern "C"
