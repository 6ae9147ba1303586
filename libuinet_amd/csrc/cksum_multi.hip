// Multi-device batches (include/uinet_cksum.h section 2e).
//
// The checksum has no cross-packet term, so a batch shards across GPUs with
// no data-path exchange: one host thread per shard, each with its own stream
// on the shard's device, and the only traffic between devices is the 2-B
// result per packet.  For device-resident shards those results are gathered
// on the root device by peer copies over xGMI (hipMemcpyPeerAsync, peer
// access enabled once per device pair); for host-mbuf batches every shard
// writes its own slice of the caller's host array.  This is the C-ABI form of
// the bench's torch.distributed layout (one process per GPU, RCCL gather):
// it serves a libuinet process whose RX/TX kthreads
// (/root/reference/lib/libuinet/uinet_if_netmap.c:1652-1665) call into one
// library on a multi-GPU host, without torch or a launcher.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include <atomic>
#include <vector>

#include "cksum_internal.h"
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

int in_cksum_skip_batch_multi(const int* devices, int ndev, struct mbuf* const* m, const int* len,
                              const int* skip, unsigned short* out, int n) {
  if (ndev <= 0 || !devices || n < 0) return UINET_CKSUM_EINVAL;
  if (n > 0 && (!m || !len || !skip || !out)) return UINET_CKSUM_EINVAL;
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
