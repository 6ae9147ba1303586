// Test-only: the three per-call entry points exactly as cksum_api.hip exports
// them, for a sanitizer build of cksum_percall.cpp that links without the HIP
// runtime (tests/test_percall_host.py::test_percall_fold_sanitized).
#include "host_batch.h"
#include "uinet_cksum.h"

using namespace uinet;

extern "C" {
unsigned short in_cksum_skip(struct mbuf* m, int len, int skip) {
  return host_cksum_skip(reinterpret_cast<const MbufHdr*>(m), len, skip, 0u);
}
uint16_t in_cksum_pseudo_header(struct mbuf* m, int plen, int off0, uint32_t src, uint32_t dst,
                                uint8_t protonum) {
  return host_cksum_pseudo(reinterpret_cast<const MbufHdr*>(m), plen, off0, src, dst, protonum);
}
unsigned int in_cksum_hdr(const struct ip* ip) { return host_cksum_hdr(ip); }
}
