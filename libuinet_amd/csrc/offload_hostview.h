// The driver hooks' view of a packet in host memory (offload_parse.h's View
// over host mbufs): the host hook (cksum_offload.hip) parses through it, and
// tests/native/parse_host.cpp runs the same parse on the CPU against the
// oracle.  Internal; not part of the C ABI.
#pragma once

#include <stdint.h>
#include <string.h>

#include "host_batch.h"

namespace uinet {
namespace hook {

// Copies up to n bytes at chain offset `off`; returns the count copied.
inline int chain_read(const MbufHdr* m, int off, uint8_t* dst, int n) {
  int got = 0;
  for (; m && got < n; m = m->m_next) {
    const int l = m->m_len;
    if (l <= 0) continue;
    if (off >= l) {
      off -= l;
      continue;
    }
    const int k = (l - off < n - got) ? l - off : n - got;
    memcpy(dst + got, m->m_data + off, (size_t)k);
    got += k;
    off = 0;
  }
  return got;
}

inline long chain_len(const MbufHdr* m) {
  long t = 0;
  for (; m; m = m->m_next) t += m->m_len > 0 ? m->m_len : 0;
  return t;
}

// The parse's view of a packet on the host (offload_parse.h).
struct HostView {
  MbufHdr* m;
  uint64_t addr() const { return reinterpret_cast<uint64_t>(m); }
  int read(int off, uint8_t* dst, int n) const { return chain_read(m, off, dst, n); }
  const uint8_t* bytes(int off, uint8_t* tmp, int n, int* got) const {
    if (m && off >= 0 && m->m_len > 0 && off + n <= m->m_len) {  // in the first mbuf
      *got = n;
      return reinterpret_cast<const uint8_t*>(m->m_data) + off;
    }
    *got = chain_read(m, off, tmp, n);
    return tmp;
  }
  long length() const { return chain_len(m); }
  int m_flags() const { return m->m_flags; }
  int m_len() const { return m->m_len; }
  int csum_flags() const { return pkthdr_of(m)->csum_flags; }
  int csum_data() const { return pkthdr_of(m)->csum_data; }
  uint32_t take_ip_sum(int off) {  // ip_output.c:665-667: ip_sum = 0
    m->m_data[off] = 0;
    m->m_data[off + 1] = 0;
    return 0u;
  }
};

}  // namespace hook
}  // namespace uinet
