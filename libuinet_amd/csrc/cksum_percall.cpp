// The per-call drop-in ABI on the calling CPU thread:
//   in_cksum_skip, in_cksum_pseudo_header, in_cksum_hdr, in6_cksum.
//
// Why the host: these symbols are called once per packet, synchronously, by
// protocol code that holds one mbuf chain (ip_input.c:460-468 IP options,
// ip_icmp.c, igmp.c, ip_fastfwd.c, timers; the hot RX/TX paths go through the
// batch hooks).  A GPU round trip per call costs ~16 us against ~0.2 us of
// folding 1500 bytes here, and the reference KPI has no error channel
// (/root/reference/sys/amd64/amd64/in_cksum.c:193-285): these functions
// must always return a sum, GPU or no GPU (SURVEY.md sections 7.3 and 8b).
// The batch, device-resident and offload entry points are the GPU engine and
// keep failing with UINET_CKSUM_ENODEV where there is no gfx950 device.
//
// Arithmetic.  A piece of the chain is summed as little-endian 64-bit words
// loaded from ITS OWN start (unaligned loads, no read outside the piece), with
// end-around carry; 2^64 = 1 (mod 65535), so the 64-bit one's-complement sum
// is congruent to the 16-bit one and is zero only for all-zero bytes.  Byte k
// of a piece then weighs 256^(k&1); a piece whose first byte sits at an odd
// LOGICAL offset of the packet is byte-rotated once (x * 256 mod 65535) --
// the reference reaches the same value by weighing with ADDRESS parity and
// rotating when address and logical parity differ (:222-225).  The fold is
// end-around carry (REDUCE16, :65-71), never "% 65535", so all-zero data
// gives 0xffff and a sum of 0xffff gives 0.
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <immintrin.h>

#include <algorithm>

#include "host_batch.h"
#include "uinet_cksum.h"

namespace uinet {
namespace {

inline uint64_t add_eac(uint64_t a, uint64_t b) {
  uint64_t s;
  return __builtin_add_overflow(a, b, &s) ? s + 1 : s;  // s + 1 cannot wrap here
}

inline uint64_t load64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

// 64-bit one's-complement sum of [p, p + n), byte k weighted 256^(k&1).
uint64_t piece_sum(const uint8_t* p, size_t n) {
  uint64_t a = 0, b = 0, c = 0, d = 0;  // four independent carry chains
  while (n >= 32) {
    a = add_eac(a, load64(p));
    b = add_eac(b, load64(p + 8));
    c = add_eac(c, load64(p + 16));
    d = add_eac(d, load64(p + 24));
    p += 32;
    n -= 32;
  }
  while (n >= 8) {
    a = add_eac(a, load64(p));
    p += 8;
    n -= 8;
  }
  if (n) {  // the last 1..7 bytes, zero-padded: byte k keeps weight 256^(k&1)
    uint64_t t = 0;
    size_t k = 0;
    if (n & 4) {
      uint32_t v;
      memcpy(&v, p, 4);
      t = v;
      k = 4;
    }
    if (n & 2) {
      uint16_t v;
      memcpy(&v, p + k, 2);
      t |= (uint64_t)v << (8 * k);
      k += 2;
    }
    if (n & 1) t |= (uint64_t)p[k] << (8 * k);
    b = add_eac(b, t);
  }
  return add_eac(add_eac(a, b), add_eac(c, d));
}

// The same sum 64 bytes per step with AVX2, for hosts that have it (the
// dispatch below checks once): each 32-bit little-endian word of the piece is
// added into 64-bit lanes (its low and high halves of every 64-bit word
// separately, no carries to chase); a 32-bit word is congruent mod 65535 to
// the sum of its two 16-bit halves (2^16 = 1), so the lanes' total is the
// same one's-complement sum -- zero only for all-zero bytes.  Offsets from
// the piece start stay even, so the scalar tail keeps byte k's weight.
__attribute__((target("avx2"))) uint64_t piece_sum_avx2(const uint8_t* p, size_t n) {
  const __m256i lo32 = _mm256_set1_epi64x(0xffffffffll);
  __m256i a = _mm256_setzero_si256(), b = a, c = a, d = a;
  while (n >= 64) {
    const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p));
    const __m256i y = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + 32));
    a = _mm256_add_epi64(a, _mm256_and_si256(x, lo32));
    b = _mm256_add_epi64(b, _mm256_srli_epi64(x, 32));
    c = _mm256_add_epi64(c, _mm256_and_si256(y, lo32));
    d = _mm256_add_epi64(d, _mm256_srli_epi64(y, 32));
    p += 64;
    n -= 64;
  }
  // every lane holds at most n / 32 words of < 2^32: no 64-bit wrap below 2^36 bytes
  const __m256i s = _mm256_add_epi64(_mm256_add_epi64(a, b), _mm256_add_epi64(c, d));
  uint64_t l[4];
  _mm256_storeu_si256(reinterpret_cast<__m256i*>(l), s);
  return add_eac(add_eac(add_eac(l[0], l[1]), add_eac(l[2], l[3])), piece_sum(p, n));
}

// The same with 64-byte registers (AVX-512F), 128 bytes per step.
__attribute__((target("avx512f"))) uint64_t piece_sum_avx512(const uint8_t* p, size_t n) {
  const __m512i lo32 = _mm512_set1_epi64(0xffffffffll);
  __m512i a = _mm512_setzero_si512(), b = a, c = a, d = a;
  while (n >= 128) {
    const __m512i x = _mm512_loadu_si512(p);
    const __m512i y = _mm512_loadu_si512(p + 64);
    a = _mm512_add_epi64(a, _mm512_and_si512(x, lo32));
    b = _mm512_add_epi64(b, _mm512_srli_epi64(x, 32));
    c = _mm512_add_epi64(c, _mm512_and_si512(y, lo32));
    d = _mm512_add_epi64(d, _mm512_srli_epi64(y, 32));
    p += 128;
    n -= 128;
  }
  const __m512i s = _mm512_add_epi64(_mm512_add_epi64(a, b), _mm512_add_epi64(c, d));
  uint64_t l[8];
  _mm512_storeu_si512(l, s);
  uint64_t t = 0;
  for (int i = 0; i < 8; i++) t = add_eac(t, l[i]);
  return add_eac(t, piece_sum(p, n));
}

// Which fold this host runs, decided once: 0 scalar, 1 AVX2, 2 AVX-512F
// (lab A/B builds cap it with -DUINET_LAB_SIMD_MAX).
#ifndef UINET_LAB_SIMD_MAX
#define UINET_LAB_SIMD_MAX 2
#endif
// (a static initializer may run before libgcc's own CPU detection: run it)
const int g_simd = [] {
  __builtin_cpu_init();
  return std::min(UINET_LAB_SIMD_MAX, __builtin_cpu_supports("avx512f") ? 2
                                      : __builtin_cpu_supports("avx2") ? 1 : 0);
}();

inline uint64_t piece_sum_best(const uint8_t* p, size_t n) {
  if (n >= 256 && g_simd == 2) return piece_sum_avx512(p, n);
  if (n >= 128 && g_simd >= 1) return piece_sum_avx2(p, n);
  return piece_sum(p, n);
}

inline uint32_t fold16(uint64_t s) {
  s = (s & 0xffffffffull) + (s >> 32);
  s = (s & 0xffff) + (s >> 16);
  s = (s & 0xffff) + (s >> 16);
  s = (s & 0xffff) + (s >> 16);
  return (uint32_t)s;
}

inline uint32_t rot8(uint32_t x) { return ((x << 8) | (x >> 8)) & 0xffff; }

inline uint16_t bswap16(uint16_t x) { return (uint16_t)((x << 8) | (x >> 8)); }

// The reference chain walk (in_cksum.c:193-232, :241-276) summing as it goes.
struct Walk {
  uint64_t sum = 0;
  long clen = 0;    // logical bytes consumed
  long remain = 0;  // bytes still wanted

  // in_cksum.c:219-228 / :263-272.  A negative mlen (len < skip, m_len <
  // off0) is outside the reference's contract; it sums nothing here, and the
  // length/parity bookkeeping follows the reference (the GPU batch path and
  // the oracle do the same).
  void take(const uint8_t* addr, long mlen) {
    if (remain < mlen) mlen = remain;
    if (mlen > 0) {
      uint32_t x = fold16(piece_sum_best(addr, (size_t)mlen));
      if (clen & 1) x = rot8(x);
      sum += x;
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
};

inline uint16_t complement(uint64_t s) { return (uint16_t)(~fold16(s) & 0xffff); }

}  // namespace

// in_cksum.c:193-232 with `seed` added before the fold (0 for in_cksum_skip;
// the folded IPv6 pseudo header for in6_cksum, in6_cksum.c:150-357).
uint16_t host_cksum_skip(const MbufHdr* m, long len, long skip, uint32_t seed) {
  Walk w;
  w.sum = seed;
  w.remain = len - skip;
  while (skip && m) {  // in_cksum.c:203-212
    if (m->m_len > skip) {
      w.take(m->m_data + skip, (long)m->m_len - skip);
      m = m->m_next;
      skip = 0;
      break;
    }
    skip -= m->m_len;
    m = m->m_next;
  }
  if (skip == 0) w.take_rest(m);
  return complement(w.sum);
}

uint16_t host_cksum_pseudo(const MbufHdr* m, int plen, int off0, uint32_t src, uint32_t dst,
                           uint8_t proto) {
  Walk w;
  // in_cksum.c:252-253
  w.sum = (uint64_t)src + dst + bswap16(proto) + bswap16((uint16_t)plen);
  w.remain = plen;
  w.take(m->m_data + off0, (long)m->m_len - off0);
  w.take_rest(m->m_next);
  return complement(w.sum);
}

// in_cksum.c:278-285: in_cksumdata(ip, 20) weighs bytes by ADDRESS parity and
// never re-aligns, so a header at an odd address is the rotated sum.
uint32_t host_cksum_hdr(const void* ip) {
  const uint8_t* p = static_cast<const uint8_t*>(ip);
  uint32_t w;
  memcpy(&w, p + 16, 4);
  uint32_t x = fold16(add_eac(add_eac(load64(p), load64(p + 8)), w));
  if (reinterpret_cast<uintptr_t>(ip) & 1) x = rot8(x);
  return complement(x);
}

}  // namespace uinet
