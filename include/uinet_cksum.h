/*
 * uinet_cksum.h -- C ABI of the MI355X Internet-checksum engine.
 *
 * Two layers:
 *
 *  1. The drop-in per-call ABI of libuinet's checksum KPI, with the exact
 *     signatures of /root/reference/sys/amd64/include/in_cksum.h:44,76-83 (the
 *     object the amd64 build compiles, sys/amd64/amd64/in_cksum.c).  Linking
 *     libuinet_cksum in place of that object keeps lib/libuinet and
 *     bin/multitool unchanged.  One call folds one chain on
 *     the calling CPU thread: a synchronous GPU round trip per packet would be
 *     ~30x slower than the fold, and these functions, like the reference,
 *     have no error path -- they never touch the device and never fail.
 *
 *  2. Batch entry points for callers that hold many packets at once
 *     (the RX/TX driver batches of SURVEY.md section 8f), and the
 *     device-resident descriptor API that is the hot path proper: one HIP
 *     launch folds a whole batch of packets that already sit in HBM.
 *
 * Results are bit-identical to the reference on the same inputs.  The batch,
 * device and offload entry points (section 2) are the GPU engine and never
 * fall back to a CPU computation: without a usable gfx950 device they return
 * a negative UINET_CKSUM_E* code.
 */
#ifndef UINET_CKSUM_H
#define UINET_CKSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The library is built with -fvisibility=hidden: exactly the functions
 * declared below are exported. */
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

/* libuinet's struct mbuf (sys/sys/mbuf.h:153-171).  The checksum functions
 * read only m_next (offset 0), m_data (offset 16) and m_len (int, offset 24);
 * the chain is borrowed read-only, never modified, freed or pulled up.  Only
 * the driver offload hooks (2d) write: m_pkthdr.csum_flags / csum_data
 * (offsets 64 / 68) and, on TX, the checksum fields of the packet. */
struct mbuf;
/* struct ip (sys/netinet/ip.h:49-70): 20 bytes, ip_sum at offset 10. */
struct ip;
/* struct ip6_hdr (sys/netinet/ip6.h:74-92): 40 bytes, addresses at 8 / 24. */
struct ip6_hdr;

/* ------------------------------------------------------------------------ */
/* 1. Drop-in per-call ABI (sys/amd64/include/in_cksum.h)                    */
/* ------------------------------------------------------------------------ */

#ifndef in_cksum
/* in_cksum.h:44 -- there is no in_cksum symbol on amd64. */
#define in_cksum(m, len) in_cksum_skip(m, len, 0)
#endif

/* in_cksum.h:83, in_cksum.c:193-232.  Sums bytes [skip, len) of the chain
 * (len counts from the chain start), returns the complemented 16-bit sum. */
unsigned short in_cksum_skip(struct mbuf *m, int len, int skip);

/* in_cksum.h:78-79, in_cksum.c:241-276.  Pseudo-header seed
 * src + dst + htons(proto) + htons(plen), then plen bytes from off0 in the
 * first mbuf onward.  0 means "valid" on receive. */
uint16_t in_cksum_pseudo_header(struct mbuf *m, int plen, int off0,
    uint32_t src, uint32_t dst, uint8_t protonum);

/* in_cksum.h:77, in_cksum.c:278-285.  20-byte IPv4 header, complemented. */
unsigned int in_cksum_hdr(const struct ip *ip);

/* in_cksum.h:82, in_cksum.c:181-191.  Folded, NOT complemented. */
unsigned short in_pseudo(unsigned int a, unsigned int b, unsigned int c);

/* in_cksum.h:81, in_cksum.c:172-179.  a + b with one end-around carry. */
unsigned short in_addword(unsigned short a, unsigned short b);

/* in_cksum.h:55-61: incremental TTL-decrement update of ip_sum, on the raw
 * header bytes (ip_sum is the big-endian 16-bit field at offset 10). */
static inline void
uinet_in_cksum_update(void *ip_hdr)
{
	unsigned char *p = (unsigned char *)ip_hdr + 10;
	int s = (int)(((unsigned)p[0] << 8) | p[1]) + 256;

	s = s + (s >> 16);
	p[0] = (unsigned char)(s >> 8);
	p[1] = (unsigned char)s;
}

/* The reference's own name and type (in_cksum.h:46-61: defined when
 * <netinet/ip.h> has set IPVERSION 4), for code that includes this header
 * instead of <machine/in_cksum.h>.  Include order: a translation unit that
 * also includes the reference header must include it FIRST (its guard
 * _MACHINE_IN_CKSUM_H_ then hides this copy), or define
 * UINET_CKSUM_NO_IN_CKSUM_UPDATE before including this header; otherwise
 * the two inline definitions collide. */
#if defined(IPVERSION) && (IPVERSION == 4) && !defined(_MACHINE_IN_CKSUM_H_) && \
    !defined(UINET_CKSUM_NO_IN_CKSUM_UPDATE)
static inline void
in_cksum_update(struct ip *ip)
{
	uinet_in_cksum_update(ip);
}
#endif

/* IPv6 (sys/netinet6/in6.h:637-638, compiled
 * by the reference only with INET6).  in6_cksum.c:150-357: the transport
 * segment [off, off + len) of the chain (off counts from the chain start,
 * m_data at a contiguous IPv6 header), seeded with the IPv6 pseudo header
 * (addresses without their embedded scope zone, htonl(len), nxt); returns
 * the complemented sum.  The reference panics when the chain is shorter
 * than off + len; here the chain's bytes are summed as far as they go. */
int in6_cksum(struct mbuf *m, uint8_t nxt, uint32_t off, uint32_t len);
/* in6_cksum.c:129-140: folded pseudo-header sum plus csum, NOT complemented. */
int in6_cksum_pseudo(struct ip6_hdr *ip6, uint32_t len, uint8_t nxt,
    uint16_t csum);

/* ------------------------------------------------------------------------ */
/* 2a. Status                                                                */
/* ------------------------------------------------------------------------ */

#define UINET_CKSUM_OK       0
#define UINET_CKSUM_EINVAL (-22) /* bad argument                        */
#define UINET_CKSUM_ENODEV (-19) /* no usable gfx950 device             */
#define UINET_CKSUM_ENOMEM (-12) /* host or device allocation failed    */
#define UINET_CKSUM_EHIP   (-5)  /* HIP runtime error; see last_hip_error */

/* Result flags for the batch/device entry points. */
#define UINET_CKSUM_F_UDP           0x1u /* 0 -> 0xffff (ip_output.c:962-963) */
#define UINET_CKSUM_F_NO_COMPLEMENT 0x2u /* return the folded sum, in_pseudo-style */

/* Engine version string and HIP diagnostics. */
const char *uinet_cksum_version(void);
/* The kernel instantiation (demangled, e.g. "void uinet::(anonymous
 * namespace)::k_chains_pipe<2, 32, 2, unsigned long, unsigned int>(...)")
 * the calling thread's last launch started; "" before the first launch. */
const char *uinet_cksum_last_kernel(void);
const char *uinet_cksum_strerror(int code);
int uinet_cksum_last_hip_error(void);
/* 1 when a gfx950 device is visible to the calling thread, else 0. */
int uinet_cksum_device_ok(void);

/* Performance knobs (process-wide; they never change results):
 *   "blocks_per_cu"   grid-stride launch width, 0 = per-kernel default
 *   "chains_long"     chain segments of at least this many 16-B chunks are
 *                     streamed wave-wide; 0 = never, else >= 16 (default 128)
 *   "chains_wide"     chain API: 0 (default) one wave per packet when
 *                     len_hint (mean segment bytes) is 4096-9216, else the
 *                     tile kernel; 1 = always the tile kernel, 2 = always
 *                     one wave per packet
 *   "xcd_remap"       span kernels: give each XCD a contiguous band of
 *                     packets (1, default) or plain block order (0)
 *   "host_threads"    host threads that walk/pack a large host-mbuf batch,
 *                     1..64 (default min(16, hardware threads))
 *   "walk_device"     host-mbuf batches (2c, 2d) whose mbufs AND bytes lie in
 *                     registered memory: the GPU walks the chains, the host
 *                     only writes the jobs.  3 = walk and fold in one launch;
 *                     2 = walk into a segment list, then the chain kernel;
 *                     1 (default) = 2 for chain batches, 3 for the hooks;
 *                     0 = the host walks them
 *   "span_fast"       host-mbuf batches (2c, 2d) over registered packet bytes
 *                     whose every sum lies in the packet's first mbuf (one
 *                     mbuf per packet, the netmap RX shape): 1 (default) the
 *                     calling thread reads each head mbuf and the GPU folds the
 *                     bytes as spans, dense runs copied to HBM first, no mbuf
 *                     line crosses the link; 2 = the same with the head mbufs
 *                     read by the GPU when they are registered (less host CPU,
 *                     one 128-B link line per packet more); 0 = the walks
 *                     below
 *   "multi_gather"    uinet_cksum_spans_multi: 0 = one RCCL gather when it
 *                     applies (default), 1 = always peer copies
 * Returns UINET_CKSUM_OK, or UINET_CKSUM_EINVAL for an unknown key/value.
 * The environment variables UINET_CKSUM_BLOCKS_PER_CU,
 * UINET_CKSUM_CHAINS_LONG, UINET_CKSUM_CHAINS_WIDE, UINET_CKSUM_XCD_REMAP,
 * UINET_CKSUM_HOST_THREADS, UINET_CKSUM_WALK_DEVICE, UINET_CKSUM_SPAN_FAST and
 * UINET_CKSUM_MULTI_GATHER set the initial values. */
int uinet_cksum_set_tuning(const char *key, int value);

/* ------------------------------------------------------------------------ */
/* 2b. Device-resident descriptor API (the hot path)                         */
/*                                                                          */
/* All array pointers are device pointers (HBM).  Launches are asynchronous  */
/* on `stream` (a hipStream_t; NULL = the legacy default stream).  A         */
/* `len_hint` (mean bytes per packet, 0 = unknown) selects the lanes-per-    */
/* packet geometry; it never changes results.  A launch takes at most        */
/* UINET_CKSUM_MAX_PACKETS packets (more: UINET_CKSUM_EINVAL) and, for       */
/* chains, fewer than 2^31 segments; descriptors must point at device bytes  */
/* the kernel may read (the checksum, like the reference, trusts its input). */
/* ------------------------------------------------------------------------ */

#define UINET_CKSUM_MAX_PACKETS 0x80000000u
/* Longest span the span/strided kernels fold (their in-span byte positions
 * are 32-bit signed, like the reference's `int len`): len[i] must be below
 * this; uinet_cksum_strided returns UINET_CKSUM_EINVAL for a longer len.
 * Chain segments (uinet_cksum_chains) may hold up to 2^32 - 1 bytes. */
#define UINET_CKSUM_MAX_SPAN 0x7ffff000u

/* One contiguous span per packet:
 *   out[i] = checksum of bytes [base + off[i], base + off[i] + len[i])
 * where the span's first byte sits at logical parity parity[i] & 1
 * (parity NULL = all 0, the in_cksum_skip case) and seed[i] (NULL = 0) is
 * added before folding (the in_cksum_pseudo_header seed). */
int uinet_cksum_spans(const void *base, const uint64_t *off,
    const uint32_t *len, const uint32_t *seed, const uint8_t *parity,
    uint16_t *out, uint32_t n, uint32_t flags, uint32_t len_hint,
    void *stream);

/* Same, with packed span descriptors for an arena below 4 GiB and spans of
 * at most 65535 bytes: a 32-bit offset and a 16-bit length, 6 bytes per
 * packet instead of 12 -- the shape of a netmap ring slot, whose buf_idx and
 * len the reference's RX path reads per packet
 * (lib/libuinet/uinet_if_netmap_host.c:316-323, uinet_if_netmap.c:1477).  For 64-B packets the wide
 * descriptors are 19 % of the bytes read; these are 9 %. */
int uinet_cksum_spans32(const void *base, const uint32_t *off,
    const uint16_t *len, const uint32_t *seed, const uint8_t *parity,
    uint16_t *out, uint32_t n, uint32_t flags, uint32_t len_hint,
    void *stream);

/* Same, for the fixed-geometry batch "packet i starts at base + i * stride
 * and is len bytes long" (no descriptor arrays are read). */
int uinet_cksum_strided(const void *base, uint64_t stride, uint32_t len,
    const uint32_t *seed, uint16_t *out, uint32_t n, uint32_t flags,
    void *stream);

/* Chained packets (device-resident mbuf chains resolved to segments):
 * packet i is the chain of segments [pkt_seg[i], pkt_seg[i + 1]), segment k
 * being the device bytes [base + seg_off[k], + seg_len[k]).  out[i] is
 * in_cksum_skip(chain_i, len[i], skip[i]) exactly as in_cksum.c:193-232
 * defines it (len counts from the chain start; len NULL = whole chain, skip
 * NULL = 0), plus seed[i] (NULL = 0) before folding.  `len_hint` is the mean
 * SEGMENT length here: 4096-9216 picks one wave per packet (segments of a
 * jumbo frame or a TSO payload slice), anything else the 32-packet tile
 * kernel (knob "chains_wide"). */
int uinet_cksum_chains(const void *base, const uint64_t *seg_off,
    const uint32_t *seg_len, const uint32_t *pkt_seg, const uint32_t *len,
    const uint32_t *skip, const uint32_t *seed, uint16_t *out, uint32_t n,
    uint32_t flags, uint32_t len_hint, void *stream);

/* Same, with packed segment descriptors for an arena below 4 GiB whose
 * mbufs hold at most 65535 bytes each (MCLBYTES, MJUMPAGESIZE and 9/16-KiB
 * jumbo clusters all do): a 32-bit offset and a 16-bit length, 6 bytes per
 * segment instead of 12.  The chain kernel reads 12 B per segment of
 * descriptors against ~106 B of packet bytes on config 3; this halves that. */
int uinet_cksum_chains32(const void *base, const uint32_t *seg_off,
    const uint16_t *seg_len, const uint32_t *pkt_seg, const uint32_t *len,
    const uint32_t *skip, const uint32_t *seed, uint16_t *out, uint32_t n,
    uint32_t flags, uint32_t len_hint, void *stream);

/* Chained packets as struct mbuf chains that live in HBM (config 3 "as
 * chained mbufs with m_next scatter"): heads[i] is the device address of
 * packet i's first mbuf, and every m_next and m_data in the chains is a
 * device address too, used as is (the mbufs and their bytes were allocated
 * in device memory).  out[i] is in_cksum_skip(heads[i], len[i], skip[i])
 * exactly as in_cksum.c:193-232 defines it -- the GPU follows m_next /
 * m_data / m_len (sys/sys/mbuf.h:90-98) as far as the reference does -- plus
 * seed[i] (NULL = 0) before folding; len NULL = the whole chain, skip NULL =
 * 0.  The in_cksum_pseudo_header form is in_cksum_skip(m, off0 + plen, off0)
 * with the folded pseudo-header sum as seed (when off0 lies in the first
 * mbuf, in_cksum.c:254-256).  One launch walks and folds; nothing else is
 * allocated or written.  `status` (a device u32, may be NULL) receives the
 * OR of UINET_CKSUM_MBUF_* bits for inputs outside the reference's contract;
 * it is never cleared here.  `seg_hint` (mean bytes per mbuf, 0 = unknown)
 * picks the kernel's load policy; it never changes results.  The chains are
 * trusted as the reference trusts them: every pointer the walk reaches must
 * be readable device memory. */
#define UINET_CKSUM_MBUF_TRUNC  0x1u /* a chain of more than UINET_CKSUM_MBUF_HOPS_MAX
                                        mbufs: summed up to there */
#define UINET_CKSUM_MBUF_BADLEN 0x2u /* a negative m_len: the chain ends there */
#define UINET_CKSUM_MBUF_BADARG 0x4u /* a negative skip: the packet sums nothing */
#define UINET_CKSUM_MBUF_HOPS_MAX 0x20000u
int uinet_cksum_mbufs(const struct mbuf *const *heads, const int32_t *len,
    const int32_t *skip, const uint32_t *seed, uint16_t *out, uint32_t n,
    uint32_t flags, uint32_t seg_hint, uint32_t *status, void *stream);

/* ------------------------------------------------------------------------ */
/* 2c. Host-mbuf batch API (synchronous; for the driver RX/TX batch hooks)   */
/*                                                                          */
/* The chains are walked on the host exactly as the per-call functions walk  */
/* them, the bytes are staged through pinned memory to HBM, one launch folds */
/* the batch, and the results are copied back.  Thread-safe: every calling   */
/* thread owns its own stream and staging.                                   */
/* ------------------------------------------------------------------------ */

int in_cksum_skip_batch(struct mbuf *const *m, const int *len,
    const int *skip, unsigned short *out, int n);
int in_cksum_pseudo_header_batch(struct mbuf *const *m, const int *plen,
    const int *off0, const uint32_t *src, const uint32_t *dst,
    const uint8_t *protonum, uint16_t *out, int n);
int in_cksum_hdr_batch(const struct ip *const *ip, unsigned int *out, int n);
int in6_cksum_batch(struct mbuf *const *m, const uint8_t *nxt,
    const uint32_t *off, const uint32_t *len, uint16_t *out, int n);

/* Zero-copy host regions.  Register the host memory that holds packet data
 * (the netmap ring buffers, uinet_if_netmap_host.c:153; the UMA slabs behind
 * mbufs and clusters, uinet_vm_kern.c:48-51) once; a host-mbuf batch whose
 * bytes all lie in registered regions is then folded in place by the GPU over
 * PCIe -- the host only walks the chains, it copies no packet bytes.  When the
 * mbufs themselves lie in registered regions too, the GPU also walks the
 * chains (m_next / m_data / m_len read over PCIe; knob "walk_device"): the host
 * writes 20 bytes of job per packet and sleeps until the results are back.
 * Other batches are staged through pinned memory as before.  Regions must not
 * overlap; memory that is already pinned (hipHostMalloc) is accepted as is.
 * Unregistering waits for the batches in flight that may read the region;
 * batches on different threads run concurrently. */
int uinet_cksum_register_host(void *base, size_t len);
int uinet_cksum_unregister_host(void *base);

/* ------------------------------------------------------------------------ */
/* 2d. Driver batch offload            */
/*                                                                          */
/* Whole RX / TX batches of IPv4 and IPv6 packets, each one mbuf chain with */
/* M_PKTHDR set.  `l2len` is the byte offset of the IP header from m_data:  */
/* -1 = parse an Ethernet header (14 bytes, 18 with one 802.1Q tag; type    */
/* 0x0800 or 0x86dd), >= 0 = the IP header is there and its version nibble  */
/* tells IPv4 from IPv6 (ip_output's view: 0).  One GPU batch per call;     */
/* status[i] (may be NULL) receives UINET_RX_* / UINET_TX_* bits.  When the */
/* mbufs and frames all lie in registered memory (2c) and "walk_device" is  */
/* not 0, the whole hook runs on the GPU -- header parse, walk, fold and    */
/* the writes into the mbufs -- and the host only copies the mbuf pointers; */
/* otherwise the host pool parses and walks.  Same results either way.      */
/* ------------------------------------------------------------------------ */

#define UINET_RX_IPV4    0x01 /* IPv4 header parsed */
#define UINET_RX_IP_OK   0x02 /* header checksum verifies */
#define UINET_RX_L4      0x04 /* TCP/UDP checksum computed */
#define UINET_RX_L4_OK   0x08 /* ... and it verifies */
#define UINET_RX_NOSUM   0x10 /* UDP datagram without checksum (uh_sum 0) */
#define UINET_RX_FRAG    0x20 /* fragment: L4 left to the stack after reassembly */
#define UINET_RX_IPV6    0x40 /* IPv6 header parsed (no header checksum) */

/* RX (first-look hook / uinet_pd_deliver_to_stack, uinet_api.c:2165-2187):
 * verifies every packet's IPv4 header and TCP/UDP checksum and records the
 * result in m_pkthdr the way a checksum-offloading NIC does, so ip_input
 * (ip_input.c:460-471), tcp_input (tcp_input.c:697-718) and udp_input
 * (udp_usrreq.c:428-449) skip the software sums yet reach the same verdict:
 *   csum_flags |= CSUM_IP_CHECKED, | CSUM_IP_VALID when the header sums to 0;
 *   TCP, and UDP with uh_sum != 0: csum_flags |= CSUM_DATA_VALID |
 *   CSUM_PSEUDO_HDR, csum_data = in_cksum_pseudo_header(...) ^ 0xffff
 *   (0xffff for a good packet, as if_loop.c:96-101 sets it).
 * UDP covers uh_ulen bytes (udp_usrreq.c:404-412); fragments, truncated
 * chains and non-IP frames get no L4 marks.
 * IPv6 (UINET_RX_IPV6): TCP or UDP after the fixed header and any
 * hop-by-hop (first only), destination-options and routing headers the stack
 * walks past (ip6_input.c:906-913,986-1019, dest6.c:62-123, route6.c:59-108)
 * gets the same CSUM_DATA_VALID_IPV6 | CSUM_PSEUDO_HDR marks over the IPv6
 * pseudo header (in6_cksum.c:86-126) and the transport's 40 + ip6_plen - off0
 * bytes, read back by tcp_input.c:627-639 and udp6_usrreq.c:216-246.  No
 * marks for: fragment headers anywhere in the chain (UINET_RX_FRAG; frag6
 * reassembles first), routing headers with segments left (dropped), more
 * than 15 headers, jumbograms (ip6_plen 0), truncated chains, UDP whose
 * uh_ulen differs from the transport length (udps_badlen) or whose uh_sum is
 * 0 (UINET_RX_NOSUM; an error in IPv6), and link-local / interface-local
 * addresses carrying a zone word, which ip6_input.c:658-661 drops.
 * TX (CSUM_TCP_IPV6 / CSUM_UDP_IPV6) finds the transport past the same
 * extension headers, as an offloading NIC must. */
int uinet_cksum_rx_offload(struct mbuf *const *m, int n, int l2len,
    uint8_t *status);

#define UINET_TX_L4      0x01 /* th_sum / uh_sum computed and stored */
#define UINET_TX_IP      0x02 /* ip_sum computed and stored */
#define UINET_TX_L4_LOST 0x04 /* checksum field beyond the first mbuf: not stored */
#define UINET_TX_SKIP    0x08 /* no M_PKTHDR, not IP, nothing asked, CSUM_TSO, or an
                                 IP header the chain cuts short */
#define UINET_TX_IPV6    0x10 /* an IPv6 packet (with UINET_TX_L4 or _L4_LOST) */

/* TX (if_netmap_batch_send, uinet_if_netmap.c:1196-1262, with if_hwassist =
 * CSUM_IP|CSUM_TCP|CSUM_UDP so ip_output defers, ip_output.c:645-656): for
 * every packet whose csum_flags ask for it, does what in_delayed_cksum
 * (ip_output.c:953-976, the in_pseudo seed already in th_sum) and the
 * ip_sum store (:665-667) do, then clears those csum_flags bits.
 * IPv6 (if_hwassist also CSUM_TCP_IPV6|CSUM_UDP_IPV6 0x4000|0x2000, so
 * ip6_output.c:966-988 defers): in6_delayed_cksum (ip6_output.c:188-209),
 * in_cksum_skip(m, 40 + ip6_plen, 40) over the in6_cksum_pseudo seed that
 * tcp_output.c:1069-1071 / udp6_usrreq.c:786 stored, UDP 0 -> 0xffff,
 * stored at 40 + csum_data; jumbograms (ip6_plen 0) are skipped. */
int uinet_cksum_tx_offload(struct mbuf *const *m, int n, int l2len,
    uint8_t *status);

/* ------------------------------------------------------------------------ */
/* 2e. Multi-device batches                           */
/*                                                                          */
/* Packets are independent, so a batch shards across GPUs with no exchange  */
/* but the results.  Each shard runs on its own host thread with its own    */
/* stream on its device; shards may share a device.  Both calls are         */
/* synchronous and thread-safe.                                             */
/* ------------------------------------------------------------------------ */

/* One device-resident shard: the span batch of uinet_cksum_spans, its
 * pointers on `device`. */
struct uinet_cksum_shard {
	int device;
	uint32_t n;
	const void *base;
	const uint64_t *off;
	const uint32_t *len;
	const uint32_t *seed;    /* may be NULL */
	const uint8_t *parity;   /* may be NULL */
};

/* Folds every shard on its own device (the span kernel, as
 * uinet_cksum_spans) and gathers the 16-bit results into root_out, a device
 * pointer on root_device: shard k's results start at the sum of the n of
 * shards 0..k-1.  The gather is ONE RCCL gather over xGMI (an in-process
 * communicator over the shards' devices, built on first use per device list;
 * RCCL is loaded at run time) when every shard has its own device and one of
 * them is root_device; otherwise (or with the "multi_gather" knob at 1, or
 * without RCCL) peer copies over xGMI.  Returns when every result is in
 * root_out. */
int uinet_cksum_spans_multi(const struct uinet_cksum_shard *shards, int nshards,
    uint32_t flags, uint32_t len_hint, int root_device, uint16_t *root_out);
/* How the calling thread's last uinet_cksum_spans_multi gathered: 1 RCCL
 * (also when that call failed inside the RCCL path), 0 peer copies, -1 no
 * call yet or the last call was rejected before any gather. */
int uinet_cksum_multi_last_gather(void);

/* A host-mbuf batch (in_cksum_skip_batch semantics) over ndev devices: the
 * packets are cut into ndev contiguous ranges of about equal summed bytes
 * (len[i] - skip[i]); range j is walked, staged (or read in place from
 * registered memory) and folded on devices[j], and its results land in out[]
 * at their own indices.  For libuinet's per-interface RX/TX threads
 * (uinet_if_netmap.c:1652-1665) on a multi-GPU host. */
int in_cksum_skip_batch_multi(const int *devices, int ndev, struct mbuf *const *m,
    const int *len, const int *skip, unsigned short *out, int n);

/* ------------------------------------------------------------------------ */
/* 2f. Host CPU accounting                                                   */
/*                                                                          */
/* What the host-memory entry points (2c, 2d, in_cksum_skip_batch_multi)    */
/* cost the host: every such call adds to the CALLING thread's counters its */
/* wall time, its own CPU time (CLOCK_THREAD_CPUTIME_ID, including any wait */
/* for the GPU that spins) and the CPU time the engine's host-pool helper   */
/* threads spent on it.  The per-call ABI (section 1) is not counted.       */
/* ------------------------------------------------------------------------ */

struct uinet_cksum_host_cpu {
	uint64_t calls;          /* counted calls */
	uint64_t packets;        /* packets / frames / headers they took */
	uint64_t wall_ns;        /* wall time inside them */
	uint64_t caller_cpu_ns;  /* the calling thread's CPU time inside them */
	uint64_t helper_cpu_ns;  /* host-pool helpers' CPU time for them */
	uint64_t device_walks;   /* calls whose mbuf chains the GPU walked */
	uint64_t span_batches;   /* calls folded as single-mbuf spans: the host read
	                            each head mbuf, the GPU the bytes (no walk) */
	uint64_t span_dma_bytes; /* bytes those calls moved to HBM by DMA copies
	                            of dense packet ranges (the rest the GPU read
	                            in place over PCIe) */
};

/* Copies the calling thread's counters to *st (may be NULL) and, when reset
 * is non-zero, zeroes them.  Returns UINET_CKSUM_OK. */
int uinet_cksum_host_cpu(struct uinet_cksum_host_cpu *st, int reset);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}
#endif

#endif /* UINET_CKSUM_H */
