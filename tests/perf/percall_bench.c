/*
 * Per-call latency of the drop-in ABI in C (no ctypes): the engine's
 * in_cksum_skip / in_cksum_hdr (libuinet_cksum.so) against the reference
 * object's own (oracle/_ref/libref_cksum.so, refh_* entry points), one
 * thread, same host mbufs, best of 6 passes over 65,536 packets (the two
 * sides alternate which runs first).
 * Usage: percall_bench [len] [npkt]   (prints one JSON object)
 * npkt (default 65,536) packets are cycled through 65,536 calls per pass: a
 * small npkt keeps them in cache (the fold's own speed), the default streams
 * 100 MB (the memory's).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "uinet_cksum.h"

struct mbuf {
	struct mbuf *m_next;
	void *m_nextpkt;
	char *m_data;
	int m_len;
	int m_flags;
	short m_type;
	char m_pad[6];
	char m_rest[216];
};

unsigned short refh_in_cksum_skip(struct mbuf *m, int len, int skip);
unsigned refh_in_cksum_hdr(const struct ip *ip);

static double
now(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + t.tv_nsec * 1e-9;
}

#define NPKT 65536 /* calls per pass */

int
main(int argc, char **argv)
{
	int len = argc > 1 ? atoi(argv[1]) : 1500, i, j, rep;
	int npkt = argc > 2 ? atoi(argv[2]) : NPKT;
	size_t stride = (size_t)len + 14;
	unsigned char *arena = aligned_alloc(4096, stride * NPKT + 4096);
	struct mbuf *mb = calloc(NPKT, sizeof(*mb));
	double best_e = 1e30, best_r = 1e30, best_he = 1e30, best_hr = 1e30;
	unsigned acc_e = 0, acc_r = 0;

	for (i = 0; i < (int)(stride * NPKT); i++)
		arena[i] = (unsigned char)(i * 2654435761u >> 13);
	for (i = 0; i < NPKT; i++) {
		mb[i].m_data = (char *)arena + (size_t)i * stride + 14; /* RX: +14, 2 mod 4 */
		mb[i].m_len = len;
	}
	/* the engine and the reference alternate which runs first in a pass, so
	 * each is timed both on cold data and on data the other just pulled into
	 * the caches; best of 6 */
	for (rep = 0; rep < 6; rep++) {
		int eng_first = !(rep & 1), k;
		for (k = 0; k < 2; k++) {
			double t0 = now();
			if ((k == 0) == eng_first)
				for (i = 0, j = 0; i < NPKT; i++, j = j + 1 == npkt ? 0 : j + 1)
					acc_e += in_cksum_skip(&mb[j], len, 0);
			else
				for (i = 0, j = 0; i < NPKT; i++, j = j + 1 == npkt ? 0 : j + 1)
					acc_r += refh_in_cksum_skip(&mb[j], len, 0);
			double dt = now() - t0;
			if ((k == 0) == eng_first) { if (dt < best_e) best_e = dt; }
			else if (dt < best_r) best_r = dt;
		}
		for (k = 0; k < 2; k++) {
			double t0 = now();
			if ((k == 0) == eng_first)
				for (i = 0, j = 0; i < NPKT; i++, j = j + 1 == npkt ? 0 : j + 1)
					acc_e += in_cksum_hdr((const struct ip *)mb[j].m_data);
			else
				for (i = 0, j = 0; i < NPKT; i++, j = j + 1 == npkt ? 0 : j + 1)
					acc_r += refh_in_cksum_hdr((const struct ip *)mb[j].m_data);
			double dt = now() - t0;
			if ((k == 0) == eng_first) { if (dt < best_he) best_he = dt; }
			else if (dt < best_hr) best_hr = dt;
		}
	}
	printf("{\"len\": %d, \"npkt\": %d, \"engine_skip_ns\": %.1f, \"reference_skip_ns\": %.1f, "
	    "\"engine_skip_gibs\": %.2f, \"reference_skip_gibs\": %.2f, "
	    "\"engine_hdr_ns\": %.1f, \"reference_hdr_ns\": %.1f, \"same_sums\": %s}\n",
	    len, npkt, best_e / NPKT * 1e9, best_r / NPKT * 1e9,
	    (double)len * NPKT / best_e / (1 << 30), (double)len * NPKT / best_r / (1 << 30),
	    best_he / NPKT * 1e9, best_hr / NPKT * 1e9, acc_e == acc_r ? "true" : "false");
	return 0;
}
