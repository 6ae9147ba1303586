/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Host harness linked against the *reference* object
 * (/root/reference/sys/amd64/amd64/in_cksum.c compiled unmodified with
 * libuinet's kernel flags by oracle/Makefile; its global symbols are renamed
 * ref_* with objcopy so they can never be confused with the product's).
 * The result is oracle/_ref/libref_cksum.so, used to
 *   - generate tests/golden/ vectors (tests/golden/gen_golden.py), and
 *   - time the reference's own scalar in_cksum_skip on host cores for
 *     bench.py's cpu_baseline ("kind": "reference").
 * The product never loads it.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>

struct mbuf;
struct ip;

/* Reference entry points (sys/amd64/include/in_cksum.h:76-83), renamed. */
unsigned short ref_in_cksum_skip(struct mbuf *m, int len, int skip);
uint16_t ref_in_cksum_pseudo_header(struct mbuf *m, int plen, int off0,
    uint32_t src, uint32_t dst, uint8_t protonum);
unsigned ref_in_cksum_hdr(const struct ip *ip);
unsigned short ref_in_pseudo(unsigned a, unsigned b, unsigned c);
unsigned short ref_in_addword(unsigned short a, unsigned short b);

unsigned short
refh_in_cksum_skip(struct mbuf *m, int len, int skip)
{
	return ref_in_cksum_skip(m, len, skip);
}

uint16_t
refh_in_cksum_pseudo_header(struct mbuf *m, int plen, int off0, uint32_t src,
    uint32_t dst, uint8_t proto)
{
	return ref_in_cksum_pseudo_header(m, plen, off0, src, dst, proto);
}

unsigned
refh_in_cksum_hdr(const void *ip)
{
	return ref_in_cksum_hdr((const struct ip *)ip);
}

unsigned short
refh_in_pseudo(unsigned a, unsigned b, unsigned c)
{
	return ref_in_pseudo(a, b, c);
}

unsigned short
refh_in_addword(unsigned short a, unsigned short b)
{
	return ref_in_addword(a, b);
}

/* sys/netinet6/in6_cksum.c (renamed ref_*; see oracle/Makefile). */
struct ip6_hdr;
int ref_in6_cksum(struct mbuf *m, unsigned char nxt, unsigned off, unsigned len);
int ref_in6_cksum_pseudo(struct ip6_hdr *ip6, unsigned len, unsigned char nxt,
    unsigned short csum);

/* The kernel's panic(), reached by in6_cksum only when the chain is shorter
 * than off + len (in6_cksum.c:347); the tests never build such a chain. */
void ref_panic(const char *fmt, ...) __attribute__((noreturn));
void
ref_panic(const char *fmt, ...)
{
	(void)fmt;
	abort();
}

int
refh_in6_cksum(struct mbuf *m, unsigned char nxt, unsigned off, unsigned len)
{
	return ref_in6_cksum(m, nxt, off, len);
}

int
refh_in6_cksum_pseudo(struct ip6_hdr *ip6, unsigned len, unsigned char nxt,
    unsigned short csum)
{
	return ref_in6_cksum_pseudo(ip6, len, nxt, csum);
}

void
refh_in6_batch(struct mbuf *const *m, const unsigned char *nxt,
    const unsigned *off, const unsigned *len, uint16_t *out, int n)
{
	for (int i = 0; i < n; i++)
		out[i] = (uint16_t)ref_in6_cksum(m[i], nxt[i], off[i], len[i]);
}

void
refh_skip_batch(struct mbuf *const *m, const int *len, const int *skip,
    uint16_t *out, int n)
{
	for (int i = 0; i < n; i++)
		out[i] = ref_in_cksum_skip(m[i], len[i], skip[i]);
}

void
refh_pseudo_batch(struct mbuf *const *m, const int *plen, const int *off0,
    const uint32_t *src, const uint32_t *dst, const uint8_t *proto,
    uint16_t *out, int n)
{
	for (int i = 0; i < n; i++)
		out[i] = ref_in_cksum_pseudo_header(m[i], plen[i], off0[i],
		    src[i], dst[i], proto[i]);
}

void
refh_hdr_batch(const void *const *ip, unsigned *out, int n)
{
	for (int i = 0; i < n; i++)
		out[i] = ref_in_cksum_hdr((const struct ip *)ip[i]);
}

/* ---- timing: static contiguous partition, one pinned thread per core ---- */

struct job {
	int kind; /* 0 = in_cksum_skip, 1 = in_cksum_pseudo_header */
	struct mbuf *const *m;
	const int *len, *skip;
	const uint32_t *src, *dst;
	const uint8_t *proto;
	uint16_t *out;
	int lo, hi, cpu;
	pthread_barrier_t *bar;
};

static void *
worker(void *arg)
{
	struct job *j = arg;

	if (j->cpu >= 0) {
		cpu_set_t set;
		CPU_ZERO(&set);
		CPU_SET(j->cpu, &set);
		pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
	}
	pthread_barrier_wait(j->bar);
	if (j->kind == 0) {
		for (int i = j->lo; i < j->hi; i++)
			j->out[i] = ref_in_cksum_skip(j->m[i], j->len[i],
			    j->skip[i]);
	} else {
		for (int i = j->lo; i < j->hi; i++)
			j->out[i] = ref_in_cksum_pseudo_header(j->m[i],
			    j->len[i], j->skip[i], j->src[i], j->dst[i],
			    j->proto[i]);
	}
	pthread_barrier_wait(j->bar);
	return NULL;
}

static double
now(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/*
 * Run the batch `reps` times on `nthreads` pinned threads (cpus[] may be
 * NULL: no pinning) and return the best wall time in seconds.  For kind 1
 * `len` is plen and `skip` is off0.
 */
double
refh_time_batch(int kind, struct mbuf *const *m, const int *len,
    const int *skip, const uint32_t *src, const uint32_t *dst,
    const uint8_t *proto, uint16_t *out, int n, int nthreads,
    const int *cpus, int reps)
{
	pthread_t tid[256];
	struct job job[256];
	pthread_barrier_t bar;
	double best = 1e30;

	if (nthreads < 1)
		nthreads = 1;
	if (nthreads > 256)
		nthreads = 256;
	for (int r = 0; r < reps; r++) {
		double t0, t1;

		pthread_barrier_init(&bar, NULL, (unsigned)nthreads + 1);
		for (int t = 0; t < nthreads; t++) {
			job[t] = (struct job){ kind, m, len, skip, src, dst,
				proto, out, (int)((long)n * t / nthreads),
				(int)((long)n * (t + 1) / nthreads),
				cpus ? cpus[t] : -1, &bar };
			pthread_create(&tid[t], NULL, worker, &job[t]);
		}
		pthread_barrier_wait(&bar); /* all threads pinned and ready */
		t0 = now();
		pthread_barrier_wait(&bar); /* all threads done */
		t1 = now();
		for (int t = 0; t < nthreads; t++)
			pthread_join(tid[t], NULL);
		pthread_barrier_destroy(&bar);
		if (t1 - t0 < best)
			best = t1 - t0;
	}
	return best;
}
