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
#include <emmintrin.h>
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

/* ---- timing: static contiguous partition, one thread per share ----
 *
 * Every worker stamps CLOCK_MONOTONIC itself, right after the start barrier
 * (workers only) and right after its last packet; a pass is
 * max(end) - min(start).  The main thread only creates and joins the workers:
 * its own scheduling never enters the measurement (round 5 read t0/t1 on the
 * main thread around the barriers, and with every CPU of the mask busy a late
 * t0 produced passes above the host's memory bandwidth).
 */

static double
now(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void
pin_self(int cpu)
{
	if (cpu >= 0) {
		cpu_set_t set;
		CPU_ZERO(&set);
		CPU_SET(cpu, &set);
		pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
	}
}

struct job {
	int kind; /* 0 in_cksum_skip, 1 in_cksum_pseudo_header, 2 plain read */
	struct mbuf *const *m;
	const int *len, *skip;
	const uint32_t *src, *dst;
	const uint8_t *proto;
	uint16_t *out;
	long lo, hi; /* packets, or bytes for kind 2 */
	int cpu;
	pthread_barrier_t *bar;
	const unsigned char *base; /* kind 2 */
	uint64_t sink;
	double t_start, t_end;
};

/*
 * The read-bandwidth pass (kind 2): a plain streaming sum of 16-byte SSE2
 * loads into four independent accumulators, no checksum semantics -- what one
 * thread can pull from memory, the ceiling any fold of the same bytes runs
 * under (8-15 % faster than eight scalar 64-bit accumulators here).
 */
static uint64_t
read_sum(const unsigned char *p, long n)
{
	const __m128i *w = (const __m128i *)p;
	long nv = n / 16, i = 0;
	__m128i a0 = _mm_setzero_si128(), a1 = a0, a2 = a0, a3 = a0;
	uint64_t r[2], tail = 0;

	for (; i + 4 <= nv; i += 4) {
		a0 = _mm_add_epi64(a0, _mm_loadu_si128(w + i));
		a1 = _mm_add_epi64(a1, _mm_loadu_si128(w + i + 1));
		a2 = _mm_add_epi64(a2, _mm_loadu_si128(w + i + 2));
		a3 = _mm_add_epi64(a3, _mm_loadu_si128(w + i + 3));
	}
	for (; i < nv; i++)
		a0 = _mm_add_epi64(a0, _mm_loadu_si128(w + i));
	for (long b = nv * 16; b < n; b++)
		tail += p[b];
	a0 = _mm_add_epi64(_mm_add_epi64(a0, a1), _mm_add_epi64(a2, a3));
	_mm_storeu_si128((__m128i *)r, a0);
	return r[0] + r[1] + tail;
}

static void *
worker(void *arg)
{
	struct job *j = arg;

	pin_self(j->cpu);
	pthread_barrier_wait(j->bar); /* every worker pinned and ready */
	j->t_start = now();
	if (j->kind == 0) {
		for (long i = j->lo; i < j->hi; i++)
			j->out[i] = ref_in_cksum_skip(j->m[i], j->len[i],
			    j->skip[i]);
	} else if (j->kind == 1) {
		for (long i = j->lo; i < j->hi; i++)
			j->out[i] = ref_in_cksum_pseudo_header(j->m[i],
			    j->len[i], j->skip[i], j->src[i], j->dst[i],
			    j->proto[i]);
	} else {
		j->sink = read_sum(j->base + j->lo, j->hi - j->lo);
	}
	j->t_end = now();
	return NULL;
}

#define REFH_MAX_THREADS 1024

/*
 * One pass of `proto` split into nthreads contiguous shares of `total`
 * units (packets; bytes for kind 2); returns max(end) - min(start) and, if
 * stamps is not NULL, each worker's start and end (2 * nthreads doubles,
 * seconds of CLOCK_MONOTONIC).  A share of bytes starts on an 8-B boundary.
 */
static double
run_pass(const struct job *proto, long total, int nthreads, const int *cpus,
    double *stamps, uint64_t *sink)
{
	struct job *job = calloc((size_t)nthreads, sizeof(*job));
	pthread_t *tid = calloc((size_t)nthreads, sizeof(*tid));
	pthread_barrier_t bar;
	double t0 = 1e300, t1 = -1e300;

	if (job == NULL || tid == NULL)
		abort();

	pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
	for (int t = 0; t < nthreads; t++) {
		job[t] = *proto;
		job[t].lo = total * t / nthreads;
		job[t].hi = total * (t + 1) / nthreads;
		if (proto->kind == 2) {
			job[t].lo &= ~7L;
			job[t].hi = t + 1 == nthreads ? total : job[t].hi & ~7L;
		}
		job[t].cpu = cpus ? cpus[t] : -1;
		job[t].bar = &bar;
		pthread_create(&tid[t], NULL, worker, &job[t]);
	}
	for (int t = 0; t < nthreads; t++)
		pthread_join(tid[t], NULL);
	pthread_barrier_destroy(&bar);
	for (int t = 0; t < nthreads; t++) {
		if (job[t].t_start < t0)
			t0 = job[t].t_start;
		if (job[t].t_end > t1)
			t1 = job[t].t_end;
		if (stamps) {
			stamps[2 * t] = job[t].t_start;
			stamps[2 * t + 1] = job[t].t_end;
		}
		if (sink)
			*sink += job[t].sink;
	}
	free(job);
	free(tid);
	return t1 - t0;
}

static int
clamp_threads(int nthreads)
{
	return nthreads < 1 ? 1 : nthreads > REFH_MAX_THREADS ? REFH_MAX_THREADS : nthreads;
}

/*
 * Run the batch `reps` times on `nthreads` threads (cpus[] may be NULL: no
 * pinning) and return the best pass in seconds.  For kind 1 `len` is plen
 * and `skip` is off0.  stamps (may be NULL): the last pass's per-worker
 * start / end times.
 */
double
refh_time_batch(int kind, struct mbuf *const *m, const int *len,
    const int *skip, const uint32_t *src, const uint32_t *dst,
    const uint8_t *proto, uint16_t *out, int n, int nthreads,
    const int *cpus, int reps, double *stamps)
{
	const struct job p = { .kind = kind ? 1 : 0, .m = m, .len = len,
		.skip = skip, .src = src, .dst = dst, .proto = proto, .out = out };
	double best = 1e30;

	nthreads = clamp_threads(nthreads);
	for (int r = 0; r < reps; r++) {
		double t = run_pass(&p, n, nthreads, cpus, stamps, NULL);
		if (t < best)
			best = t;
	}
	return best;
}

/*
 * The host's read bandwidth over the same bytes: `reps` passes of the plain
 * streaming sum over [base, base + bytes) on nthreads threads, timed like
 * refh_time_batch; returns the best pass in seconds (*sink: the sum, so the
 * reads cannot be optimised away).
 */
double
refh_time_read(const void *base, long bytes, int nthreads, const int *cpus,
    int reps, double *stamps, uint64_t *sink)
{
	const struct job p = { .kind = 2, .base = base };
	double best = 1e30;
	uint64_t s = 0;

	nthreads = clamp_threads(nthreads);
	for (int r = 0; r < reps; r++) {
		double t = run_pass(&p, bytes, nthreads, cpus, stamps, &s);
		if (t < best)
			best = t;
	}
	if (sink)
		*sink = s;
	return best;
}
