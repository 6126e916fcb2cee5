/*
 * mt_bursts.c -- several mTCP-like threads, each with its own context on the
 * SAME GPU, pushing 64-frame bursts through the host entry points at once
 * (TEST ONLY).  mTCP runs one thread per core and maps thread k to GPU
 * k mod n (gpucsum_module.c), so with 64 cores and 8 GPUs eight contexts --
 * and with the burst server eight resident grids -- share one device and its
 * GPU_MAX_HW_QUEUES hardware queues.  Every burst is checked against the
 * oracle (oracle/csum_ref.c) on the thread that made it.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/mtcp_gpucsum.h"
#include "../../oracle/csum_ref.h"

#define ROOM 2048
#define BURST 64

struct job {
	int id, iters, server, rings;
	uint64_t mismatches, frames;
	int rc;
	double us, cpu_us;
	gcs_server_stats sst;     /* summed over the thread's rings (means weighted below) */
};

/* Server figures of the last mt_bursts / mt_rings call, over every ring:
 * out[0] requests, [1] post->done us, [2] GPU span us, [3] poll us, [4] seen
 * poll us, [5] acquire us, [6] frames us, [7] records us, [8] release us,
 * [9] polls per block request, [10] seen skew us, [11] slowest block us,
 * [12] cold fraction, [13] polls over 2 us, [14] over 5 us, [15] torn polls,
 * [16] longest poll us, [17..24] mean lateness of blocks 0..7 us, [25] wait
 * before the GPU saw a request (over the fastest) us, [26] after the GPU us. */
#define NSST 27
static double g_sst[NSST];
int mt_last_server_stats(double *out, int n)
{
	int k;
	for (k = 0; k < n && k < NSST; k++)
		out[k] = g_sst[k];
	return 0;
}

static void sst_add(gcs_server_stats *acc, const gcs_server_stats *s)
{
	/* weights: requests for the host figures, block requests for the rest */
	double w0 = (double)acc->requests, w1 = (double)s->requests;
	double b0 = (double)acc->block_requests, b1 = (double)s->block_requests;
	double p0 = (double)acc->polls, p1 = (double)s->polls;
	if (w0 + w1 > 0) {
		acc->post_to_done_us = (acc->post_to_done_us * w0 + s->post_to_done_us * w1) / (w0 + w1);
		acc->gpu_span_us = (acc->gpu_span_us * w0 + s->gpu_span_us * w1) / (w0 + w1);
		acc->seen_skew_us = (acc->seen_skew_us * w0 + s->seen_skew_us * w1) / (w0 + w1);
		acc->block_serve_us = (acc->block_serve_us * w0 + s->block_serve_us * w1) / (w0 + w1);
		for (int b = 0; b < 8; b++)
			acc->late_us[b] = (acc->late_us[b] * w0 + s->late_us[b] * w1) / (w0 + w1);
		acc->seen_wait_us = (acc->seen_wait_us * w0 + s->seen_wait_us * w1) / (w0 + w1);
		acc->after_gpu_us = (acc->after_gpu_us * w0 + s->after_gpu_us * w1) / (w0 + w1);
	}
	if (b0 + b1 > 0) {
		acc->seen_poll_us = (acc->seen_poll_us * b0 + s->seen_poll_us * b1) / (b0 + b1);
		acc->acquire_us = (acc->acquire_us * b0 + s->acquire_us * b1) / (b0 + b1);
		acc->frames_us = (acc->frames_us * b0 + s->frames_us * b1) / (b0 + b1);
		acc->records_us = (acc->records_us * b0 + s->records_us * b1) / (b0 + b1);
		acc->release_us = (acc->release_us * b0 + s->release_us * b1) / (b0 + b1);
		acc->cold_frac = (acc->cold_frac * b0 + s->cold_frac * b1) / (b0 + b1);
	}
	if (p0 + p1 > 0)
		acc->poll_us = (acc->poll_us * p0 + s->poll_us * p1) / (p0 + p1);
	acc->slow_polls_2us += s->slow_polls_2us;
	acc->slow_polls_5us += s->slow_polls_5us;
	acc->torn_polls += s->torn_polls;
	if (s->max_poll_us > acc->max_poll_us)
		acc->max_poll_us = s->max_poll_us;
	acc->requests += s->requests;
	acc->block_requests += s->block_requests;
	acc->polls += s->polls;
}

static void sst_publish(struct job *jobs, int threads)
{
	gcs_server_stats acc;
	int t;
	memset(&acc, 0, sizeof acc);
	for (t = 0; t < threads; t++)
		sst_add(&acc, &jobs[t].sst);
	g_sst[0] = (double)acc.requests;
	g_sst[1] = acc.post_to_done_us;
	g_sst[2] = acc.gpu_span_us;
	g_sst[3] = acc.poll_us;
	g_sst[4] = acc.seen_poll_us;
	g_sst[5] = acc.acquire_us;
	g_sst[6] = acc.frames_us;
	g_sst[7] = acc.records_us;
	g_sst[8] = acc.release_us;
	g_sst[9] = acc.block_requests ? (double)acc.polls / (double)acc.block_requests : 0.0;
	g_sst[10] = acc.seen_skew_us;
	g_sst[11] = acc.block_serve_us;
	g_sst[12] = acc.cold_frac;
	g_sst[13] = (double)acc.slow_polls_2us;
	g_sst[14] = (double)acc.slow_polls_5us;
	g_sst[15] = (double)acc.torn_polls;
	g_sst[16] = acc.max_poll_us;
	for (t = 0; t < 8; t++)
		g_sst[17 + t] = acc.late_us[t];
	g_sst[25] = acc.seen_wait_us;
	g_sst[26] = acc.after_gpu_us;
}

/* Thread CPU time inside the gcs calls over wall time inside them, averaged
 * over the threads of the last mt_bursts call: below 1 when threads were
 * descheduled while they waited (more threads than the process's cores). */
static double g_cpu_frac;
static int g_check_every = 1;
double mt_last_cpu_frac(void) { return g_cpu_frac; }

static double cpu_us(void)
{
	struct timespec t;
	clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
	return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static uint32_t xorshift(uint64_t *s)
{
	*s ^= *s << 13;
	*s ^= *s >> 7;
	*s ^= *s << 17;
	return (uint32_t)*s;
}

/* An mTCP-shaped TCP frame of len bytes (IMIX length), checks zero. */
static void make_frame(uint8_t *f, uint32_t len, uint64_t *rng)
{
	uint32_t k, tot = len - 14;
	for (k = 0; k < len; k++)
		f[k] = (uint8_t)xorshift(rng);
	f[12] = 0x08; f[13] = 0x00; f[14] = 0x45; f[15] = 0;
	f[16] = (uint8_t)(tot >> 8); f[17] = (uint8_t)tot;
	f[20] = 0x40; f[21] = 0; f[22] = 64; f[23] = 6; f[24] = f[25] = 0;
	f[46] = (uint8_t)((len < 66 ? 5 : 8) << 4); f[47] = 0x10;
	f[50] = f[51] = 0;
	if (len >= 66) { f[54] = 1; f[55] = 1; f[56] = 8; f[57] = 10; }
}

/* MT_PIN=1: pin worker t to the t-th CPU this process may run on, as mTCP pins
 * each of its threads to one core (core.c:1153-1245, mtcp_core_affinitize). */
static void pin_self(int t)
{
	const char *e = getenv("MT_PIN");
	cpu_set_t allowed, one;
	int c, k = 0;

	if (!e || atoi(e) == 0 || sched_getaffinity(0, sizeof allowed, &allowed) != 0)
		return;
	for (c = 0; c < CPU_SETSIZE; c++)
		if (CPU_ISSET(c, &allowed) && k++ == t % CPU_COUNT(&allowed)) {
			CPU_ZERO(&one);
			CPU_SET(c, &one);
			(void)pthread_setaffinity_np(pthread_self(), sizeof one, &one);
			return;
		}
}

static double now_us(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void *run(void *arg)
{
	struct job *j = arg;
	pin_self(j->id);
	uint8_t *rooms = malloc((size_t)BURST * ROOM), *ref = malloc((size_t)BURST * ROOM);
	uint8_t *ptrs[BURST], st[BURST], vd[BURST];
	uint16_t len[BURST];
	uint32_t cs[BURST];
	uint64_t rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)(j->id + 1) * 0x100000001B3ull;
	gcs_ctx *ctx = NULL;
	double in_calls = 0, in_cpu = 0;
	int it, i;

	j->rc = gcs_ctx_create(&ctx, 0, 4096, 8u << 20);
	if (!j->rc && j->server)
		j->rc = gcs_ctx_set_burst_server(ctx, 1);
	if (j->rc == GCS_ERANGE)   /* the device's grid serves kHubRings contexts: launch per call */
		j->rc = 0;
	for (it = 0; it < j->iters && !j->rc; it++) {
		double t0, t1;
		/* MT_CHECK_EVERY=k (tools/mt_probe.py): new frames and the oracle check
		 * on every k-th burst only, the others refill and re-verify the same
		 * frames -- less host CPU per burst when threads outnumber cores */
		const int check = it % g_check_every == 0;
		for (i = 0; check && i < BURST; i++) {
			uint32_t u = xorshift(&rng) % 12;
			len[i] = (uint16_t)(u < 7 ? 64 : u < 11 ? 576 : 1500);
			ptrs[i] = rooms + (size_t)i * ROOM;
			make_frame(ptrs[i], len[i], &rng);
			memcpy(ref + (size_t)i * ROOM, ptrs[i], len[i]);
		}
		double c0 = cpu_us();
		t0 = now_us();
		j->rc = gcs_compute_ptrs(ctx, ptrs, len, BURST, st, cs);
		in_calls += now_us() - t0;
		in_cpu += cpu_us() - c0;
		if (j->rc)
			break;
		for (i = 0; check && i < BURST; i++) {
			uint32_t rc2 = 0;
			uint8_t *r = ref + (size_t)i * ROOM;
			int rs = ref_tx_fill(r, len[i], &rc2);
			if (rs != st[i] || rc2 != cs[i] || memcmp(r, ptrs[i], len[i]))
				j->mismatches++;
			if (xorshift(&rng) % 8 == 0) {         /* corrupt one byte */
				uint32_t p = 14 + xorshift(&rng) % (len[i] - 14);
				uint8_t x = (uint8_t)(1 + xorshift(&rng) % 255);
				ptrs[i][p] ^= x;
				r[p] ^= x;
			}
		}
		c0 = cpu_us();
		t1 = now_us();
		j->rc = gcs_verify_ptrs(ctx, ptrs, len, BURST, vd, GCS_VF_ZERO_BAD_TCP_CHECK);
		in_calls += now_us() - t1;
		in_cpu += cpu_us() - c0;
		if (j->rc)
			break;
		for (i = 0; check && i < BURST; i++) {
			uint8_t *r = ref + (size_t)i * ROOM;
			int v = ref_rx_verdict(r, len[i], GCS_VF_ZERO_BAD_TCP_CHECK);
			if (v != vd[i] || memcmp(r, ptrs[i], len[i]))
				j->mismatches++;
		}
		j->frames += 2 * BURST;
	}
	j->us = in_calls / (2.0 * (it ? it : 1));     /* inside the gcs calls only */
	j->cpu_us = in_cpu / (2.0 * (it ? it : 1));
	if (ctx && j->server && gcs_server_stats_get(ctx, &j->sst) != 0)
		memset(&j->sst, 0, sizeof j->sst);
	if (ctx)
		gcs_ctx_destroy(ctx);
	free(rooms);
	free(ref);
	return NULL;
}

/* threads x iters bursts (fill, then verify, per iteration).  Returns the
 * first non-zero status; mismatches / frames / mean us per call summed or
 * averaged over the threads. */
int mt_bursts(int threads, int iters, int server, uint64_t *mismatches, uint64_t *frames,
              double *us_per_call)
{
	pthread_t tid[64];
	struct job jobs[64];
	int t, rc = 0;

	if (threads < 1 || threads > 64)
		return GCS_EINVAL;
	g_check_every = getenv("MT_CHECK_EVERY") ? atoi(getenv("MT_CHECK_EVERY")) : 1;
	if (g_check_every < 1)
		g_check_every = 1;
	for (t = 0; t < threads; t++) {
		memset(&jobs[t], 0, sizeof(jobs[t]));
		jobs[t].id = t;
		jobs[t].iters = iters;
		jobs[t].server = server;
		pthread_create(&tid[t], NULL, run, &jobs[t]);
	}
	*mismatches = *frames = 0;
	*us_per_call = 0;
	g_cpu_frac = 0;
	for (t = 0; t < threads; t++) {
		pthread_join(tid[t], NULL);
		if (jobs[t].rc && !rc)
			rc = jobs[t].rc;
		*mismatches += jobs[t].mismatches;
		*frames += jobs[t].frames;
		*us_per_call += jobs[t].us / threads;
		g_cpu_frac += (jobs[t].us > 0 ? jobs[t].cpu_us / jobs[t].us : 1.0) / threads;
	}
	sst_publish(jobs, threads);
	return rc;
}

/* One thread drives `rings` contexts (rings of the one grid) at once, as the
 * async entry points let it: per iteration it posts a 64-frame IMIX fill on
 * every context, waits for each, then does the same with a verify.  Runs
 * `threads` such threads, so threads x rings rings are hot with only
 * `threads` CPUs busy: the GPU side's scaling with rings, without the CPU
 * oversubscription of one spinning thread per ring. */
static void *run_rings(void *arg)
{
	struct job *j = arg;
	enum { R = 8 };
	pin_self(j->id);
	uint8_t *rooms[R], *ref[R], *ptrs[R][BURST], st[R][BURST], vd[R][BURST];
	uint16_t len[R][BURST];
	uint32_t cs[R][BURST];
	uint64_t tk[R];
	uint64_t rng = 0xC2B2AE3D27D4EB4Full ^ (uint64_t)(j->id + 1) * 0x9E3779B97F4A7C15ull;
	gcs_ctx *ctx[R] = {0};
	double in_calls = 0, in_cpu = 0;
	int it, i, k, nr = j->rings < R ? j->rings : R;

	for (k = 0; k < nr; k++) {
		rooms[k] = malloc((size_t)BURST * ROOM);
		ref[k] = malloc((size_t)BURST * ROOM);
		if (!j->rc)
			j->rc = gcs_ctx_create(&ctx[k], 0, 4096, 8u << 20);
		if (!j->rc)
			j->rc = gcs_ctx_set_burst_server(ctx[k], 1);
	}
	for (it = 0; it < j->iters && !j->rc; it++) {
		const int check = it % g_check_every == 0;
		for (k = 0; check && k < nr; k++)
			for (i = 0; i < BURST; i++) {
				uint32_t u = xorshift(&rng) % 12;
				len[k][i] = (uint16_t)(u < 7 ? 64 : u < 11 ? 576 : 1500);
				ptrs[k][i] = rooms[k] + (size_t)i * ROOM;
				make_frame(ptrs[k][i], len[k][i], &rng);
				memcpy(ref[k] + (size_t)i * ROOM, ptrs[k][i], len[k][i]);
			}
		double c0 = cpu_us(), t0 = now_us();
		for (k = 0; k < nr && !j->rc; k++)
			j->rc = gcs_compute_ptrs_async(ctx[k], ptrs[k], len[k], BURST, st[k], cs[k], &tk[k]);
		for (k = 0; k < nr && !j->rc; k++)
			j->rc = gcs_wait(ctx[k], tk[k]);
		in_calls += now_us() - t0;
		in_cpu += cpu_us() - c0;
		if (j->rc)
			break;
		for (k = 0; check && k < nr; k++)
			for (i = 0; i < BURST; i++) {
				uint32_t rc2 = 0;
				uint8_t *r = ref[k] + (size_t)i * ROOM;
				int rs = ref_tx_fill(r, len[k][i], &rc2);
				if (rs != st[k][i] || rc2 != cs[k][i] || memcmp(r, ptrs[k][i], len[k][i]))
					j->mismatches++;
			}
		c0 = cpu_us();
		t0 = now_us();
		for (k = 0; k < nr && !j->rc; k++)
			j->rc = gcs_verify_ptrs_async(ctx[k], ptrs[k], len[k], BURST, vd[k], 0, &tk[k]);
		for (k = 0; k < nr && !j->rc; k++)
			j->rc = gcs_wait(ctx[k], tk[k]);
		in_calls += now_us() - t0;
		in_cpu += cpu_us() - c0;
		if (j->rc)
			break;
		for (k = 0; check && k < nr; k++)
			for (i = 0; i < BURST; i++)
				if (ref_rx_verdict(ref[k] + (size_t)i * ROOM, len[k][i], 0) != vd[k][i])
					j->mismatches++;
		j->frames += 2 * BURST * nr;
	}
	/* per round (all rings' posts, then their waits) */
	j->us = in_calls / (2.0 * (it ? it : 1));
	j->cpu_us = in_cpu / (2.0 * (it ? it : 1));
	memset(&j->sst, 0, sizeof j->sst);
	for (k = 0; k < nr; k++) {
		gcs_server_stats s1;
		if (ctx[k] && gcs_server_stats_get(ctx[k], &s1) == 0)
			sst_add(&j->sst, &s1);
		if (ctx[k])
			gcs_ctx_destroy(ctx[k]);
		free(rooms[k]);
		free(ref[k]);
	}
	return NULL;
}

/* threads x rings_per_thread rings; *us_per_round = mean time of one round
 * (posts on all of a thread's rings + their waits). */
int mt_rings(int threads, int rings_per_thread, int iters, uint64_t *mismatches,
             uint64_t *frames, double *us_per_round)
{
	pthread_t tid[64];
	struct job jobs[64];
	int t, rc = 0;

	if (threads < 1 || threads > 64 || rings_per_thread < 1 || rings_per_thread > 8)
		return GCS_EINVAL;
	g_check_every = getenv("MT_CHECK_EVERY") ? atoi(getenv("MT_CHECK_EVERY")) : 1;
	if (g_check_every < 1)
		g_check_every = 1;
	for (t = 0; t < threads; t++) {
		memset(&jobs[t], 0, sizeof(jobs[t]));
		jobs[t].id = t;
		jobs[t].iters = iters;
		jobs[t].server = 1;
		jobs[t].rings = rings_per_thread;
		pthread_create(&tid[t], NULL, run_rings, &jobs[t]);
	}
	*mismatches = *frames = 0;
	*us_per_round = 0;
	g_cpu_frac = 0;
	for (t = 0; t < threads; t++) {
		pthread_join(tid[t], NULL);
		if (jobs[t].rc && !rc)
			rc = jobs[t].rc;
		*mismatches += jobs[t].mismatches;
		*frames += jobs[t].frames;
		*us_per_round += jobs[t].us / threads;
		g_cpu_frac += (jobs[t].us > 0 ? jobs[t].cpu_us / jobs[t].us : 1.0) / threads;
	}
	sst_publish(jobs, threads);
	return rc;
}
