/*
 * asan_driver.c -- host-side sanitizer run (ASan + UBSan, or TSan) of the host
 * code (TEST ONLY; built by tests/plugin/Makefile.asan, run on the GPU box by
 * tests/test_host_asan.py).  GPU-side sanitizers are not available on this
 * pool, so the device code runs uninstrumented; everything the host does --
 * gcs_api.cpp's staging slots, gather pool and burst server, the plugin
 * decorator gpucsum_module.c -- is compiled with -fsanitize=address and
 * checked here, every result against the oracle (oracle/csum_ref.c):
 *   1  threads with contexts of their own pushing 64-frame bursts, with and
 *      without the burst server (mt_bursts.c)
 *   2  a large pageable host batch split over the staging slots and gathered by
 *      the thread pool; then the same frames through gcs_*_ptrs
 *   3  frames in a registered region (in place) through the burst server
 *   4  the plugin decorating the synthetic NIC module under mini_mtcp's RX and
 *      TX loops, against the bare module (software folds)
 *   5  argument errors come back as status codes
 * Prints one line per part and "HOST DRIVER OK" at the end; exits non-zero on
 * a mismatch (ASan aborts on its own on a memory error).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gpucsum_io_module.h"
#include "../../include/mtcp_gpucsum.h"
#include "../../oracle/csum_ref.h"

/* mt_bursts.c */
int mt_bursts(int threads, int iters, int server, uint64_t *mismatches, uint64_t *frames,
              double *us_per_call);
/* synth_module.c */
extern io_module_func synth_module_func;
int synth_reset(uint32_t burst);
int synth_set_rx(const uint8_t *buf, const uint64_t *off, const uint16_t *len, uint32_t n);
uint32_t synth_tx_sent(void);
int synth_tx_frame(uint32_t k, uint8_t *out);
/* mini_mtcp.c */
struct mini_stats {
	uint64_t rx_packets, rx_errors, accepted, released, not_tcp, non_ip;
};
int mini_start(io_module_func *iom, struct mtcp_thread_context *ctx);
void mini_stop(io_module_func *iom, struct mtcp_thread_context *ctx);
int mini_rx_loop(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                 struct mini_stats *st, uint8_t *disp, uint32_t max);
int mini_tx(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
            const uint8_t *buf, const uint64_t *off, const uint16_t *len, uint32_t n,
            uint32_t burst);

static int g_fail;

#define CHECK(cond, ...)                                                                      \
	do {                                                                                  \
		if (!(cond)) {                                                                \
			fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                  \
			fprintf(stderr, __VA_ARGS__);                                         \
			fprintf(stderr, "\n");                                                \
			g_fail = 1;                                                           \
		}                                                                             \
	} while (0)

static uint32_t xs(uint64_t *s)
{
	*s ^= *s << 13;
	*s ^= *s >> 7;
	*s ^= *s << 17;
	return (uint32_t)*s;
}

/* IMIX TCP frames packed at 64 B (pslib layout), checks zero; a few frames get
 * IP options, odd lengths or a non-TCP protocol. */
static uint8_t *imix(uint32_t n, uint64_t seed, uint64_t **off_out, uint16_t **len_out,
                     uint64_t *bytes)
{
	uint64_t *off = malloc(n * sizeof(*off)), total = 0, rng = seed;
	uint16_t *len = malloc(n * sizeof(*len));
	uint8_t *buf;
	uint32_t i, k;

	for (i = 0; i < n; i++) {
		uint32_t u = xs(&rng) % 12;
		len[i] = (uint16_t)(u < 7 ? 64 : u < 11 ? 576 : 1500);
		if (xs(&rng) % 16 == 0)
			len[i] = (uint16_t)(60 + xs(&rng) % 1441);          /* any length, odd too */
		off[i] = total;
		total += (len[i] + 63u) / 64u * 64u;
	}
	buf = malloc(total + 64);
	for (k = 0; k < total + 64; k++)
		buf[k] = (uint8_t)xs(&rng);
	for (i = 0; i < n; i++) {
		uint8_t *f = buf + off[i];
		uint32_t L = len[i], tot = L - 14, ihl = 5;
		if (xs(&rng) % 8 == 0 && L >= 14 + 4 * 10 + 20)
			ihl = 5 + xs(&rng) % 6;
		f[12] = 0x08; f[13] = 0x00; f[14] = (uint8_t)(0x40 | ihl); f[15] = 0;
		f[16] = (uint8_t)(tot >> 8); f[17] = (uint8_t)tot;
		f[20] = 0x40; f[21] = 0; f[22] = 64; f[23] = (uint8_t)(xs(&rng) % 32 ? 6 : 17);
		f[24] = f[25] = 0;
		f[14 + 4 * ihl + 12] = (uint8_t)((L < 14 + 4 * ihl + 32 ? 5 : 8) << 4);
		f[14 + 4 * ihl + 13] = 0x10;
		f[14 + 4 * ihl + 16] = f[14 + 4 * ihl + 17] = 0;
	}
	*off_out = off;
	*len_out = len;
	*bytes = total;
	return buf;
}

/* Part 2: a pageable host batch (staging slots + gather pool), then ptrs. */
static void part_host_batch(void)
{
	const uint32_t n = 20000;
	uint64_t *off, bytes, k;
	uint16_t *len;
	uint8_t *buf = imix(n, 0xA5A5, &off, &len, &bytes), *ref = malloc(bytes + 64);
	uint8_t *st = malloc(n), *vd = malloc(n), **ptrs = malloc(n * sizeof(*ptrs));
	uint32_t *cs = malloc(n * sizeof(*cs)), i, bad = 0;
	gcs_ctx *ctx = NULL;
	int rc = gcs_ctx_create(&ctx, 0, 1024, 1u << 20);          /* small slots: many chunks */

	CHECK(rc == 0, "gcs_ctx_create %d", rc);
	memcpy(ref, buf, bytes + 64);
	rc = gcs_compute(ctx, buf, off, len, n, st, cs);
	CHECK(rc == 0, "gcs_compute %d %s", rc, gcs_last_hip_error());
	for (i = 0; i < n; i++) {
		uint32_t c2 = 0;
		int s2 = ref_tx_fill(ref + off[i], len[i], &c2);
		if (s2 != st[i] || (s2 == 0 && c2 != cs[i]))
			bad++;
	}
	CHECK(memcmp(ref, buf, bytes) == 0, "filled bytes differ from the oracle");
	for (k = 0; k < 300; k++) {                                   /* corrupt some frames */
		i = (uint32_t)((k * 7919) % n);
		buf[off[i] + 14 + (k % (len[i] - 14))] ^= 0x5A;
		ref[off[i] + 14 + (k % (len[i] - 14))] ^= 0x5A;
	}
	rc = gcs_verify(ctx, buf, off, len, n, vd, GCS_VF_ZERO_BAD_TCP_CHECK);
	CHECK(rc == 0, "gcs_verify %d", rc);
	for (i = 0; i < n; i++)
		if (ref_rx_verdict(ref + off[i], len[i], GCS_VF_ZERO_BAD_TCP_CHECK) != vd[i])
			bad++;
	CHECK(memcmp(ref, buf, bytes) == 0, "verify side effects differ from the oracle");
	for (i = 0; i < n; i++)
		ptrs[i] = (i % 97 == 5) ? NULL : buf + off[i];           /* some frames absent */
	rc = gcs_verify_ptrs(ctx, ptrs, len, n, vd, 0);
	CHECK(rc == 0, "gcs_verify_ptrs %d", rc);
	for (i = 0; i < n; i++)
		if (ptrs[i] && ref_rx_verdict(ref + off[i], len[i], 0) != vd[i])
			bad++;
	CHECK(bad == 0, "%u frames differ from the oracle", bad);
	printf("part 2 host batch: %u frames, %llu bytes, mismatches %u\n", n,
	       (unsigned long long)bytes, bad);
	gcs_ctx_destroy(ctx);
	free(buf); free(ref); free(st); free(vd); free(ptrs); free(cs); free(off); free(len);
}

/* Part 3: frames in a registered region, in place, through the burst server. */
static void part_registered(void)
{
	const uint32_t n = 64, room = 2048;
	uint8_t *region = NULL, *ref = malloc((size_t)n * room), *ptrs[64], st[64], vd[64];
	uint16_t len[64];
	uint32_t cs[64], i, it, bad = 0;
	uint64_t rng = 77;
	gcs_ctx *ctx = NULL;
	int rc = posix_memalign((void **)&region, 4096, (size_t)n * room);

	CHECK(rc == 0, "posix_memalign %d", rc);
	rc = gcs_host_register(region, (uint64_t)n * room);      /* an mbuf pool would be */
	CHECK(rc == 0, "gcs_host_register %d", rc);
	rc = gcs_ctx_create(&ctx, 0, 256, 1u << 20);
	CHECK(rc == 0, "gcs_ctx_create %d", rc);
	rc = gcs_ctx_set_burst_server(ctx, 1);
	CHECK(rc == 0, "burst server %d", rc);
	for (it = 0; it < 200; it++) {
		for (i = 0; i < n; i++) {
			uint8_t *f = region + (size_t)i * room;
			uint32_t L = 64 + xs(&rng) % 1437, k, tot = L - 14;
			for (k = 0; k < L; k++)
				f[k] = (uint8_t)xs(&rng);
			f[12] = 8; f[13] = 0; f[14] = 0x45; f[16] = (uint8_t)(tot >> 8);
			f[17] = (uint8_t)tot; f[23] = 6; f[24] = f[25] = 0; f[46] = 5 << 4;
			f[50] = f[51] = 0;
			len[i] = (uint16_t)L;
			ptrs[i] = f;
			memcpy(ref + (size_t)i * room, f, L);
		}
		rc = gcs_compute_ptrs(ctx, ptrs, len, n, st, cs);
		CHECK(rc == 0, "compute_ptrs %d", rc);
		for (i = 0; i < n; i++) {
			uint32_t c2 = 0;
			uint8_t *r = ref + (size_t)i * room;
			if (ref_tx_fill(r, len[i], &c2) != st[i] || memcmp(r, ptrs[i], len[i]))
				bad++;
		}
		rc = gcs_verify_ptrs(ctx, ptrs, len, n, vd, 0);
		CHECK(rc == 0, "verify_ptrs %d", rc);
		for (i = 0; i < n; i++)
			if (ref_rx_verdict(ref + (size_t)i * room, len[i], 0) != vd[i])
				bad++;
	}
	CHECK(bad == 0, "registered bursts: %u mismatches", bad);
	printf("part 3 registered region, burst server: 200 x 64 frames, mismatches %u\n", bad);
	gcs_ctx_destroy(ctx);
	gcs_host_unregister(region);
	free(region);
	free(ref);
}

/* Part 4: the decorator over the synthetic NIC under mini_mtcp, vs the bare
 * module (software folds). */
static void part_plugin(void)
{
	const uint32_t n = 3000;
	uint64_t *off, bytes;
	uint16_t *len;
	uint8_t *buf = imix(n, 0xBEEF, &off, &len, &bytes);
	uint8_t *d_sw = malloc(n), *d_gpu = malloc(n), *rx = malloc(bytes + 64);
	uint8_t *f_sw = malloc(2048), *f_gpu = malloc(2048);
	struct mini_stats s_sw, s_gpu;
	struct mtcp_thread_context *ctx = (struct mtcp_thread_context *)(uintptr_t)0x1000;
	uint32_t i, sent_sw, sent_gpu, diff = 0;
	int k_sw, k_gpu, rc;

	/* RX: frames with valid checks, a few corrupted */
	memcpy(rx, buf, bytes + 64);
	for (i = 0; i < n; i++) {
		uint32_t c2;
		ref_tx_fill(rx + off[i], len[i], &c2);
		if (i % 13 == 3)
			rx[off[i] + 14 + (i % (len[i] - 14))] ^= 0x81;
	}
	synth_reset(64);
	synth_set_rx(rx, off, len, n);
	mini_start(&synth_module_func, ctx);
	k_sw = mini_rx_loop(&synth_module_func, ctx, 0, &s_sw, d_sw, n);
	mini_stop(&synth_module_func, ctx);

	synth_reset(64);
	synth_set_rx(rx, off, len, n);
	rc = gpucsum_set_inner(&synth_module_func);
	CHECK(rc == 0, "gpucsum_set_inner %d", rc);
	mini_start(&gpucsum_module_func, ctx);
	k_gpu = mini_rx_loop(&gpucsum_module_func, ctx, 0, &s_gpu, d_gpu, n);
	CHECK(k_sw == (int)n && k_gpu == (int)n, "RX frame counts %d %d", k_sw, k_gpu);
	/* an error is MINI_ERROR in software (the stack's own check) and MINI_NULL
	 * through the decorator (get_rptr NULL, counted by core.c:794-799) */
	for (i = 0; i < n; i++) {
		const int e_sw = d_sw[i] == 1 || d_sw[i] == 5, e_gpu = d_gpu[i] == 1 || d_gpu[i] == 5;
		if (e_sw != e_gpu || (!e_sw && d_sw[i] != d_gpu[i]))
			diff++;
	}
	CHECK(diff == 0 && s_sw.rx_errors == s_gpu.rx_errors && s_sw.accepted == s_gpu.accepted,
	      "RX dispositions differ on %u frames (errors %llu vs %llu)", diff,
	      (unsigned long long)s_sw.rx_errors, (unsigned long long)s_gpu.rx_errors);

	/* TX: the same frames, check fields zero, through the decorator vs bare */
	synth_reset(64);
	mini_tx(&gpucsum_module_func, ctx, 0, buf, off, len, n, 64);
	sent_gpu = synth_tx_sent();
	mini_stop(&gpucsum_module_func, ctx);
	for (i = 0; i < sent_gpu && i < n; i++) {
		uint32_t c2;
		memcpy(f_sw, buf + off[i], len[i]);
		if (ref_tx_fill(f_sw, len[i], &c2) < 0)
			continue;
		synth_tx_frame(i, f_gpu);
		if (memcmp(f_sw, f_gpu, len[i]))
			diff++;
	}
	synth_reset(64);
	mini_start(&synth_module_func, ctx);
	mini_tx(&synth_module_func, ctx, 0, buf, off, len, n, 64);
	sent_sw = synth_tx_sent();
	mini_stop(&synth_module_func, ctx);
	CHECK(sent_sw == sent_gpu, "TX sent %u vs %u", sent_sw, sent_gpu);
	CHECK(diff == 0, "%u TX frames differ from the oracle fill", diff);
	printf("part 4 plugin over the synthetic NIC: RX %d frames (%llu errors), TX %u frames, "
	       "differences %u\n", k_gpu, (unsigned long long)s_gpu.rx_errors, sent_gpu, diff);
	free(buf); free(d_sw); free(d_gpu); free(rx); free(f_sw); free(f_gpu); free(off); free(len);
}

/* Part 5: argument errors are status codes. */
static void part_errors(void)
{
	gcs_ctx *ctx = NULL;
	uint8_t frame[64] = {0}, vd[4];
	uint8_t *ptrs[1] = {frame};
	uint16_t len[1] = {64};
	uint64_t off[1] = {0};
	int rc = gcs_ctx_create(&ctx, 0, 64, 1u << 16);

	CHECK(rc == 0, "gcs_ctx_create %d", rc);
	CHECK(gcs_verify(NULL, frame, off, len, 1, vd, 0) != 0, "NULL ctx accepted");
	CHECK(gcs_verify_ptrs(ctx, NULL, len, 1, vd, 0) != 0, "NULL ptrs accepted");
	CHECK(gcs_verify_ptrs(ctx, ptrs, len, 1, NULL, 0) != 0, "NULL verdicts accepted");
	CHECK(gcs_verify(ctx, frame, off, len, 0, vd, 0) == 0, "an empty batch refused");
	len[0] = 60000;                                      /* larger than the staging */
	CHECK(gcs_verify_ptrs(ctx, ptrs, len, 1, vd, 0) != 0, "oversized frame accepted");
	CHECK(gcs_ctx_create(&ctx, 999, 64, 1u << 16) != 0, "device 999 accepted");
	printf("part 5 argument errors: ok\n");
}

/* Part 6: async TX fills (gcs_compute_ptrs_async / gcs_wait): groups of 1..100
 * frames, up to 20 outstanding (past the 8 request slots: slot reuse), waits
 * on older and newer tickets, a synchronous verify on the same context in
 * between; pageable frames (staged) and frames in a registered region. */
static void part_async(int registered)
{
	const uint32_t n = 3000;
	uint64_t *off, bytes, rng = 0xC0FFEE + registered;
	uint16_t *len;
	uint8_t *src = imix(n, 0x6A6A + registered, &off, &len, &bytes), *ref = malloc(bytes + 64);
	uint8_t *buf, *mem = NULL, *st = malloc(n), *vd = malloc(n), **ptrs = malloc(n * sizeof(*ptrs));
	uint32_t *cs = malloc(n * sizeof(*cs)), i, bad = 0, posts = 0;
	uint64_t tk[32] = {0};
	gcs_ctx *ctx = NULL;
	int rc = gcs_ctx_create(&ctx, 0, 4096, 8u << 20), nt = 0;

	CHECK(rc == 0, "gcs_ctx_create %d", rc);
	CHECK(gcs_ctx_set_burst_server(ctx, 1) == 0, "server on");
	if (registered) {
		mem = aligned_alloc(4096, (bytes + 64 + 4095) / 4096 * 4096);
		memcpy(mem, src, bytes + 64);
		rc = gcs_host_register(mem, (bytes + 64 + 4095) / 4096 * 4096);
		CHECK(rc == 0, "gcs_host_register %d", rc);
		buf = mem;
	} else {
		buf = src;
	}
	memcpy(ref, buf, bytes + 64);
	for (i = 0; i < n; i++) {
		ptrs[i] = buf + off[i];
		st[i] = 0xEE;
		cs[i] = 0xEEEEEEEEu;
	}
	for (i = 0; i < n;) {
		uint32_t m = 1 + xs(&rng) % 100;
		uint64_t t = 0;
		if (m > n - i)
			m = n - i;
		rc = gcs_compute_ptrs_async(ctx, ptrs + i, len + i, m, st + i, cs + i, &t);
		CHECK(rc == 0, "async post %d %s", rc, gcs_last_hip_error());
		tk[nt++ % 32] = t;
		posts++;
		i += m;
		if (posts % 7 == 0) {                        /* an older ticket */
			rc = gcs_wait(ctx, tk[(nt + 28) % 32]);
			CHECK(rc == 0, "gcs_wait (older) %d", rc);
		}
		if (posts % 11 == 0) {                       /* synchronous work in between */
			uint16_t l1 = len[0];
			uint8_t *p1 = ref;
			rc = gcs_verify_ptrs(ctx, &p1, &l1, 1, vd, 0);
			CHECK(rc == 0, "sync verify between async posts %d", rc);
		}
	}
	rc = gcs_wait(ctx, tk[(nt - 1) % 32]);
	CHECK(rc == 0, "gcs_wait (last) %d", rc);
	for (i = 0; i < n; i++) {
		uint32_t c2 = 0;
		int s2 = ref_tx_fill(ref + off[i], len[i], &c2);
		if (s2 != st[i] || (s2 == 0 && c2 != cs[i]))
			bad++;
	}
	CHECK(memcmp(ref, buf, bytes) == 0, "async filled bytes differ from the oracle");
	CHECK(bad == 0, "%u async statuses differ from the oracle", bad);
	CHECK(gcs_wait(ctx, 0) == 0, "gcs_wait(0)");
	printf("part 6 async fills (%s): %u frames in %u posts, mismatches %u\n",
	       registered ? "registered" : "pageable", n, posts, bad);
	gcs_ctx_destroy(ctx);
	if (registered) {
		CHECK(gcs_host_unregister(mem) == 0, "unregister");
		free(mem);
	}
	free(src); free(ref); free(st); free(vd); free(ptrs); free(cs); free(off); free(len);
}

/* Part 7: the decorator's GPU-failure paths (gpucsum_io_module.h "GPU
 * failures"), forced with the test-only GCS_FAULT_INJECT switch: an RX burst
 * whose verify fails comes back NULL; in-place TX frames whose fill, or whose
 * async wait, fails go out as mTCP left them, counted; a failed async post
 * falls back to the synchronous fill. */
static void part_faults(void)
{
	const uint32_t n = 700;
	uint64_t *off, bytes;
	uint16_t *len;
	uint8_t *buf = imix(n, 0xFA17, &off, &len, &bytes), *rx = malloc(bytes + 64);
	uint8_t *d = malloc(n), *f = malloc(2048);
	struct mini_stats s;
	struct gpucsum_stats g0, g1;
	struct mtcp_thread_context *ctx = (struct mtcp_thread_context *)(uintptr_t)0x2000;
	uint32_t i, filled = 0;
	int rc;

	memcpy(rx, buf, bytes + 64);
	for (i = 0; i < n; i++) {
		uint32_t c2;
		ref_tx_fill(rx + off[i], len[i], &c2);
	}
	setenv("GCS_FAULT_INJECT", "none", 1);           /* armed when the context is made */
	setenv("GPUCSUM_TX_GROUP", "8", 1);
	rc = gpucsum_set_inner(&synth_module_func);
	CHECK(rc == 0, "gpucsum_set_inner %d", rc);
	mini_start(&gpucsum_module_func, ctx);
	gpucsum_get_stats(ctx, &g0);

	setenv("GCS_FAULT_INJECT", "verify_ptrs", 1);
	synth_reset(64);
	synth_set_rx(rx, off, len, n);
	rc = mini_rx_loop(&gpucsum_module_func, ctx, 0, &s, d, n);
	gpucsum_get_stats(ctx, &g1);
	CHECK(rc == (int)n && s.accepted == 0 && s.rx_errors == n &&
	      g1.rx_unverified - g0.rx_unverified == n,
	      "RX verify failure: %d frames, %llu accepted, %llu unverified", rc,
	      (unsigned long long)s.accepted, (unsigned long long)(g1.rx_unverified - g0.rx_unverified));

	setenv("GCS_FAULT_INJECT", "wait", 1);             /* async waits fail: fills cancelled */
	synth_reset(64);
	mini_tx(&gpucsum_module_func, ctx, 0, buf, off, len, n, 64);
	gpucsum_get_stats(ctx, &g0);
	CHECK(synth_tx_sent() == n && g0.tx_unfilled_sent == n, "TX wait failure: %u sent, %llu unfilled",
	      synth_tx_sent(), (unsigned long long)g0.tx_unfilled_sent);
	for (i = 0; i < n; i++) {
		synth_tx_frame(i, f);
		filled += f[24] != 0 || f[25] != 0;            /* no check written */
	}
	CHECK(filled == 0, "%u frames with an IP check after cancelled fills", filled);

	setenv("GCS_FAULT_INJECT", "compute_async", 1);    /* async post fails: sync fill */
	synth_reset(64);
	mini_tx(&gpucsum_module_func, ctx, 0, buf, off, len, n, 64);
	gpucsum_get_stats(ctx, &g1);
	filled = 0;
	for (i = 0; i < n; i++) {
		uint32_t c2;
		memcpy(rx, buf + off[i], len[i]);
		if (ref_tx_fill(rx, len[i], &c2) < 0)
			continue;
		synth_tx_frame(i, f);
		filled += memcmp(rx, f, len[i]) != 0;
	}
	CHECK(synth_tx_sent() == n && filled == 0 && g1.tx_unfilled_sent == g0.tx_unfilled_sent,
	      "TX after a failed post: %u sent, %u differ from the oracle", synth_tx_sent(), filled);
	mini_stop(&gpucsum_module_func, ctx);
	unsetenv("GCS_FAULT_INJECT");
	unsetenv("GPUCSUM_TX_GROUP");
	printf("part 7 GPU-failure paths: RX burst NULL, TX unfilled counted %llu, failures %llu\n",
	       (unsigned long long)g1.tx_unfilled_sent, (unsigned long long)g1.gpu_failures);
	free(buf); free(rx); free(d); free(f); free(off); free(len);
}

int main(void)
{
	uint64_t mism = 0, frames = 0;
	double us = 0;
	int rc;

	rc = mt_bursts(4, 40, 1, &mism, &frames, &us);
	CHECK(rc == 0 && mism == 0, "mt_bursts (server) rc %d mismatches %llu", rc,
	      (unsigned long long)mism);
	printf("part 1 threads, burst server: %llu frames, mismatches %llu\n",
	       (unsigned long long)frames, (unsigned long long)mism);
	rc = mt_bursts(3, 20, 0, &mism, &frames, &us);
	CHECK(rc == 0 && mism == 0, "mt_bursts (launch per call) rc %d mismatches %llu", rc,
	      (unsigned long long)mism);
	printf("part 1 threads, one launch per call: %llu frames, mismatches %llu\n",
	       (unsigned long long)frames, (unsigned long long)mism);
	part_host_batch();
	part_registered();
	part_plugin();
	part_errors();
	part_async(0);
	part_async(1);
	part_faults();
	if (g_fail) {
		printf("HOST DRIVER FAILED\n");
		return 1;
	}
	printf("HOST DRIVER OK\n");
	return 0;
}
