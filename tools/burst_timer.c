/*
 * burst_timer.c -- per-call latency of the host-batch entry points as a C
 * caller (the io_module plugin, mTCP) sees it: clock_gettime around each
 * call, no interpreter in the loop (MEASUREMENT TOOL, not product code).
 * The entry point comes in as a function pointer, so this library does not
 * link libmtcp_gpucsum itself.
 */
#include <stdint.h>
#include <time.h>

typedef int (*burst_fn)(void *ctx, uint8_t *const *pkts, const uint16_t *len, uint32_t n,
                        uint8_t *out, void *extra);

static double now_us(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

/* reps calls of fn(ctx, pkts, len, n, out, extra); us[r] = duration of call r.
 * Returns the first non-zero status, or 0. */
int bt_run(burst_fn fn, void *ctx, uint8_t *const *pkts, const uint16_t *len, uint32_t n,
           uint8_t *out, void *extra, uint32_t reps, double *us)
{
	uint32_t r;
	for (r = 0; r < reps; r++) {
		double t0 = now_us();
		int rc = fn(ctx, pkts, len, n, out, extra);
		us[r] = now_us() - t0;
		if (rc)
			return rc;
	}
	return 0;
}
