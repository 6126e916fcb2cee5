/* sanitize_check.c -- memory-safety fuzz of the oracle (test infrastructure).
 *
 * SURVEY.md §5 (race detection / sanitizers): the reference has none, and its
 * own folds read past short buffers (tcp_in.c:1231 trusts tot_len; ps.h's
 * generic ip_fast_csum overruns for ihl <= 4).  The oracle defines those cases
 * (DROP_TRUNC, BAD_DESC ...) and must never read or write outside a frame.
 * This driver builds seeded random frames -- mostly well-formed mTCP frames,
 * with ihl, tot_len, doff, protocol, ethertype and lengths mutated -- each in
 * its OWN exactly-sized heap block, so AddressSanitizer reports any access
 * past a frame, and runs every per-frame and batch entry point of
 * csum_ref.h over them under -fsanitize=address,undefined.
 *
 *   make -C oracle sanitize && oracle/_san/sanitize_check [iterations] [seed]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "csum_ref.h"

static uint64_t g_x = 0x6d746370u;

static uint32_t rnd(void)
{
	g_x ^= g_x << 13;
	g_x ^= g_x >> 7;
	g_x ^= g_x << 17;
	return (uint32_t)(g_x >> 11);
}

static uint32_t pick(uint32_t n) { return n ? rnd() % n : 0; }

/* An mTCP-shaped frame of `len` bytes (eth 14 | ip 4*ihl | tcp 4*doff | payload),
 * then some header fields mutated. */
static void make_frame(uint8_t *f, uint32_t len)
{
	for (uint32_t k = 0; k < len; k++)
		f[k] = (uint8_t)rnd();
	uint32_t ihl = pick(8) ? 5 : pick(16);
	uint32_t doff = pick(4) ? 8 : pick(16);
	uint32_t tot = len >= 14 ? len - 14 : 0;
	switch (pick(6)) {
	case 0: tot = pick(70000); break;          /* anything, incl. past the frame */
	case 1: tot = tot ? tot - pick(tot + 1) : 0; break;   /* Ethernet padding */
	default: break;
	}
	const uint8_t proto = pick(10) ? 6 : (pick(2) ? 1 : (uint8_t)rnd());
	if (len > 13) { f[12] = pick(20) ? 0x08 : (uint8_t)rnd(); f[13] = pick(20) ? 0 : (uint8_t)rnd(); }
	if (len > 14) f[14] = (uint8_t)((pick(20) ? 4 : pick(16)) << 4 | ihl);
	if (len > 17) { f[16] = (uint8_t)(tot >> 8); f[17] = (uint8_t)tot; }
	if (len > 23) f[23] = proto;
	const uint32_t ts = 14 + 4 * ihl;
	if (len > ts + 12) f[ts + 12] = (uint8_t)(doff << 4);
	if (pick(2)) {                         /* valid checks on half of them */
		uint32_t cs;
		ref_tx_fill_f(f, len, &cs, pick(2) ? REF_CF_ICMP : 0);
	}
	if (len && pick(8) == 0)
		f[pick(len)] ^= (uint8_t)(1 + pick(255));
}

static uint32_t frame_len(void)
{
	switch (pick(5)) {
	case 0: return pick(80);
	case 1: return 54 + pick(1460);
	case 2: return 64;
	case 3: return 1500;
	default: return pick(2100);
	}
}

int main(int argc, char **argv)
{
	const int iters = argc > 1 ? atoi(argv[1]) : 20000;
	if (argc > 2)
		g_x = strtoull(argv[2], NULL, 0) | 1;
	uint64_t acc = 0;

	/* 1. per-frame entry points, every frame in its own exact-size block */
	for (int it = 0; it < iters; it++) {
		const uint32_t len = frame_len();
		uint8_t *f = malloc(len ? len : 1);
		make_frame(f, len);
		uint8_t *g = malloc(len ? len : 1);
		memcpy(g, f, len);
		acc += (uint32_t)ref_rx_verdict(g, len, REF_VF_ZERO_BAD_TCP_CHECK | (pick(2) ? REF_VF_ICMP : 0));
		memcpy(g, f, len);
		uint32_t cs = 0;
		acc += (uint32_t)ref_tx_fill_f(g, len, &cs, pick(2) ? REF_CF_ICMP : 0) + cs;
		/* payload source of exactly the size the headers ask for, or less */
		const uint32_t sl = pick(len + 64);
		uint8_t *src = malloc(sl ? sl : 1);
		for (uint32_t k = 0; k < sl; k++)
			src[k] = (uint8_t)rnd();
		memcpy(g, f, len);
		acc += (uint32_t)ref_tx_copy_fill(g, len, pick(16) ? src : NULL, sl, &cs) + cs;
		/* the element-wise folds on exact buffers */
		if (len >= 2) {
			const uint32_t o = 2 * pick(len / 2);
			uint32_t l = len - o;
			if (l & 1)
				l--;                   /* the reference reads the whole last halfword */
			acc += ref_tcp_calc_checksum(f + o, (uint16_t)l, rnd(), rnd());
			acc += ref_icmp_checksum(f + o, (int)(len - o));
		}
		if (len >= 4) {
			const unsigned ihl = pick(16);
			if (ihl <= 4 || 4 * ihl <= len)
				acc += ref_ip_fast_csum(f, ihl);
		}
		acc += (uint32_t)ref_rss_core(len < 16 || pick(2) ? NULL : f, rnd(), rnd(), (uint16_t)rnd(),
		                              (uint16_t)rnd(), 1 + (int)pick(64), (int)pick(2));
		free(src);
		free(g);
		free(f);
	}

	/* 2. batch entry points over one packed buffer that ends at the last frame */
	for (int rep = 0; rep < 40; rep++) {
		const uint32_t n = 1 + pick(300);
		uint64_t *off = malloc(n * sizeof *off);
		uint16_t *ln = malloc(n * sizeof *ln);
		uint64_t total = 0;
		for (uint32_t i = 0; i < n; i++) {
			total = (total + 15) & ~15ull;
			off[i] = total;
			ln[i] = (uint16_t)frame_len();
			total += ln[i];
		}
		uint8_t *buf = malloc(total ? total : 1);
		for (uint32_t i = 0; i < n; i++)
			make_frame(buf + off[i], ln[i]);
		for (uint32_t i = 0; i < n; i++)       /* a few descriptors out of the buffer */
			if (pick(50) == 0)
				off[i] = total - pick(32) + 16 * pick(3);
		uint8_t *v = malloc(n);
		uint32_t *cs = malloc(n * sizeof *cs), *h = malloc(n * sizeof *h);
		uint16_t *q = malloc(n * sizeof *q);
		ref_verify_batch(buf, total, off, ln, n, v, REF_VF_ZERO_BAD_TCP_CHECK);
		ref_classify_batch(buf, total, off, ln, n, v, h, q, REF_VF_ICMP, NULL, 16, 1);
		ref_compute_batch_f(buf, total, off, ln, n, v, cs, REF_CF_ICMP);
		const uint64_t sb = 4096 + pick(4096);
		uint8_t *src = malloc(sb);
		memset(src, 0x5A, sb);
		uint64_t *so = malloc(n * sizeof *so);
		for (uint32_t i = 0; i < n; i++)
			so[i] = pick((uint32_t)sb + 64);
		ref_compute_copy_batch(buf, total, off, ln, n, src, sb, so, v, cs);
		ref_verify_batch(buf, total, off, ln, n, v, 0);
		const uint64_t ob = pick(2) ? total : total / 2 + pick(64);
		uint8_t *out = malloc(ob ? ob : 1);
		uint64_t *oo = malloc(n * sizeof *oo);
		uint16_t *ol = malloc(n * sizeof *ol);
		ref_gro_batch(buf, total, off, ln, v, n, 1 + pick(256), 64 + pick(65472), out, ob, oo,
		              ol, h);
		for (uint32_t i = 0; i < n; i++)
			acc += v[i] + cs[i] + h[i] + ol[i];
		free(ol); free(oo); free(out); free(so); free(src);
		free(q); free(h); free(cs); free(v); free(buf); free(ln); free(off);
	}
	printf("sanitize_check ok: %d frames + 40 batches, digest %llu\n", iters,
	       (unsigned long long)acc);
	return 0;
}
