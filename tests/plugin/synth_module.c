/*
 * synth_module.c -- a synthetic NIC behind mTCP's io_module_func (TEST ONLY).
 *
 * Plays the role dpdk_module.c plays in production: RX hands out bursts of at
 * most `burst` frames (MAX_PKT_BURST = 64, dpdk_module.c:76) from a queue the
 * test loads, each frame in its own 2 KiB buffer (an mbuf's data room); TX
 * hands out 2 KiB buffers from get_wptr and "transmits" them into a capture
 * buffer the test reads back.  dev_ioctl is NULL (like psio/netmap,
 * psio_module.c:399, netmap_module.c:268), so mTCP-shaped callers run the
 * software checksum path when this module is used directly.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gpucsum_io_module.h"

#define SYN_BUF 2048
#define SYN_MAX_TX 65536

static struct {
	/* RX wire queue */
	uint8_t *rx_bufs;            /* n * SYN_BUF */
	uint16_t *rx_len;
	uint32_t rx_n, rx_next, burst;
	uint32_t cur_first, cur_n;   /* current burst */
	/* TX */
	uint8_t *tx_bufs;            /* SYN_MAX_TX * SYN_BUF */
	uint16_t tx_len[SYN_MAX_TX];
	uint32_t tx_pending, tx_sent;
	uint32_t released, sends;
} S;

int synth_reset(uint32_t burst)
{
	free(S.rx_bufs);
	free(S.rx_len);
	free(S.tx_bufs);
	memset(&S, 0, sizeof(S));
	S.burst = burst ? burst : 64;
	S.tx_bufs = calloc(SYN_MAX_TX, SYN_BUF);
	return S.tx_bufs ? 0 : -1;
}

/* Queue n frames (buf + off[i], len[i] bytes) on the RX wire. */
int synth_set_rx(const uint8_t *buf, const uint64_t *off, const uint16_t *len, uint32_t n)
{
	uint32_t i;

	free(S.rx_bufs);
	free(S.rx_len);
	S.rx_bufs = calloc(n ? n : 1, SYN_BUF);
	S.rx_len = calloc(n ? n : 1, sizeof(uint16_t));
	if (!S.rx_bufs || !S.rx_len)
		return -1;
	for (i = 0; i < n; i++) {
		uint16_t l = len[i] > SYN_BUF ? SYN_BUF : len[i];
		memcpy(S.rx_bufs + (uint64_t)i * SYN_BUF, buf + off[i], l);
		S.rx_len[i] = l;
	}
	S.rx_n = n;
	S.rx_next = 0;
	S.cur_n = 0;
	return 0;
}

uint32_t synth_tx_sent(void) { return S.tx_sent; }

/* The RX rooms (rx_n x SYN_BUF bytes, the frames as the NIC "received" them):
 * for registering them as an mbuf pool would be registered (gcs_host_register). */
uint8_t *synth_rx_base(uint64_t *bytes)
{
	*bytes = (uint64_t)(S.rx_n ? S.rx_n : 1) * SYN_BUF;
	return S.rx_bufs;
}

/* The TX rooms (SYN_MAX_TX x SYN_BUF bytes): for registering them as an mbuf
 * pool would be registered (gcs_host_register). */
uint8_t *synth_tx_base(uint64_t *bytes)
{
	*bytes = (uint64_t)SYN_MAX_TX * SYN_BUF;
	return S.tx_bufs;
}
uint32_t synth_released(void) { return S.released; }
uint32_t synth_sends(void) { return S.sends; }

/* Copy transmitted frame k out (returns its length). */
int synth_tx_frame(uint32_t k, uint8_t *out)
{
	if (k >= S.tx_sent)
		return -1;
	memcpy(out, S.tx_bufs + (uint64_t)k * SYN_BUF, S.tx_len[k]);
	return S.tx_len[k];
}

static void syn_load(void) {}
static void syn_init(struct mtcp_thread_context *ctx) { (void)ctx; }
static int32_t syn_link(struct mtcp_thread_context *ctx) { (void)ctx; return 0; }

static void syn_release(struct mtcp_thread_context *ctx, int ifidx, unsigned char *p, int len)
{
	(void)ctx; (void)ifidx; (void)p; (void)len;
	S.released++;
}

static uint8_t *syn_get_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
	uint32_t k = S.tx_sent + S.tx_pending;
	(void)ctx; (void)ifidx;
	if (k >= SYN_MAX_TX || len > SYN_BUF)
		return NULL;
	S.tx_len[k] = len;
	S.tx_pending++;
	memset(S.tx_bufs + (uint64_t)k * SYN_BUF, 0, SYN_BUF);
	return S.tx_bufs + (uint64_t)k * SYN_BUF;
}

static int32_t syn_send(struct mtcp_thread_context *ctx, int nif)
{
	int32_t n = (int32_t)S.tx_pending;
	(void)ctx; (void)nif;
	S.tx_sent += S.tx_pending;
	S.tx_pending = 0;
	S.sends++;
	return n;
}

static int32_t syn_recv(struct mtcp_thread_context *ctx, int ifidx)
{
	uint32_t left = S.rx_n - S.rx_next;
	(void)ctx; (void)ifidx;
	S.cur_first = S.rx_next;
	S.cur_n = left < S.burst ? left : S.burst;
	S.rx_next += S.cur_n;
	return (int32_t)S.cur_n;
}

static uint8_t *syn_get_rptr(struct mtcp_thread_context *ctx, int ifidx, int index,
                             uint16_t *len)
{
	uint32_t i;
	(void)ctx; (void)ifidx;
	if (index < 0 || (uint32_t)index >= S.cur_n)
		return NULL;
	i = S.cur_first + (uint32_t)index;
	*len = S.rx_len[i];
	return S.rx_bufs + (uint64_t)i * SYN_BUF;
}

static int32_t syn_select(struct mtcp_thread_context *ctx) { (void)ctx; return 0; }
static void syn_destroy(struct mtcp_thread_context *ctx) { (void)ctx; }

io_module_func synth_module_func = {
	.load_module    = syn_load,
	.init_handle    = syn_init,
	.link_devices   = syn_link,
	.release_pkt    = syn_release,
	.get_wptr       = syn_get_wptr,
	.send_pkts      = syn_send,
	.get_rptr       = syn_get_rptr,
	.recv_pkts      = syn_recv,
	.select         = syn_select,
	.destroy_handle = syn_destroy,
	.dev_ioctl      = NULL,
};
