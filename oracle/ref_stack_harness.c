/*
 * ref_stack_harness.c -- drives mTCP's OWN RX/TX code around the checksum
 * path through any io_module_func (TEST INFRASTRUCTURE ONLY; never linked into
 * the product).
 *
 * oracle/Makefile compiles the reference's eth_in.c, ip_in.c, tcp_in.c,
 * icmp.c, ip_out.c, tcp_out.c, eth_out.c, arp.c and tcp_util.c in place from
 * /root/reference with the reference flags and WITHOUT -DDISABLE_HWCSUM, i.e.
 * exactly the objects in which every fold is guarded by mtcp->iom->dev_ioctl
 * (ip_in.c:28-37, tcp_in.c:1224-1241, ip_out.c:84-101, tcp_out.c:202-214).
 * This file supplies what those objects need around the checksum prefix:
 *
 *   CONFIG        one port (eths[0], nif_to_eidx), one route and one ARP entry
 *                 that match every address (ip_out.c:8-37, arp.c:98-128)
 *   mtcp_manager  zeroed except iom / ctx / cur_ts (core.c:1187-1190)
 *   RX loop       core.c:785-801: recv_pkts, get_rptr per index, NULL ->
 *                 rx_errors, else ProcessPacket (eth_in.c:9-60)
 *   TX            SendTCPPacketStandalone (tcp_out.c:135-217) per segment,
 *                 send_pkts every `burst` segments (core.c:846-848); and the
 *                 data path: SendTCPPacket -> IPOutput (tcp_out.c:223-357,
 *                 ip_out.c:106-175) over established tcp_streams with their
 *                 send/recv variables, timestamps and payload copy.  timer.c
 *                 is compiled in too: SendTCPPacket puts a stream with
 *                 payload on the RTO list (AddtoRTOList, tcp_out.c:350).
 *
 * Everything beyond the checksum path stays out of reach: ProcessTCPPacket's
 * first call after its checksum prefix is StreamHTSearch (tcp_in.c:1251),
 * which ref_stack_traps.c turns into a longjmp back here ("ACCEPT").  The
 * stack functions the objects reference but the checksum path never reaches
 * are traps that abort (ref_stack_traps.c).
 */
#include <setjmp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mtcp.h"
#include "eth_in.h"
#include "tcp_out.h"
#include "timer.h"
#include "tcp_in.h"

struct mtcp_config CONFIG;

/* ref_stack_traps.c */
extern jmp_buf refs_accept_jb;
extern int refs_accept_armed;

enum { REFS_ACCEPT = 0, REFS_ERROR = 1, REFS_TRUE = 2, REFS_FALSE = 3, REFS_NULL = 5 };

static struct eth_table g_eth[1];
static int g_nif_to_eidx[MAX_DEVICES];
static struct route_table g_route[1];
static struct arp_entry g_arp[1];
static struct mtcp_manager refs_mgr;

/* Configure the one port: our IP address (ICMP echo requests to it are
 * answered, icmp.c:110-119) and MACs. */
void refs_config(uint32_t my_ip)
{
	static const unsigned char src[6] = {0x02, 0, 0, 0, 0, 0x01};
	static const unsigned char dst[6] = {0x02, 0, 0, 0, 0, 0x02};
	int i;

	memset(&CONFIG, 0, sizeof(CONFIG));
	memset(g_eth, 0, sizeof(g_eth));
	strcpy(g_eth[0].dev_name, "gpucsum0");
	g_eth[0].ifindex = 0;
	memcpy(g_eth[0].haddr, src, 6);
	g_eth[0].ip_addr = my_ip;
	g_eth[0].netmask = 0;
	for (i = 0; i < MAX_DEVICES; i++)
		g_nif_to_eidx[i] = i == 0 ? 0 : -1;
	g_route[0].daddr = 0;
	g_route[0].mask = 0;
	g_route[0].masked = 0;
	g_route[0].prefix = 1;
	g_route[0].nif = 0;
	memset(g_arp, 0, sizeof(g_arp));
	g_arp[0].prefix = 8;              /* masked entry: matches every dip */
	g_arp[0].ip_mask = 0;
	g_arp[0].ip_masked = 0;
	memcpy(g_arp[0].haddr, dst, 6);
	CONFIG.eths = g_eth;
	CONFIG.eths_num = 1;
	CONFIG.nif_to_eidx = g_nif_to_eidx;
	CONFIG.rtable = g_route;
	CONFIG.routes = 1;
	CONFIG.arp.entry = g_arp;
	CONFIG.arp.entries = 1;
	CONFIG.num_cores = 1;
}

static void refs_bind(struct io_module_func *iom, struct mtcp_thread_context *ctx, uint32_t ts)
{
	memset(&refs_mgr, 0, sizeof(refs_mgr));
	refs_mgr.iom = iom;
	refs_mgr.ctx = ctx;
	refs_mgr.cur_ts = ts;
}

static int process_one(int ifidx, uint32_t ts, unsigned char *pkt, int len)
{
	int ret;

	refs_accept_armed = 1;
	if (setjmp(refs_accept_jb)) {
		refs_accept_armed = 0;
		return REFS_ACCEPT;                  /* reached StreamHTSearch */
	}
	ret = ProcessPacket(&refs_mgr, ifidx, ts, pkt, len);
	refs_accept_armed = 0;
	return ret < 0 ? REFS_ERROR : ret ? REFS_TRUE : REFS_FALSE;
}

static double refs_now_us(void);

/* refs_rx_loop, timed per burst when blocked_us is not NULL: blocked_us[b] =
 * the time burst b's recv_pkts and get_rptr calls kept the mTCP thread inside
 * the I/O module (core.c:789-793; through the decorator, the GPU verify it
 * waits for), burst_us[b] = recv_pkts to the end of the burst's last
 * ProcessPacket (core.c:789-801, without the send round). */
int refs_rx_loop_timed(struct io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                       uint8_t *disp, uint32_t max, uint64_t *rx_errors, double *blocked_us,
                       double *burst_us, double *recv_us, uint32_t max_bursts);

/* core.c:785-801 plus the send_pkts of core.c:846-848 after each round (ICMP
 * echo replies and ARP answers go out through get_wptr).  Returns frames seen;
 * disp[k] per frame in arrival order; *rx_errors as nstat.rx_errors counts them. */
int refs_rx_loop(struct io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                 uint8_t *disp, uint32_t max, uint64_t *rx_errors)
{
	return refs_rx_loop_timed(iom, ctx, ifidx, disp, max, rx_errors, NULL, NULL, NULL, 0);
}

int refs_rx_loop_timed(struct io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                       uint8_t *disp, uint32_t max, uint64_t *rx_errors, double *blocked_us,
                       double *burst_us, double *recv_us, uint32_t max_bursts)
{
	uint32_t k = 0, b = 0;
	int32_t n, i;
	const int timed = blocked_us != NULL;
	double t0 = 0, t1 = 0, in_mod = 0;

	refs_bind(iom, ctx, 1000);
	*rx_errors = 0;
	for (;;) {
		if (timed)
			t0 = refs_now_us();
		n = iom->recv_pkts(ctx, ifidx);
		if (timed) {
			in_mod = refs_now_us() - t0;
			if (recv_us && b < max_bursts)
				recv_us[b] = in_mod;
		}
		if (n <= 0)
			break;
		for (i = 0; i < n; i++) {
			uint16_t len = 0;
			unsigned char *p;
			int d;
			if (timed) {
				t1 = refs_now_us();
				p = iom->get_rptr(ctx, ifidx, i, &len);
				in_mod += refs_now_us() - t1;
			} else {
				p = iom->get_rptr(ctx, ifidx, i, &len);
			}
			d = p ? process_one(ifidx, refs_mgr.cur_ts, p, len) : REFS_NULL;
			if (d == REFS_NULL || d == REFS_ERROR)
				(*rx_errors)++;
			if (k < max)
				disp[k] = (uint8_t)d;
			k++;
		}
		if (timed && b < max_bursts) {
			blocked_us[b] = in_mod;
			burst_us[b] = refs_now_us() - t0;
		}
		b++;
		iom->send_pkts(ctx, ifidx);
		refs_mgr.cur_ts++;
	}
	return (int)k;
}

/* n segments through SendTCPPacketStandalone (tcp_out.c:135-217), which
 * builds the headers (IPOutputStandalone, ip_out.c:41-101; EthernetOutput,
 * eth_out.c:36-80), copies the payload and -- unless the module's dev_ioctl
 * answers 0 -- folds both checks.  Segment k: payload + pay_off[k],
 * pay_len[k] bytes (<= 1448 with the timestamp option), tuple / seq / flags
 * from the arrays.  Returns segments written (-1 on a NULL get_wptr that a
 * send round does not cure). */
int refs_tx_tcp(struct io_module_func *iom, struct mtcp_thread_context *ctx, uint32_t n,
                const uint32_t *saddr, const uint16_t *sport, const uint32_t *daddr,
                const uint16_t *dport, const uint32_t *seq, const uint32_t *ack,
                const uint16_t *window, const uint8_t *flags, const uint8_t *payload,
                const uint64_t *pay_off, const uint16_t *pay_len, uint32_t burst)
{
	uint32_t k;

	refs_bind(iom, ctx, 5000);
	for (k = 0; k < n; k++) {
		int rc = SendTCPPacketStandalone(&refs_mgr, saddr[k], sport[k], daddr[k], dport[k],
		                                 seq[k], ack[k], window[k], flags[k],
		                                 (uint8_t *)payload + pay_off[k], pay_len[k],
		                                 refs_mgr.cur_ts, 77u + k);
		if (rc < 0) {
			iom->send_pkts(ctx, 0);          /* tcp_out.c:799-802: retry later */
			rc = SendTCPPacketStandalone(&refs_mgr, saddr[k], sport[k], daddr[k], dport[k],
			                             seq[k], ack[k], window[k], flags[k],
			                             (uint8_t *)payload + pay_off[k], pay_len[k],
			                             refs_mgr.cur_ts, 77u + k);
			if (rc < 0)
				return -1;
		}
		if (burst && (k + 1) % burst == 0)
			iom->send_pkts(ctx, 0);
	}
	iom->send_pkts(ctx, 0);
	return (int)n;
}

/* mTCP's data path: SendTCPPacket (tcp_out.c:223-357) -> IPOutput
 * (ip_out.c:106-175) -> EthernetOutput over `ns` established streams, as
 * FlushTCPSendingBuffer / SendControlPacket call it.  Stream j: the tuple in
 * network order, snd_nxt / rcv_nxt, the receive window and the peer's last
 * timestamp (echoed in every segment's TS option, tcp_out.c:62-70), MSS 1460
 * (so payloads up to 1448 B with the 12 B timestamp option).  Segment k goes
 * out on stream sidx[k] with flags[k] and payload bytes pay_off/pay_len;
 * cur_ts advances by one per send round.  Returns segments written, or -1 on a
 * NULL get_wptr that a send round does not cure (tcp_out.c:799-802 retries). */
static double refs_now_us(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

/* refs_tx_stream, with send_us[k] = the time the k-th every-`burst` send_pkts
 * call blocked the mTCP thread (core.c:846-848), when send_us is not NULL. */
int refs_tx_stream_timed(struct io_module_func *iom, struct mtcp_thread_context *ctx,
                         uint32_t ns, const uint32_t *saddr, const uint16_t *sport,
                         const uint32_t *daddr, const uint16_t *dport, const uint32_t *snd_nxt,
                         const uint32_t *rcv_nxt, const uint32_t *rcv_wnd,
                         const uint32_t *ts_recent, uint32_t n, const uint16_t *sidx,
                         const uint8_t *flags, const uint8_t *payload, const uint64_t *pay_off,
                         const uint16_t *pay_len, uint32_t burst, double *send_us);

int refs_tx_stream(struct io_module_func *iom, struct mtcp_thread_context *ctx, uint32_t ns,
                   const uint32_t *saddr, const uint16_t *sport, const uint32_t *daddr,
                   const uint16_t *dport, const uint32_t *snd_nxt, const uint32_t *rcv_nxt,
                   const uint32_t *rcv_wnd, const uint32_t *ts_recent, uint32_t n,
                   const uint16_t *sidx, const uint8_t *flags, const uint8_t *payload,
                   const uint64_t *pay_off, const uint16_t *pay_len, uint32_t burst)
{
	return refs_tx_stream_timed(iom, ctx, ns, saddr, sport, daddr, dport, snd_nxt, rcv_nxt,
	                            rcv_wnd, ts_recent, n, sidx, flags, payload, pay_off, pay_len,
	                            burst, NULL);
}

int refs_tx_stream_timed(struct io_module_func *iom, struct mtcp_thread_context *ctx,
                         uint32_t ns, const uint32_t *saddr, const uint16_t *sport,
                         const uint32_t *daddr, const uint16_t *dport, const uint32_t *snd_nxt,
                         const uint32_t *rcv_nxt, const uint32_t *rcv_wnd,
                         const uint32_t *ts_recent, uint32_t n, const uint16_t *sidx,
                         const uint8_t *flags, const uint8_t *payload, const uint64_t *pay_off,
                         const uint16_t *pay_len, uint32_t burst, double *send_us)
{
	uint32_t kb = 0;
	tcp_stream *st;
	struct tcp_send_vars *sv;
	struct tcp_recv_vars *rv;
	uint32_t j, k;
	int ret = (int)n;

	refs_bind(iom, ctx, 7000);
	refs_mgr.rto_store = InitRTOHashstore();
	st = calloc(ns, sizeof(*st));
	sv = calloc(ns, sizeof(*sv));
	rv = calloc(ns, sizeof(*rv));
	if (!refs_mgr.rto_store || !st || !sv || !rv) {
		ret = -1;
		goto out;
	}
	for (j = 0; j < ns; j++) {
		st[j].sndvar = &sv[j];
		st[j].rcvvar = &rv[j];
		st[j].id = j;
		st[j].saddr = saddr[j];
		st[j].daddr = daddr[j];
		st[j].sport = sport[j];
		st[j].dport = dport[j];
		st[j].state = TCP_ST_ESTABLISHED;
		st[j].on_rto_idx = -1;
		st[j].snd_nxt = snd_nxt[j];
		st[j].rcv_nxt = rcv_nxt[j];
		sv[j].iss = snd_nxt[j];
		sv[j].snd_una = snd_nxt[j];
		sv[j].mss = TCP_DEFAULT_MSS;
		sv[j].eff_mss = TCP_DEFAULT_MSS - TCP_OPT_TIMESTAMP_LEN - 2;
		sv[j].wscale_mine = TCP_DEFAULT_WSCALE;
		sv[j].nif_out = -1;           /* IPOutput routes it (ip_out.c:114-118) */
		sv[j].ip_id = (uint16_t)(0x1234 + 97 * j);
		sv[j].rto = TCP_INITIAL_RTO;
		rv[j].rcv_wnd = rcv_wnd[j];
		rv[j].ts_recent = ts_recent[j];
	}
	for (k = 0; k < n; k++) {
		tcp_stream *s = &st[sidx[k] < ns ? sidx[k] : 0];
		uint8_t *pl = (uint8_t *)payload + pay_off[k];
		int rc = SendTCPPacket(&refs_mgr, s, refs_mgr.cur_ts, flags[k], pl, pay_len[k]);
		if (rc == -2) {
			iom->send_pkts(ctx, 0);
			refs_mgr.cur_ts++;
			rc = SendTCPPacket(&refs_mgr, s, refs_mgr.cur_ts, flags[k], pl, pay_len[k]);
		}
		if (rc < 0) {
			ret = -1;
			goto out;
		}
		if (burst && (k + 1) % burst == 0) {
			double t0 = refs_now_us();
			iom->send_pkts(ctx, 0);
			if (send_us)
				send_us[kb] = refs_now_us() - t0;
			kb++;
			refs_mgr.cur_ts++;
		}
	}
	iom->send_pkts(ctx, 0);
out:
	free(st);
	free(sv);
	free(rv);
	if (refs_mgr.rto_store) {
		free(refs_mgr.rto_store);
		refs_mgr.rto_store = NULL;
	}
	return ret;
}
