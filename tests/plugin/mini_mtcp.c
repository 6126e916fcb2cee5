/*
 * mini_mtcp.c -- the control flow of mTCP around the checksum path, restated
 * for tests (TEST ONLY; software folds come from the oracle, oracle/csum_ref.c).
 *
 * As compiled WITHOUT -DDISABLE_HWCSUM, i.e. every fold is guarded by the
 * module's dev_ioctl answer (a NULL dev_ioctl means software):
 *   RX  core.c:785-801       recv_pkts, get_rptr per index, NULL -> rx_errors
 *       eth_in.c:35-53       ethertype dispatch, ret < 0 -> rx_errors
 *       ip_in.c:21-59        ip_len < 20, PKT_RX_IP_CSUM / ip_fast_csum, version,
 *                            protocol dispatch
 *       tcp_in.c:1221-1241   length check, PKT_RX_TCP_CSUM / TCPCalcChecksum,
 *                            tcph->check = 0 on failure
 *   TX  eth_out.c:58         get_wptr(iplen + 14)
 *       ip_out.c:143-173     header with check = 0, PKT_TX_TCPIP_CSUM_PEEK (TCP) or
 *                            PKT_TX_IP_CSUM (other) / ip_fast_csum
 *       tcp_out.c:244,323-333  TCP header zeroed, PKT_TX_TCPIP_CSUM / TCPCalcChecksum
 *       core.c:846-848       send_pkts
 * Reads the reference would make past the frame (undefined there) are
 * counted as errors, as in the oracle.
 */
#include <stdint.h>
#include <string.h>
#include <time.h>

#include "../../include/gpucsum_io_module.h"
#include "../../oracle/csum_ref.h"

enum { MINI_ACCEPT = 0, MINI_ERROR = 1, MINI_RELEASE = 2, MINI_NOT_TCP = 3, MINI_NON_IP = 4,
       MINI_NULL = 5 };

struct mini_stats {
	uint64_t rx_packets, rx_errors, accepted, released, not_tcp, non_ip;
};

static uint16_t ld16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t ld32(const uint8_t *p)
{
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
	       ((uint32_t)p[3] << 24);
}
static uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }

static int process_tcp(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                       uint8_t *pkt, uint32_t len, uint8_t *iph, uint32_t ip_len)
{
	uint32_t ihl = iph[0] & 15, ts = 14 + 4 * ihl, doff;
	uint8_t *tcph = iph + 4 * ihl;
	int rc = -1;

	if (ts + 13 > len)
		return MINI_ERROR;
	doff = tcph[12] >> 4;
	if (ip_len < 4 * (ihl + doff))                            /* tcp_in.c:1221 */
		return MINI_ERROR;
	if (iom->dev_ioctl)                                        /* tcp_in.c:1227 */
		rc = iom->dev_ioctl(ctx, ifidx, PKT_RX_TCP_CSUM, NULL);
	if (rc == -1) {
		if (14 + ip_len > len)
			return MINI_ERROR;
		if (ref_tcp_calc_checksum(tcph, (uint16_t)(ip_len - 4 * ihl), ld32(iph + 12),
		                          ld32(iph + 16))) {
			if (ts + 18 <= len)
				tcph[16] = tcph[17] = 0;                   /* tcp_in.c:1237 */
			return MINI_ERROR;
		}
	}
	return MINI_ACCEPT;
}

static int process_ipv4(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                        uint8_t *pkt, uint32_t len)
{
	uint8_t *iph = pkt + 14;
	uint32_t ip_len, ihl;
	int rc = -1;

	if (len < 34)
		return MINI_ERROR;
	ip_len = be16(iph + 2);
	ihl = iph[0] & 15;
	if (ip_len < 20)                                           /* ip_in.c:25 */
		return MINI_ERROR;
	if (iom->dev_ioctl)                                        /* ip_in.c:29-30 */
		rc = iom->dev_ioctl(ctx, ifidx, PKT_RX_IP_CSUM, iph);
	if (rc == -1) {
		if (ihl >= 5 && 14 + 4 * ihl > len)
			return MINI_ERROR;
		if (ref_ip_fast_csum(iph, ihl))                    /* ip_in.c:31 */
			return MINI_ERROR;
	}
	if ((iph[0] >> 4) != 4) {                                 /* ip_in.c:47-50 */
		if (iom->release_pkt)
			iom->release_pkt(ctx, ifidx, pkt, (int)len);
		return MINI_RELEASE;
	}
	if (iph[9] == 6)
		return process_tcp(iom, ctx, ifidx, pkt, len, iph, ip_len);
	return MINI_NOT_TCP;
}

static int process_packet(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                          uint8_t *pkt, uint32_t len)
{
	if (len < 14)
		return MINI_ERROR;
	if (ld16(pkt + 12) != 0x0008)                              /* eth_in.c:35 */
		return MINI_NON_IP;
	return process_ipv4(iom, ctx, ifidx, pkt, len);
}

/* Lifecycle as mtcp_init / MTCPRunThread / mtcp_free_context drive it
 * (core.c:1639, :1190, :1232, :1490). */
int mini_start(io_module_func *iom, struct mtcp_thread_context *ctx)
{
	if (iom->load_module)
		iom->load_module();
	if (iom->init_handle)
		iom->init_handle(ctx);
	return iom->link_devices ? iom->link_devices(ctx) : 0;
}

void mini_stop(io_module_func *iom, struct mtcp_thread_context *ctx)
{
	if (iom->destroy_handle)
		iom->destroy_handle(ctx);
}

int32_t mini_ioctl(io_module_func *iom, struct mtcp_thread_context *ctx, int nif, int cmd,
                   void *argp)
{
	return iom->dev_ioctl ? iom->dev_ioctl(ctx, nif, cmd, argp) : -1;
}

size_t mini_vtable_size(void) { return sizeof(io_module_func); }

/* Run RX bursts until the module returns 0 frames; disposition per frame. */
int mini_rx_loop(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                 struct mini_stats *st, uint8_t *disp, uint32_t max)
{
	uint32_t k = 0;
	int32_t n, i;

	memset(st, 0, sizeof(*st));
	while ((n = iom->recv_pkts(ctx, ifidx)) > 0) {            /* core.c:789 */
		for (i = 0; i < n; i++) {
			uint16_t len = 0;
			uint8_t *p = iom->get_rptr(ctx, ifidx, i, &len);
			int d;
			st->rx_packets++;
			if (!p) {                                  /* core.c:794-799 */
				st->rx_errors++;
				d = MINI_NULL;
			} else {
				d = process_packet(iom, ctx, ifidx, p, len);
				if (d == MINI_ERROR)
					st->rx_errors++;           /* eth_in.c:49-53 */
				else if (d == MINI_ACCEPT)
					st->accepted++;
				else if (d == MINI_RELEASE)
					st->released++;
				else if (d == MINI_NOT_TCP)
					st->not_tcp++;
				else
					st->non_ip++;
			}
			if (k < max)
				disp[k] = (uint8_t)d;
			k++;
		}
	}
	return (int)k;
}

/* RX loop that also delivers each ACCEPT frame's TCP payload the way
 * RBPut's __MEMCPY_DATA_2_BUFFER does under ENABLELRO (tcp_ring_buffer.c:15-21):
 * a payload longer than TCP_DEFAULT_MSS (tcp_in.h:36) is an LRO chain and is
 * gathered by dev_ioctl(PKT_RX_TCP_LROSEG) from the module's current mbuf when
 * `lro` is set (the module-identity test of tcp_ring_buffer.c:18), otherwise
 * memcpy'd.  Payload k goes to out + out_off[k] (out_off[k] = ~0 for frames
 * that delivered nothing). */
int mini_rx_deliver(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                    struct mini_stats *st, uint8_t *disp, uint32_t max, int lro,
                    uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint32_t *out_len)
{
	uint32_t k = 0;
	uint64_t used = 0;
	int32_t n, i;

	memset(st, 0, sizeof(*st));
	while ((n = iom->recv_pkts(ctx, ifidx)) > 0) {
		for (i = 0; i < n; i++) {
			uint16_t len = 0;
			uint8_t *p = iom->get_rptr(ctx, ifidx, i, &len);
			int d;
			st->rx_packets++;
			if (k < max) {
				out_off[k] = ~(uint64_t)0;
				out_len[k] = 0;
			}
			if (!p) {
				st->rx_errors++;
				d = MINI_NULL;
			} else {
				d = process_packet(iom, ctx, ifidx, p, len);
				if (d == MINI_ERROR)
					st->rx_errors++;
				else if (d == MINI_ACCEPT)
					st->accepted++;
				else if (d == MINI_RELEASE)
					st->released++;
				else if (d == MINI_NOT_TCP)
					st->not_tcp++;
				else
					st->non_ip++;
			}
			if (d == MINI_ACCEPT && k < max) {
				uint8_t *iph = p + 14;
				uint32_t ihl = iph[0] & 15, ip_len = be16(iph + 2);
				uint8_t *tcph = iph + 4 * ihl;
				uint32_t hl = 4 * (ihl + (tcph[12] >> 4));
				uint32_t plen = ip_len - hl;
				if (used + plen <= out_cap) {
					if (lro && plen > 1460)        /* TCP_DEFAULT_MSS */
						iom->dev_ioctl(ctx, 0, PKT_RX_TCP_LROSEG, out + used);
					else
						memcpy(out + used, tcph + (hl - 4 * ihl), plen);
					out_off[k] = used;
					out_len[k] = plen;
					used += plen;
				}
			}
			if (k < max)
				disp[k] = (uint8_t)d;
			k++;
		}
	}
	return (int)k;
}

int32_t mini_send(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx)
{
	return iom->send_pkts(ctx, ifidx);
}

/* TX: write n prepared frames (check fields as mTCP leaves them: 0) through
 * the module in mTCP's order, flushing with send_pkts every `burst` frames. */
static double now_us(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int mini_tx_impl(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                        const uint8_t *buf, const uint64_t *off, const uint16_t *len,
                        uint32_t n, uint32_t burst, double *send_us, double *burst_us);

int mini_tx(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
            const uint8_t *buf, const uint64_t *off, const uint16_t *len, uint32_t n,
            uint32_t burst)
{
	return mini_tx_impl(iom, ctx, ifidx, buf, off, len, n, burst, NULL, NULL);
}

/* mini_tx, timed: send_us[k] = the k-th send_pkts call (what blocks the mTCP
 * thread after its burst, core.c:846-848), burst_us[k] = its whole burst from
 * the first get_wptr to send_pkts' return (clock_gettime, microseconds). */
int mini_tx_timed(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                  const uint8_t *buf, const uint64_t *off, const uint16_t *len, uint32_t n,
                  uint32_t burst, double *send_us, double *burst_us)
{
	return mini_tx_impl(iom, ctx, ifidx, buf, off, len, n, burst, send_us, burst_us);
}

/* mTCP's TX ioctls name the route's interface (ifindex: sndvar->nif_out,
 * tcp_out.c:206, 326) while get_wptr / send_pkts take the configured port's
 * eidx (CONFIG.nif_to_eidx[nif], eth_out.c:52; core.c:846).  They differ
 * whenever the configured ports are not 0..n-1; the loop models that. */
#define MINI_NIF(eidx) ((eidx) + 3)

static int mini_tx_impl(io_module_func *iom, struct mtcp_thread_context *ctx, int ifidx,
                        const uint8_t *buf, const uint64_t *off, const uint16_t *len,
                        uint32_t n, uint32_t burst, double *send_us, double *burst_us)
{
	uint32_t i, sent = 0, k = 0;
	double t_burst = now_us();

	for (i = 0; i < n; i++) {
		const uint8_t *src = buf + off[i];
		uint32_t L = len[i], ihl = src[14] & 15;
		uint8_t *f = iom->get_wptr(ctx, ifidx, (uint16_t)L);   /* eth_out.c:58 */
		int rc = -1;

		if (!f) {
			/* no TX buffer: the stream stays queued (tcp_out.c:799-802) and
			 * goes out after the next send_pkts round frees buffers */
			iom->send_pkts(ctx, ifidx);
			f = iom->get_wptr(ctx, ifidx, (uint16_t)L);
		}
		if (!f)
			return -1;
		/* Ethernet + IP header, check = 0 (ip_out.c:143-153) */
		memcpy(f, src, 14 + 4 * ihl);
		f[24] = f[25] = 0;
		if (iom->dev_ioctl)                                /* ip_out.c:157-166 */
			rc = iom->dev_ioctl(ctx, MINI_NIF(ifidx), src[23] == 6 ? PKT_TX_TCPIP_CSUM_PEEK
			                                             : PKT_TX_IP_CSUM, f + 14);
		if (rc == -1) {
			uint16_t c = ref_ip_fast_csum(f + 14, ihl);  /* ip_out.c:168 */
			memcpy(f + 24, &c, 2);
		}
		/* TCP header zeroed then filled, payload copied (tcp_out.c:244-321) */
		memcpy(f + 14 + 4 * ihl, src + 14 + 4 * ihl, L - 14 - 4 * ihl);
		if (src[23] == 6) {
			uint8_t *tcph = f + 14 + 4 * ihl;
			uint32_t ip_len = be16(f + 16);
			tcph[16] = tcph[17] = 0;
			rc = -1;
			if (iom->dev_ioctl)                        /* tcp_out.c:325-327 */
				rc = iom->dev_ioctl(ctx, MINI_NIF(ifidx), PKT_TX_TCPIP_CSUM, NULL);
			if (rc == -1) {
				uint16_t c = ref_tcp_calc_checksum(tcph, (uint16_t)(ip_len - 4 * ihl),
				                                   ld32(f + 26), ld32(f + 30));
				memcpy(tcph + 16, &c, 2);          /* tcp_out.c:330 */
			}
		}
		if (burst && (i + 1) % burst == 0) {
			double t0 = now_us();
			iom->send_pkts(ctx, ifidx);                /* core.c:846-848 */
			double t1 = now_us();
			if (send_us)
				send_us[k] = t1 - t0;
			if (burst_us)
				burst_us[k] = t1 - t_burst;
			k++;
			t_burst = now_us();
			sent = i + 1;
		}
	}
	if (sent < n)
		iom->send_pkts(ctx, ifidx);
	return (int)n;
}
