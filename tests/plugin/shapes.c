/*
 * shapes.c -- synthetic inner I/O modules with the buffer contracts of mTCP's
 * other backends (TEST ONLY).  Each one moves frames between a wire queue the
 * test loads and a capture of transmitted frames the test reads back.
 *
 *   nmshape   netmap (netmap_module.c:102-210): RX ring slots; TX through ONE
 *             send buffer per port -- get_wptr transmits the previous frame
 *             first (:155-156) and hands out the same buffer again (:160);
 *             dev_ioctl NULL (:268).
 *   psshape   PSIO (psio_module.c:145-289, io_engine/lib/pslib.c:132-156): RX
 *             as one chunk, a contiguous buffer + {offset, len} per packet at
 *             64 B-aligned offsets; TX through a chunk ring whose get_wptr
 *             assigns the next 64 B-aligned offset; send_pkts may send only
 *             part of the chunk (ps_send_chunk_buf), the rest stays queued;
 *             dev_ioctl NULL (:399).
 *   dfshape   DPDK with a working IP_DEFRAG (dpdk_module.c:474-513, 527-529):
 *             get_rptr feeds a fragment to the reassembly table on EVERY call;
 *             a fragment that does not complete its datagram gives NULL, the
 *             completing one the reassembled datagram (contiguous here), and a
 *             fragment fed twice starts a new table entry (NULL).  The
 *             reference dereferences the NULL of an absorbed fragment at
 *             dpdk_module.c:530 (*len = m->pkt_len); this shape returns it, as
 *             a fixed module would.
 *   lroshape  DPDK built with ENABLELRO (dpdk_module.c:399-548, 805-928): RX
 *             mbufs, some of them chains (NIC LRO), *len = pkt_len of the
 *             chain; get_rptr records cur_rx_m (:543-545) and returns NULL for
 *             a frame the NIC flagged bad (:536-542); dev_ioctl answers 0 for
 *             the RX checksum commands (NIC offload), -1 for TX, and gathers
 *             cur_rx_m's payload for PKT_RX_TCP_LROSEG (:855-881).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gpucsum_io_module.h"

#define ROOM 2048
#define CAP_MAX 65536

/* transmitted frames, in wire order */
static struct {
	uint8_t *buf;           /* CAP_MAX * ROOM */
	uint16_t len[CAP_MAX];
	uint32_t n;
} W;

static int wire_reset(void)
{
	free(W.buf);
	memset(&W, 0, sizeof(W));
	W.buf = calloc(CAP_MAX, ROOM);
	return W.buf ? 0 : -1;
}

static void wire_put(const uint8_t *p, uint32_t len)
{
	if (W.n >= CAP_MAX || len > ROOM)
		return;
	memcpy(W.buf + (uint64_t)W.n * ROOM, p, len);
	W.len[W.n++] = (uint16_t)len;
}

uint32_t shape_wire_count(void) { return W.n; }

int shape_wire_frame(uint32_t k, uint8_t *out)
{
	if (k >= W.n)
		return -1;
	memcpy(out, W.buf + (uint64_t)k * ROOM, W.len[k]);
	return W.len[k];
}

/* RX wire queue shared by the shapes: frame i = buf + off[i], len[i] */
static struct {
	uint8_t *bufs;          /* n * ROOM (chains: first segment only for lroshape) */
	uint16_t *len;
	uint32_t n, next, burst, cur_first, cur_n;
} R;

static int rx_load(const uint8_t *buf, const uint64_t *off, const uint16_t *len, uint32_t n,
                   uint32_t burst)
{
	uint32_t i;

	free(R.bufs);
	free(R.len);
	memset(&R, 0, sizeof(R));
	R.bufs = calloc(n ? n : 1, ROOM);
	R.len = calloc(n ? n : 1, sizeof(uint16_t));
	if (!R.bufs || !R.len)
		return -1;
	for (i = 0; i < n; i++) {
		uint16_t l = len[i] > ROOM ? ROOM : len[i];
		memcpy(R.bufs + (uint64_t)i * ROOM, buf + off[i], l);
		R.len[i] = l;
	}
	R.n = n;
	R.burst = burst ? burst : 64;
	return 0;
}

static int32_t rx_next_burst(void)
{
	uint32_t left = R.n - R.next;

	R.cur_first = R.next;
	R.cur_n = left < R.burst ? left : R.burst;
	R.next += R.cur_n;
	return (int32_t)R.cur_n;
}

static void nop_load(void) {}
static void nop_init(struct mtcp_thread_context *c) { (void)c; }
static int32_t nop_link(struct mtcp_thread_context *c) { (void)c; return 0; }
static void nop_release(struct mtcp_thread_context *c, int i, unsigned char *p, int l)
{
	(void)c; (void)i; (void)p; (void)l;
}
static int32_t nop_select(struct mtcp_thread_context *c) { (void)c; return 0; }
static void nop_destroy(struct mtcp_thread_context *c) { (void)c; }

/* ---- netmap shape ------------------------------------------------------ */

static struct {
	uint8_t snd_pktbuf[GPUCSUM_MAX_IFS][ROOM];
	uint32_t snd_pkt_size[GPUCSUM_MAX_IFS];
	uint32_t wptr_calls;
} NM;

int nmshape_reset(const uint8_t *buf, const uint64_t *off, const uint16_t *len, uint32_t n,
                  uint32_t burst)
{
	memset(&NM, 0, sizeof(NM));
	return wire_reset() || rx_load(buf, off, len, n, burst);
}

static int32_t nm_send(struct mtcp_thread_context *c, int nif)
{
	(void)c;
	if (NM.snd_pkt_size[nif] == 0)
		return 0;
	wire_put(NM.snd_pktbuf[nif], NM.snd_pkt_size[nif]);
	NM.snd_pkt_size[nif] = 0;
	return 1;
}

static uint8_t *nm_get_wptr(struct mtcp_thread_context *c, int nif, uint16_t pktsize)
{
	NM.wptr_calls++;
	if (NM.snd_pkt_size[nif] != 0)
		nm_send(c, nif);                        /* netmap_module.c:155-156 */
	NM.snd_pkt_size[nif] = pktsize;
	memset(NM.snd_pktbuf[nif], 0, ROOM);
	return NM.snd_pktbuf[nif];
}

static int32_t nm_recv(struct mtcp_thread_context *c, int ifidx)
{
	(void)c; (void)ifidx;
	return rx_next_burst();
}

static uint8_t *nm_get_rptr(struct mtcp_thread_context *c, int ifidx, int index, uint16_t *len)
{
	uint32_t i = R.cur_first + (uint32_t)index;
	(void)c; (void)ifidx;
	*len = R.len[i];
	return R.bufs + (uint64_t)i * ROOM;
}

io_module_func nmshape_module_func = {
	.load_module = nop_load, .init_handle = nop_init, .link_devices = nop_link,
	.release_pkt = nop_release, .get_wptr = nm_get_wptr, .send_pkts = nm_send,
	.get_rptr = nm_get_rptr, .recv_pkts = nm_recv, .select = nop_select,
	.destroy_handle = nop_destroy, .dev_ioctl = NULL,
};

/* ---- PSIO shape -------------------------------------------------------- */

#define PS_ENTRY_CNT 256        /* ENTRY_CNT is 4096 (ps.h:175): smaller, to wrap */

static struct {
	/* RX chunk */
	uint8_t *chunk;         /* PS_CHUNK_SIZE frames, 64 B-aligned */
	uint32_t info_off[64];
	uint16_t info_len[64];
	/* TX chunk ring (ps_chunk_buf) */
	uint8_t *wbuf;          /* PS_ENTRY_CNT * ROOM */
	uint32_t w_off[PS_ENTRY_CNT];
	uint16_t w_len[PS_ENTRY_CNT];
	uint32_t cnt, next_to_use, next_to_send, next_offset;
	uint32_t send_limit;    /* frames one ps_send_chunk_buf moves */
	uint32_t partial_sends;
} PS;

int psshape_reset(const uint8_t *buf, const uint64_t *off, const uint16_t *len, uint32_t n,
                  uint32_t burst, uint32_t send_limit)
{
	free(PS.chunk);
	free(PS.wbuf);
	memset(&PS, 0, sizeof(PS));
	PS.chunk = calloc(64, ROOM);
	PS.wbuf = calloc(PS_ENTRY_CNT, ROOM);
	PS.send_limit = send_limit ? send_limit : PS_ENTRY_CNT;
	if (!PS.chunk || !PS.wbuf)
		return -1;
	return wire_reset() || rx_load(buf, off, len, n, burst > 64 ? 64 : burst);
}

uint32_t psshape_pending(void) { return PS.cnt; }
uint32_t psshape_partial_sends(void) { return PS.partial_sends; }

/* ps_assign_chunk_buf, pslib.c:132-156 */
static uint8_t *ps_get_wptr(struct mtcp_thread_context *c, int nif, uint16_t len)
{
	uint32_t w;
	(void)c; (void)nif;
	if (PS.cnt >= PS_ENTRY_CNT)
		return NULL;
	w = PS.next_to_use;
	PS.cnt++;
	PS.w_len[w] = len;
	PS.w_off[w] = PS.next_offset;
	PS.next_offset += (len + 63u) / 64u * 64u;
	PS.next_to_use = (w + 1) % PS_ENTRY_CNT;
	if (PS.next_to_use == 0)
		PS.next_offset = 0;
	memset(PS.wbuf + PS.w_off[w], 0, len);
	return PS.wbuf + PS.w_off[w];
}

/* psio_flush_pkts + ps_send_chunk_buf: sends at most send_limit frames */
static int ps_flush(void)
{
	uint32_t k, m = PS.cnt < PS.send_limit ? PS.cnt : PS.send_limit;

	for (k = 0; k < m; k++) {
		wire_put(PS.wbuf + PS.w_off[PS.next_to_send], PS.w_len[PS.next_to_send]);
		PS.next_to_send = (PS.next_to_send + 1) % PS_ENTRY_CNT;
	}
	PS.cnt -= m;
	return (int)m;
}

/* psio_send_pkts, psio_module.c:197-232 */
static int32_t ps_send(struct mtcp_thread_context *c, int nif)
{
	uint32_t prev;
	int ret;
	(void)c; (void)nif;
	while ((prev = PS.cnt) > 0) {
		ret = ps_flush();
		if (ret <= 0)
			break;
		if ((uint32_t)ret < prev) {
			PS.partial_sends++;
			break;
		}
	}
	return 0;
}

/* psio_recv_pkts: one chunk of up to PS_CHUNK_SIZE packets, packed */
static int32_t ps_recv(struct mtcp_thread_context *c, int ifidx)
{
	int32_t n = rx_next_burst(), i;
	uint32_t o = 0;
	(void)c; (void)ifidx;
	for (i = 0; i < n; i++) {
		uint32_t f = R.cur_first + (uint32_t)i;
		PS.info_off[i] = o;
		PS.info_len[i] = R.len[f];
		memcpy(PS.chunk + o, R.bufs + (uint64_t)f * ROOM, R.len[f]);
		o += (R.len[f] + 63u) / 64u * 64u;
	}
	return n;
}

static uint8_t *ps_get_rptr(struct mtcp_thread_context *c, int ifidx, int index, uint16_t *len)
{
	(void)c; (void)ifidx;
	*len = PS.info_len[index];
	return PS.chunk + PS.info_off[index];
}

io_module_func psshape_module_func = {
	.load_module = nop_load, .init_handle = nop_init, .link_devices = nop_link,
	.release_pkt = nop_release, .get_wptr = ps_get_wptr, .send_pkts = ps_send,
	.get_rptr = ps_get_rptr, .recv_pkts = ps_recv, .select = nop_select,
	.destroy_handle = nop_destroy, .dev_ioctl = NULL,
};

/* ---- DPDK + IP_DEFRAG shape -------------------------------------------- */

static struct {
	uint8_t *frag;          /* per wire frame: 0 plain, 1 absorbed, 2 completes a datagram */
	uint8_t *whole;         /* per wire frame: its reassembled datagram (frag 2), ROOM each */
	uint16_t *whole_len;
	uint8_t *fed;           /* the fragment went to the table already */
	uint32_t refeeds;
} DF;

int dfshape_reset(const uint8_t *buf, const uint64_t *off, const uint16_t *len, uint32_t n,
                  uint32_t burst, const uint8_t *frag, const uint8_t *wbuf,
                  const uint64_t *woff, const uint16_t *wlen)
{
	uint32_t i;

	free(DF.frag);
	free(DF.whole);
	free(DF.whole_len);
	free(DF.fed);
	memset(&DF, 0, sizeof(DF));
	DF.frag = calloc(n ? n : 1, 1);
	DF.whole = calloc(n ? n : 1, ROOM);
	DF.whole_len = calloc(n ? n : 1, sizeof(uint16_t));
	DF.fed = calloc(n ? n : 1, 1);
	if (!DF.frag || !DF.whole || !DF.whole_len || !DF.fed)
		return -1;
	for (i = 0; i < n; i++) {
		DF.frag[i] = frag[i];
		if (frag[i] == 2) {
			if (wlen[i] > ROOM)
				return -1;
			memcpy(DF.whole + (uint64_t)i * ROOM, wbuf + woff[i], wlen[i]);
			DF.whole_len[i] = wlen[i];
		}
	}
	return wire_reset() || rx_load(buf, off, len, n, burst);
}

uint32_t dfshape_refeeds(void) { return DF.refeeds; }

static uint8_t *df_get_rptr(struct mtcp_thread_context *c, int ifidx, int index, uint16_t *len)
{
	uint32_t i = R.cur_first + (uint32_t)index;
	(void)c; (void)ifidx;
	if (DF.frag[i] == 0) {
		*len = R.len[i];
		return R.bufs + (uint64_t)i * ROOM;
	}
	if (DF.fed[i]) {                        /* fed again: a fresh, incomplete entry */
		DF.refeeds++;
		*len = 0;
		return NULL;
	}
	DF.fed[i] = 1;
	if (DF.frag[i] == 1) {
		*len = 0;
		return NULL;
	}
	*len = DF.whole_len[i];
	return DF.whole + (uint64_t)i * ROOM;
}

/* RX only: the tests drive no TX through it (the netmap shape's TX is reused) */
io_module_func dfshape_module_func = {
	.load_module = nop_load, .init_handle = nop_init, .link_devices = nop_link,
	.release_pkt = nop_release, .get_wptr = nm_get_wptr, .send_pkts = nm_send,
	.get_rptr = df_get_rptr, .recv_pkts = nm_recv, .select = nop_select,
	.destroy_handle = nop_destroy, .dev_ioctl = NULL,
};

/* ---- DPDK + ENABLELRO shape -------------------------------------------- */

#define LRO_SEG_MAX 8

struct mbuf {
	uint8_t *seg[LRO_SEG_MAX];
	uint16_t data_len[LRO_SEG_MAX];
	uint32_t nseg, pkt_len;
	int bad;                /* NIC flagged a bad checksum (ol_flags) */
};

static struct {
	struct mbuf *m;         /* the RX wire */
	uint8_t *segbufs;       /* n * LRO_SEG_MAX * ROOM */
	uint32_t n, next, burst, cur_first, cur_n;
	struct mbuf *cur_rx_m;
	uint32_t rptr_calls, gathers;
	/* TX: DPDK wmbufs, one table of MAX_PKT_BURST per port */
	uint8_t tx[64][ROOM];
	uint16_t tx_len[64];
	uint32_t tx_n;
} LR;

/* Frame i (full logical frame at buf + off[i], len[i] bytes) arrives as
 * nseg[i] segments: the first holds first_len[i] bytes (headers + payload
 * start), the rest split the remainder evenly (dpdk_module.c:855-881 walks
 * m->next).  bad[i]: the NIC's checksum flag. */
int lroshape_reset(const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                   const uint8_t *nseg, const uint16_t *first_len, const uint8_t *bad,
                   uint32_t n, uint32_t burst)
{
	uint32_t i, s;

	free(LR.m);
	free(LR.segbufs);
	memset(&LR, 0, sizeof(LR));
	LR.m = calloc(n ? n : 1, sizeof(struct mbuf));
	LR.segbufs = calloc((size_t)(n ? n : 1) * LRO_SEG_MAX, ROOM);
	if (!LR.m || !LR.segbufs)
		return -1;
	for (i = 0; i < n; i++) {
		struct mbuf *m = &LR.m[i];
		const uint8_t *src = buf + off[i];
		uint32_t ns = nseg[i] ? nseg[i] : 1, rest, o;
		if (ns > LRO_SEG_MAX)
			return -1;
		m->nseg = ns;
		m->pkt_len = len[i];
		m->bad = bad[i];
		for (s = 0; s < ns; s++)
			m->seg[s] = LR.segbufs + ((uint64_t)i * LRO_SEG_MAX + s) * ROOM;
		m->data_len[0] = ns == 1 ? (uint16_t)len[i] : first_len[i];
		rest = len[i] - m->data_len[0];
		for (s = 1; s < ns; s++)
			m->data_len[s] = (uint16_t)(rest / (ns - 1) + (s <= rest % (ns - 1) ? 1 : 0));
		for (s = 0, o = 0; s < ns; s++) {
			if (m->data_len[s] > ROOM)
				return -1;
			memcpy(m->seg[s], src + o, m->data_len[s]);
			o += m->data_len[s];
		}
	}
	LR.n = n;
	LR.burst = burst ? burst : 64;
	return wire_reset();
}

uint32_t lroshape_gathers(void) { return LR.gathers; }

static int32_t lr_recv(struct mtcp_thread_context *c, int ifidx)
{
	uint32_t left = LR.n - LR.next;
	(void)c; (void)ifidx;
	LR.cur_first = LR.next;
	LR.cur_n = left < LR.burst ? left : LR.burst;
	LR.next += LR.cur_n;
	LR.cur_rx_m = NULL;
	return (int32_t)LR.cur_n;
}

/* dpdk_get_rptr, dpdk_module.c:517-548 */
static uint8_t *lr_get_rptr(struct mtcp_thread_context *c, int ifidx, int index, uint16_t *len)
{
	struct mbuf *m = &LR.m[LR.cur_first + (uint32_t)index];
	(void)c; (void)ifidx;
	LR.rptr_calls++;
	*len = (uint16_t)m->pkt_len;
	LR.cur_rx_m = m;                             /* :543-545 */
	return m->bad ? NULL : m->seg[0];
}

static uint8_t *lr_get_wptr(struct mtcp_thread_context *c, int nif, uint16_t pktsize)
{
	(void)c; (void)nif;
	if (LR.tx_n == 64 || pktsize > ROOM)
		return NULL;
	LR.tx_len[LR.tx_n] = pktsize;
	memset(LR.tx[LR.tx_n], 0, ROOM);
	return LR.tx[LR.tx_n++];
}

static int32_t lr_send(struct mtcp_thread_context *c, int nif)
{
	uint32_t k, n = LR.tx_n;
	(void)c; (void)nif;
	for (k = 0; k < n; k++)
		wire_put(LR.tx[k], LR.tx_len[k]);
	LR.tx_n = 0;
	return (int32_t)n;
}

/* dpdk_dev_ioctl, dpdk_module.c:805-928, for a NIC with RX checksum offload
 * and LRO but no TX offload */
static int32_t lr_ioctl(struct mtcp_thread_context *c, int nif, int cmd, void *argp)
{
	struct mbuf *m;
	const uint8_t *iph, *tcph;
	uint8_t *to;
	uint32_t seg_off, s;
	(void)c; (void)nif;

	switch (cmd) {
	case PKT_RX_IP_CSUM:
	case PKT_RX_TCP_CSUM:
		return 0;
	case PKT_RX_TCP_LROSEG:
		m = LR.cur_rx_m;
		if (!m)
			return -1;
		LR.gathers++;
		iph = m->seg[0] + 14;
		tcph = iph + ((iph[0] & 15u) << 2);
		seg_off = m->data_len[0] - 14 - ((iph[0] & 15u) << 2) - ((tcph[12] >> 4) << 2);
		to = argp;
		memcpy(to, tcph + ((tcph[12] >> 4) << 2), seg_off);
		for (s = 1; s < m->nseg; s++) {
			memcpy(to + seg_off, m->seg[s], m->data_len[s]);
			seg_off += m->data_len[s];
		}
		return 0;
	default:
		return -1;
	}
}

io_module_func lroshape_module_func = {
	.load_module = nop_load, .init_handle = nop_init, .link_devices = nop_link,
	.release_pkt = nop_release, .get_wptr = lr_get_wptr, .send_pkts = lr_send,
	.get_rptr = lr_get_rptr, .recv_pkts = lr_recv, .select = nop_select,
	.destroy_handle = nop_destroy, .dev_ioctl = lr_ioctl,
};
