/*
 * gpucsum_io_module.h -- mTCP I/O-module plugin that moves the software
 * checksum path onto MI355X (exported by libmtcp_gpucsum.so).
 *
 * The plugin surface is mTCP's own (/root/reference/mtcp/src/include/io_module.h):
 *   - struct io_module_func, 11 function pointers     io_module.h:60-72
 *   - dev_ioctl command codes PKT_*_CSUM               io_module.h:84-91
 *   - module selection by `io = <name>`               config.c:635-640, io_module.h:114-125
 * It is restated below (same field order, types and alignment -- that is the
 * ABI) only when io_module.h itself has not been included, so mTCP sources
 * can include both headers.
 *
 * gpucsum_module_func is a DECORATOR around an inner NIC module (dpdk, onvm,
 * psio, netmap, or any io_module_func):
 *   recv_pkts   inner recv_pkts, then one batched RX verify of the burst on the
 *               GPU (replaces ip_in.c:28-37 + tcp_in.c:1224-1241 per frame)
 *   get_rptr    NULL for frames whose verdict mTCP would count as an ERROR --
 *               exactly how dpdk_get_rptr surfaces bad HW checksums
 *               (dpdk_module.c:536-542); core.c:794-799 counts rx_errors.
 *               For every other frame the inner get_rptr is called again with
 *               the same index, so per-index inner state follows mTCP's walk
 *               (DPDK's cur_rx_m, dpdk_module.c:543-545, which the ENABLELRO
 *               gather PKT_RX_TCP_LROSEG reads, :856-857)
 *   get_wptr    inner get_wptr; the buffer is queued for the TX fill
 *               (GPUCSUM_INNER_TX_EAGER inners: a shadow buffer, see below)
 *   send_pkts   one batched TX fill of the queued frames on the GPU (replaces
 *               ip_out.c:155-173 + tcp_out.c:323-333), then inner send_pkts
 *   dev_ioctl   0 ("done by the device") for PKT_TX_IP_CSUM, PKT_TX_TCPIP_CSUM,
 *               PKT_RX_IP_CSUM, PKT_RX_TCP_CSUM, PKT_TX_TCPIP_CSUM_PEEK; -1
 *               (software) for PKT_TX_TCP_CSUM; anything else is forwarded to
 *               the inner module (DRV_NAME, PKT_RX_TCP_LROSEG)
 *   others      forwarded unchanged
 * Build mTCP WITHOUT -DDISABLE_HWCSUM so that ip_in.c / ip_out.c / tcp_in.c /
 * tcp_out.c consult dev_ioctl (configure.ac:119-125, Makefile.in:63-65).
 *
 * Inner-module shapes (gpucsum_set_inner_caps):
 *   in place (default: dpdk, onvm, psio)  a get_wptr buffer stays put until the
 *               inner send_pkts (dpdk_module.c:399-436, onvm_module.c:276-309,
 *               pslib.c:132-156), so frames are filled where mTCP wrote them.
 *   GPUCSUM_INNER_TX_EAGER (netmap)  the inner get_wptr transmits the previous
 *               frame and hands out ONE reused buffer (netmap_module.c:149-160).
 *               mTCP then writes into a decorator-owned shadow slot; at flush
 *               the shadow frames are filled in one GPU batch and only then
 *               copied, in order, into inner get_wptr buffers.  set_inner
 *               selects it by itself when the inner module IS mTCP's
 *               netmap_module_func (weak reference).
 *   GPUCSUM_INNER_RX_CHAINED (ENABLELRO)  the inner may return multi-segment
 *               frames whose *len is the chain's pkt_len (dpdk_module.c:530,
 *               855-881).  Frames longer than rx_seg_max (default 1514 = one
 *               MTU frame; a longer frame is an LRO chain, the same size rule
 *               tcp_ring_buffer.c:18 applies) are not read by the GPU: they are
 *               left to the inner module's own checks, as the NIC did them.
 *               set_inner selects it by itself when the inner module IS mTCP's
 *               dpdk_module_func (weak reference): a DPDK build without
 *               ENABLELRO never delivers a frame over 1518 B (jumbo frames off,
 *               dpdk_module.c:112-135), so the rule only ever sees LRO chains.
 *   GPUCSUM_INNER_RX_ONCE (IP_DEFRAG)  the inner get_rptr is not idempotent
 *               per index: DPDK built with IP_DEFRAG feeds each fragment to its
 *               reassembly table on every call (dpdk_module.c:474-513, 527-529).
 *               The decorator then calls it exactly once per index, in
 *               recv_pkts, and serves mTCP's get_rptr from what that call
 *               returned: a reassembled datagram is verified like any frame, an
 *               absorbed fragment (NULL) is an inner drop.  Not together with
 *               RX_CHAINED: ENABLELRO's gather reads the inner's cur_rx_m, which
 *               follows the last get_rptr call (dpdk_module.c:543-545, 856).
 * Without RX_ONCE, a frame whose pointer or length changes between the
 * burst's verify and mTCP's get_rptr is dropped and counted in
 * rx_rptr_changed.
 *
 * RSS check (optional): with RSS configured (gpucsum_set_rss,
 * or GPUCSUM_RSS_QUEUES=<n> [GPUCSUM_RSS_I40E=1] in the environment) each RX
 * burst is classified instead of verified: the same verdicts plus, for every
 * ACCEPT frame, the queue GetRSSCPUCore (rss.c:97-115) assigns its flow.
 * Frames whose queue is not this thread's own are counted in rx_foreign --
 * flows that mTCP's RSS-aware address pool (addr_pool.c:168,251) would have
 * placed on another core.
 * Burst server: each thread's context serves its bursts through the
 * process's resident grid for its GPU, polling the context's request ring in
 * pinned memory (gcs_ctx_set_burst_server), unless the environment sets
 * GPUCSUM_BURST_SERVER=0 (then: one kernel launch per burst).  Up to 32
 * threads per GPU share the grid; a 33rd launches per burst.
 * GPU failures (no CPU fallback: a context that cannot reach its GPU exits at
 * init_handle as dpdk_module.c:243-247 does).  A failed call after init is
 * counted in gpu_failures and reported on stderr, and its frames are:
 *   RX          returned as NULL by get_rptr (rx_errors, rx_unverified) --
 *               unverified frames never reach ProcessPacket;
 *   TX in place (dpdk, onvm, psio)  sent by the inner send_pkts as they are:
 *               the io_module API cannot withdraw a get_wptr buffer, and
 *               mTCP left both check fields 0 (ip_out.c:153, tcp_out.c:323),
 *               which the receiver's checks reject (ip_in.c:35, tcp_in.c:1231),
 *               so TCP retransmits them (tx_unfilled_sent);
 *   TX_EAGER    (netmap shadow slots) withheld from the inner module
 *               (tx_unfilled_dropped);
 *   async fill  a failed post turns fill-as-you-go off for the context and
 *               send_pkts fills the frames synchronously; a failed wait leaves
 *               the posted frames unfilled (as above).
 * GPUCSUM_ON_GPU_FAIL=exit makes any such failure fatal instead (exit, as
 * init failures are).
 * Threading (core.c:1153-1245): load_module once on the main thread; every
 * other call from the owning mTCP thread.  Per-thread state is keyed by the
 * mtcp_thread_context pointer; mTCP thread k uses GPU k mod n_gpus (override:
 * environment variable GPUCSUM_DEVICE).
 */
#ifndef GPUCSUM_IO_MODULE_H
#define GPUCSUM_IO_MODULE_H

#include <stdint.h>
#include <limits.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef IO_MODULE_H   /* not already declared by mtcp/src/include/io_module.h */
#ifndef __WORDSIZE
#define __WORDSIZE 64
#endif
struct mtcp_thread_context;
typedef struct io_module_func {
	void      (*load_module)(void);
	void      (*init_handle)(struct mtcp_thread_context *ctx);
	int32_t   (*link_devices)(struct mtcp_thread_context *ctx);
	void      (*release_pkt)(struct mtcp_thread_context *ctx, int ifidx,
	                         unsigned char *pkt_data, int len);
	uint8_t * (*get_wptr)(struct mtcp_thread_context *ctx, int ifidx, uint16_t len);
	int32_t   (*send_pkts)(struct mtcp_thread_context *ctx, int nif);
	uint8_t * (*get_rptr)(struct mtcp_thread_context *ctx, int ifidx, int index,
	                      uint16_t *len);
	int32_t   (*recv_pkts)(struct mtcp_thread_context *ctx, int ifidx);
	int32_t   (*select)(struct mtcp_thread_context *ctx);
	void      (*destroy_handle)(struct mtcp_thread_context *ctx);
	int32_t   (*dev_ioctl)(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp);
} io_module_func __attribute__((aligned(__WORDSIZE)));

#define PKT_TX_IP_CSUM          0x01
#define PKT_TX_TCP_CSUM         0x02
#define PKT_RX_TCP_LROSEG       0x03
#define PKT_TX_TCPIP_CSUM       0x04
#define PKT_RX_IP_CSUM          0x05
#define PKT_RX_TCP_CSUM         0x06
#define PKT_TX_TCPIP_CSUM_PEEK  0x07
#define DRV_NAME                0x08
#endif /* IO_MODULE_H */

/* The decorator vtable (mTCP: `io = gpucsum` once AssignIOModule knows it). */
extern io_module_func gpucsum_module_func;

/* Set the inner module the decorator wraps.  Call before load_module().
 * Resets the inner caps: GPUCSUM_INNER_TX_EAGER if inner is netmap_module_func,
 * GPUCSUM_INNER_RX_CHAINED if it is dpdk_module_func (GPUCSUM_INNER_RX_ONCE
 * instead when the program defines dpdk_module_ip_defrag = 1, which the
 * integration patch adds to a dpdk_module.c built with IP_DEFRAG), else none. */
int gpucsum_set_inner(io_module_func *inner);
/* The inner module (NULL if none): for mTCP's module-identity checks, e.g. the
 * ENABLELRO gather test at tcp_ring_buffer.c:18. */
io_module_func *gpucsum_get_inner(void);

#define GPUCSUM_INNER_TX_EAGER   0x1u  /* get_wptr may transmit / reuse earlier buffers */
#define GPUCSUM_INNER_RX_CHAINED 0x2u  /* get_rptr may return multi-segment (LRO) frames */
#define GPUCSUM_INNER_RX_ONCE    0x4u  /* get_rptr is not idempotent (IP_DEFRAG): call it
                                          once per index; not with RX_CHAINED */
/* Shape of the inner module; call after gpucsum_set_inner, before init_handle.
 * rx_seg_max: longest single-segment frame (0 = 1514). */
int gpucsum_set_inner_caps(uint32_t caps, uint32_t rx_seg_max);
/* The caps in force (after set_inner's own choice or set_inner_caps). */
uint32_t gpucsum_get_inner_caps(void);

#define GPUCSUM_MAX_IFS    16     /* MAX_DEVICES, io_engine/include/ps.h:4 */
#define GPUCSUM_MAX_BURST  8192   /* frames per GPU batch: a larger recv_pkts burst is
                                     verified whole (in several batches); a TX queue
                                     is filled and kept when it reaches this size */

/* Per-thread counters of the calling context (0 = ok, GCS_E* otherwise). */
struct gpucsum_stats {
	uint64_t rx_frames;      /* frames seen in recv_pkts                         */
	uint64_t rx_errors;      /* frames returned as NULL by get_rptr              */
	uint64_t rx_batches;     /* GPU verify launches                              */
	uint64_t tx_frames;      /* frames filled in send_pkts                       */
	uint64_t tx_batches;     /* GPU fill launches                                */
	uint64_t gpu_failures;   /* GPU calls that failed (frames then dropped/unsent)*/
	uint64_t rx_foreign;     /* RSS on: ACCEPT frames steered to another queue    */
	int      device;         /* HIP device of this context                       */
	uint64_t rx_inner;       /* RX_CHAINED: chained frames left to the inner's checks */
	uint64_t rx_rptr_changed;/* inner get_rptr changed a frame after its verify   */
	uint64_t tx_inner_full;  /* TX_EAGER: inner get_wptr had no buffer: frame lost  */
	uint64_t tx_posts;       /* async TX fill posts (GPUCSUM_TX_GROUP)            */
	/* GPU failures (gpu_failures counts the failed calls; these the frames):  */
	uint64_t tx_unfilled_sent;    /* in-place inner: frames the inner sent with the
	                               * check fields as mTCP left them (0, ip_out.c:153,
	                               * tcp_out.c:323): the receiver's checks drop them */
	uint64_t tx_unfilled_dropped; /* TX_EAGER (shadow) inner: frames withheld       */
	uint64_t rx_unverified;       /* RX frames returned as NULL (and counted in
	                               * rx_errors) because their burst's verify failed */
	uint64_t rx_posts;            /* async RX verify posts (GPUCSUM_RX_GROUP)    */
};
int gpucsum_get_stats(struct mtcp_thread_context *ctx, struct gpucsum_stats *out);

/* Verdict of frame `index` of the last recv_pkts burst on `ifidx`
 * (GCS_V_* of mtcp_gpucsum.h), or -1. */
int gpucsum_rx_verdict(struct mtcp_thread_context *ctx, int ifidx, int index);

/* RSS steering check of this context: key (NULL = the reference's built-in
 * key, rss.c:19-25; else >= 16 bytes), num_queues (0 = off), endian_check as
 * GetRSSCPUCore takes it, and the queue this thread serves.  Environment
 * default at init_handle: GPUCSUM_RSS_QUEUES / GPUCSUM_RSS_I40E, own queue =
 * thread ordinal mod num_queues. */
int gpucsum_set_rss(struct mtcp_thread_context *ctx, const uint8_t *key, uint32_t key_len,
                    uint32_t num_queues, int endian_check, int own_queue);

/* GetRSSCPUCore queue of frame `index` of the last burst on `ifidx` (RSS on,
 * ACCEPT frames), 0xFFFF for other verdicts, or -1. */
int gpucsum_rx_queue(struct mtcp_thread_context *ctx, int ifidx, int index);

#ifdef __cplusplus
}
#endif
#endif /* GPUCSUM_IO_MODULE_H */
