/*
 * mtcp_gpucsum.h -- C ABI of libmtcp_gpucsum.so: mTCP's software TCP/IP
 * checksum path (the --disable-hwcsum branch) as batched MI355X (gfx950)
 * HIP kernels.
 *
 * What each entry point replaces in the reference (/root/reference):
 *
 *   gcs_verify*        the per-frame RX checks of ProcessPacket / ProcessIPv4Packet /
 *                      ProcessTCPPacket: eth_in.c:35, ip_in.c:21-59 (ip_fast_csum at
 *                      :35) and tcp_in.c:1208-1241 (TCPCalcChecksum at :1231), one
 *                      verdict byte per frame instead of one call per frame.
 *   gcs_compute*       the TX folds of IPOutput / IPOutputStandalone (ip_out.c:153,172 /
 *                      :82,100) and SendTCPPacket / SendTCPPacketStandalone
 *                      (tcp_out.c:244,323-333 / :161,202-214), written in place.
 *   gcs_tcp_checksum_dev  TCPCalcChecksum()   mtcp/src/tcp_util.c:244-277
 *                         (declared mtcp/src/include/tcp_util.h:41-42), element-wise.
 *   gcs_ip_checksum_dev   ip_fast_csum()      io_engine/include/ps.h:66-95, element-wise,
 *                         x86 semantics incl. the ihl<=4 early exit (:72-73).
 *   gcs_icmp_checksum_dev ICMPChecksum()      mtcp/src/icmp.c:18-42 (static there), element-wise.
 *   GCS_VF_ICMP / GCS_CF_ICMP  the ICMP fold of ProcessICMPECHORequest (icmp.c:89) and
 *                         ICMPOutput (icmp.c:57-69) inside the batched verify / fill.
 *   gcs_classify*, gcs_rss_dev  RSS steering: GetRSSHash / GetRSSCPUCore
 *                         (mtcp/src/rss.c:44-115), fused into the RX verify.
 *   gcs_compute_copy_dev  SendTCPPacket's payload memcpy + both TX folds
 *                         (tcp_out.c:316-333, ip_out.c:172) in one pass.
 *   gcs_gro_dev           software LRO: in-order segment merge with refilled checks
 *                         (the NIC LRO of ENABLELRO builds, dpdk_module.c:855-881).
 *
 * The io_module_func plugin that sits on top of this ABI (the drop-in under
 * mtcp/src, io_module.h:60-72) is declared in gpucsum_io_module.h.
 *
 * Conventions
 *   - Plain C types only; every function returns GCS_OK (0) or a negative
 *     GCS_E* code; no C++ exceptions cross the ABI.
 *   - Byte order: frames are raw wire bytes.  Checksum values are returned
 *     exactly as the reference returns them (uint16_t as stored by a
 *     little-endian host, i.e. the value memcpy'd into iph->check).
 *   - Batch layout in device memory ("HBM batch"): frame i at byte offset
 *     off[i] of one buffer of frames_bytes bytes, length len[i].  off[i] must
 *     be a multiple of 16 (the pslib packing uses 64, io_engine/lib/pslib.c:146);
 *     a descriptor that is misaligned or reaches past frames_bytes yields
 *     GCS_V_BAD_DESC / GCS_TX_BAD_DESC for that frame and is never read.
 *   - Fixed-stride layout: frame i at i*stride (stride % 16 == 0), all of
 *     length frame_len <= stride.
 *   - *_dev functions take device pointers and are asynchronous on `stream`
 *     (a hipStream_t; NULL = the context's own stream).  Host functions are
 *     synchronous and stage through the context's pinned buffers.
 *   - Threading: a context belongs to one host thread (mTCP: one per core,
 *     core.c:1153-1245).  Different contexts may be used concurrently.
 */
#ifndef MTCP_GPUCSUM_H
#define MTCP_GPUCSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GCS_ABI_VERSION 2

/* ---- status codes ---------------------------------------------------- */
#define GCS_OK        0
#define GCS_EINVAL   (-1)   /* bad argument (NULL, n > capacity, stride < frame_len ...) */
#define GCS_ENODEV   (-2)   /* no HIP device / device index out of range           */
#define GCS_ENOMEM   (-3)   /* device or pinned host allocation failed             */
#define GCS_EHIP     (-4)   /* a HIP runtime call failed (see gcs_last_hip_error)  */
#define GCS_ERANGE   (-5)   /* batch larger than the context was created for       */

/* ---- RX verdicts: one byte per frame ------------------------------------
 * Same decision order as the reference (see csum order above).  "ERROR"
 * verdicts are the ones mTCP returns ERROR for and counts in
 * nstat.rx_errors (eth_in.c:49-53, core.c:796-799). */
#define GCS_V_ACCEPT        0  /* IP + TCP checksums pass (tcp_in.c:1243 onward)        */
#define GCS_V_NOT_IPV4      1  /* ethertype != 0x0800: ARP / release (eth_in.c:39-46)  */
#define GCS_V_DROP_IPLEN    2  /* ERROR: tot_len < 20 (ip_in.c:25-26)                   */
#define GCS_V_DROP_IPCSUM   3  /* ERROR: ip_fast_csum != 0 (ip_in.c:35-36)              */
#define GCS_V_NOT_V4        4  /* version != 4: released (ip_in.c:47-50)                */
#define GCS_V_NOT_TCP       5  /* IPv4, IP csum ok, protocol != TCP (ip_in.c:52-59)     */
#define GCS_V_DROP_TCPLEN   6  /* ERROR: ip_len < (ihl+doff)*4 (tcp_in.c:1221-1222)      */
#define GCS_V_DROP_TCPCSUM  7  /* ERROR: TCPCalcChecksum != 0 (tcp_in.c:1231-1239)      */
#define GCS_V_DROP_TRUNC    8  /* ERROR: the reference would read past the frame (UB
                                  there: tcp_in.c:1231 folds tot_len bytes regardless)  */
#define GCS_V_BAD_DESC      9  /* ERROR: descriptor misaligned / outside the buffer     */
#define GCS_V_ICMP_OK      10  /* GCS_VF_ICMP: IPv4 ICMP, ICMPChecksum == 0 (icmp.c:89)  */
#define GCS_V_ICMP_BADCSUM 11  /* GCS_VF_ICMP: ICMPChecksum != 0 -- mTCP sends no echo
                                  reply (icmp.c:89-91) but does NOT count an error
                                  (ProcessICMPPacket returns TRUE, icmp.c:140)          */
#define GCS_V_IS_ERROR(v) ((v) == 2 || (v) == 3 || ((v) >= 6 && (v) <= 9))

/* verify flags */
#define GCS_VF_ZERO_BAD_TCP_CHECK 0x1u  /* reproduce tcp_in.c:1237: tcph->check = 0 on
                                           a TCP checksum failure (writes the frame)   */
#define GCS_VF_ICMP               0x2u  /* give IPv4 ICMP frames (otherwise NOT_TCP) the
                                           verdict of ICMPChecksum over tot_len - ihl*4
                                           bytes; a message past the frame is TRUNC;
                                           tot_len < ihl*4 is BADCSUM (the reference
                                           folds nothing and gets 0xFFFF)              */
#define GCS_VF_ROOMS              0x8u  /* descriptor batches (gcs_verify_dev): a hint that
                                           the frames lie one per room (mbuf-shaped, e.g.
                                           2 KiB rooms, dpdk_module.c:44-49), not packed:
                                           each frame is verified by its own 32-lane group
                                           (k_desc rooms kernel) instead of the packed
                                           stream's per-frame fallback.  Same results;
                                           ignored with GCS_VF_ICMP                         */

/* ---- TX status: one byte per frame (optional output) ------------------- */
#define GCS_TX_OK           0  /* iph->check and tcph->check written                   */
#define GCS_TX_IP_ONLY      1  /* IPv4, not TCP: iph->check written (ip_out.c:90-92)   */
#define GCS_TX_NOT_IPV4     2  /* untouched                                            */
#define GCS_TX_BAD_HDR      3  /* ihl < 5 or IP header past the frame: untouched       */
#define GCS_TX_BAD_TCPLEN   4  /* iph->check written; tot_len < ihl*4+20 or the segment
                                  runs past the frame: TCP untouched                    */
#define GCS_TX_ICMP_OK      5  /* GCS_CF_ICMP: iph->check and icmph->checksum written   */
#define GCS_TX_BAD_ICMPLEN  6  /* GCS_CF_ICMP: iph->check written; tot_len < ihl*4+8 or
                                  the message runs past the frame: ICMP untouched       */
#define GCS_TX_BAD_DESC     9  /* descriptor misaligned / outside the buffer           */

/* compute flags */
#define GCS_CF_NO_INPLACE   0x1u  /* do not write the frames; only fill csums[]         */
#define GCS_CF_ICMP         0x2u  /* also fill the ICMP checksum of IPv4 ICMP frames, as
                                     ICMPOutput does (icmp.c:57-69: checksum = 0, then
                                     ICMPChecksum over the whole message); csums[] then
                                     holds ip | icmp << 16                             */
#define GCS_CF_SECTOR_WB    0x4u  /* fixed-stride fills: write back only the 64 B sectors
                                     holding the check fields, never whole 128 B lines
                                     (the line write-back is chosen by batch size,
                                     DESIGN.md §4 "TX write-back"; a measurement knob) */
#define GCS_CF_ROOMS        0x8u  /* gcs_compute_dev: the rooms hint of GCS_VF_ROOMS; the
                                     fill then writes back each frame's whole first 128 B
                                     line (its own bytes only) while the batch's lines fit
                                     the Infinity Cache, as fixed-stride fills do       */

typedef struct gcs_ctx gcs_ctx;

/* ---- library / context ------------------------------------------------- */
int         gcs_abi_version(void);
const char *gcs_strerror(int code);
const char *gcs_last_hip_error(void);          /* thread-local, "" if none        */
int         gcs_device_count(int *count);

/* Create a context on HIP device `device` with its own non-blocking stream.
 * max_frames / max_bytes size the staging used by the host-memory entry points
 * (0 = no staging: only the *_dev functions may be used). */
int gcs_ctx_create(gcs_ctx **out, int device, uint32_t max_frames, uint64_t max_bytes);
/* Releases everything whatever fails, and returns the first failure (a device
 * fault that surfaces while the context's work drains is reported here, to
 * its owner, not to the next caller). */
int gcs_ctx_destroy(gcs_ctx *ctx);
int gcs_ctx_device(const gcs_ctx *ctx, int *device);
int gcs_ctx_stream(const gcs_ctx *ctx, void **stream);   /* hipStream_t */
int gcs_sync(gcs_ctx *ctx);                               /* wait for ctx stream */
/* Health check of a device (tests run it after every GPU test; an mTCP
 * thread may after a failed call): every stream of the process drained with
 * no fault, twice, 1 ms apart (a fault reaches the process asynchronously);
 * with no context holding a burst-server ring, no server grid resident.
 * GCS_EHIP with gcs_last_hip_error() naming what failed. */
int gcs_device_check(int device);

/* Burst server (on = 1): host batches small enough for direct mode (the
 * kernel reads pinned staging over PCIe: an mTCP burst) are served by a
 * resident grid that polls a request ring in pinned memory, instead of one
 * kernel launch and one event wait per batch.  ONE grid per process and
 * device serves the rings of up to 32 contexts (one per mTCP thread; 8
 * blocks each), on a highest-priority stream of its own; a 33rd context gets
 * GCS_ERANGE and runs without it.  The grid leaves after GCS_SERVER_LIFE_US
 * (default 10000) in total, or when a ring's blocks have had no work for
 * GCS_SERVER_IDLE_US (default 10000); a later batch starts it again.  A ring
 * goes cold after GCS_SERVER_HOT_US (default 20; 0 = never) without a
 * request -- or, when 3 x the gap between its last two requests is within
 * GCS_SERVER_HOT_MAX_US (default 200), after that long, so a thread bursting
 * every few tens of us keeps it hot: then one block, not eight, polls it.  Default: off, or
 * the environment variable GCS_BURST_SERVER=1 at gcs_ctx_create. */
int gcs_ctx_set_burst_server(gcs_ctx *ctx, int on);

/* The burst server's figures for this context's ring since it was turned on
 * (like mTCP's per-thread NETSTAT, core.c:189-218): requests and post -> done
 * always; the GPU side only when the process ran with GCS_SERVER_COUNTERS=1 or
 * GCS_SERVER_PROF (the grid build with phase counters), else 0.  Per-block
 * figures are means over the (block, request) pairs that served frames.
 * GCS_SERVER_PROF also prints them at exit.  GCS_EINVAL without the server. */
typedef struct gcs_server_stats {
    uint64_t requests;        /* requests completed on this ring                      */
    uint64_t block_requests;  /* (block, request) pairs that served frames            */
    uint64_t polls;           /* polls by the ring's blocks                           */
    double post_to_done_us;   /* mean per request: posted -> completed (host clock)   */
    double gpu_span_us;       /* mean: first serving block saw it -> last one's
                                 records stored (GPU clock)                           */
    double poll_us;           /* one poll: issue -> data back, every poll             */
    double seen_poll_us;      /* ... the polls that saw a request                     */
    double acquire_us;        /* the acquire fence after that poll                    */
    double frames_us;         /* frame loads and folds, record stores issued          */
    double records_us;        /* the record stores acknowledged                       */
    double release_us;        /* release fence + ack (requests that wrote frames)     */
    double seen_skew_us;      /* mean per request: last serving block saw it - first  */
    double block_serve_us;    /* mean per request: the slowest block, saw it -> its
                                 records stored                                       */
    double cold_frac;         /* (block, request) pairs whose block was cold (polling
                                 the leader's copy) when the request came             */
    uint64_t slow_polls_2us;  /* polls whose round trip took over 2 us                */
    uint64_t slow_polls_5us;  /* ... over 5 us                                        */
    uint64_t torn_polls;      /* polls that saw a request's line A before all its
                                 other lines had landed                               */
    double max_poll_us;       /* the longest poll round trip                          */
    double late_us[8];        /* mean per request: how long after the first serving
                                 block each of the ring's blocks saw it (block index) */
    double seen_wait_us;      /* mean per request: how much longer than the ring's
                                 fastest request it took from the post until the first
                                 block saw it (host and GPU clocks compared)          */
    double after_gpu_us;      /* mean per request: the fastest post -> seen, plus from
                                 the last records stored until the host completed it;
                                 post_to_done = seen_wait + gpu_span + after_gpu      */
} gcs_server_stats;
int gcs_server_stats_get(gcs_ctx *ctx, gcs_server_stats *out);

/* Pinned host memory for zero-copy host batches: when every frame of a
 * gcs_verify / gcs_compute call lies in pinned memory (allocated here, or an
 * existing buffer such as an mbuf pool registered with gcs_host_register) and
 * the offsets are 16 B-aligned and increasing, the frames go to the GPU with
 * one DMA per staging slot and no host copy.  Otherwise they are gathered
 * into the context's pinned staging (environment GCS_GATHER_THREADS threads,
 * default 8, for large batches).
 * gcs_host_register: regions are process-wide, at most 64 GiB each, and may
 * not overlap (GCS_EINVAL).  gcs_host_unregister takes the pointer that was
 * registered; no batch reading the region may be in flight on any context
 * (calls are synchronous, so: none running on another thread). */
int gcs_host_alloc(void **p, uint64_t bytes);
int gcs_host_free(void *p);
int gcs_host_register(void *p, uint64_t bytes);
int gcs_host_unregister(void *p);
/* Device memory on the context's device. */
int gcs_dev_alloc(gcs_ctx *ctx, void **p, uint64_t bytes);
int gcs_dev_free(gcs_ctx *ctx, void *p);

/* ---- device-resident batches (async on stream) ------------------------ */
int gcs_verify_fixed_dev(gcs_ctx *ctx, uint8_t *d_frames, uint64_t stride,
                         uint32_t frame_len, uint32_t n, uint8_t *d_verdict,
                         uint32_t flags, void *stream);
int gcs_compute_fixed_dev(gcs_ctx *ctx, uint8_t *d_frames, uint64_t stride,
                          uint32_t frame_len, uint32_t n, uint8_t *d_status,
                          uint32_t *d_csums, uint32_t flags, void *stream);
/* One iteration of mTCP's loop over two device-resident fixed-stride batches
 * (core.c:761-877 folds RX and TX every iteration): the TX fill of d_tx (as
 * gcs_compute_fixed_dev) and the RX verify of d_rx (as gcs_verify_fixed_dev)
 * in ONE launch when both frame sizes take the same kernel shape and no
 * GCS_*_ICMP flag is set -- the verify's first blocks then run in the fill's
 * tail instead of behind a kernel boundary -- else as those two launches, in
 * that order.  The batches may not overlap (GCS_EINVAL); n_tx or n_rx may
 * be 0. */
int gcs_step_fixed_dev(gcs_ctx *ctx, uint8_t *d_tx, uint64_t tx_stride, uint32_t tx_len,
                       uint32_t n_tx, uint8_t *d_tx_status, uint32_t *d_tx_csums,
                       uint32_t tx_flags, uint8_t *d_rx, uint64_t rx_stride, uint32_t rx_len,
                       uint32_t n_rx, uint8_t *d_rx_verdict, uint32_t rx_flags, void *stream);
int gcs_verify_dev(gcs_ctx *ctx, uint8_t *d_frames, uint64_t frames_bytes,
                   const uint64_t *d_off, const uint16_t *d_len, uint32_t n,
                   uint8_t *d_verdict, uint32_t flags, void *stream);
int gcs_compute_dev(gcs_ctx *ctx, uint8_t *d_frames, uint64_t frames_bytes,
                    const uint64_t *d_off, const uint16_t *d_len, uint32_t n,
                    uint8_t *d_status, uint32_t *d_csums, uint32_t flags,
                    void *stream);

/* Element-wise reference functions.  Item i: buf + off[i] (off[i] even, the
 * reference takes a uint16_t*), the bytes it reads must lie inside
 * buf_bytes (else out[i] = 0 and the item is skipped).
 *   tcp: out[i] = TCPCalcChecksum(buf+off[i], len[i], saddr[i], daddr[i])
 *   ip : out[i] = ip_fast_csum(buf+off[i], ihl[i] & 15)                  */
int gcs_tcp_checksum_dev(gcs_ctx *ctx, const uint8_t *d_buf, uint64_t buf_bytes,
                         const uint64_t *d_off, const uint16_t *d_len,
                         const uint32_t *d_saddr, const uint32_t *d_daddr,
                         uint32_t n, uint16_t *d_out, void *stream);
int gcs_ip_checksum_dev(gcs_ctx *ctx, const uint8_t *d_buf, uint64_t buf_bytes,
                        const uint64_t *d_off, const uint8_t *d_ihl, uint32_t n,
                        uint16_t *d_out, void *stream);
/*   icmp: out[i] = ICMPChecksum(buf+off[i], len[i]).  An odd final byte is the
 *   low byte of a word with a zero high byte: the C leaves that high byte
 *   uninitialised (icmp.c:24,33-34) and the reference's gcc -O3 object
 *   zero-extends it (movzbl).                                            */
int gcs_icmp_checksum_dev(gcs_ctx *ctx, const uint8_t *d_buf, uint64_t buf_bytes,
                          const uint64_t *d_off, const uint16_t *d_len, uint32_t n,
                          uint16_t *d_out, void *stream);

/* ---- TX payload copy + fill (SendTCPPacket, tcp_out.c:316-333) ----------
 * mTCP writes the headers of a data segment, memcpy's the payload behind them
 * and then folds header + payload (and the IP header).  gcs_compute_copy_dev
 * does the copy and both folds in one pass over device memory: frame i (at
 * d_off[i], d_len[i] bytes, headers already written) receives its TCP payload
 * -- tot_len + 14 - hl bytes, hl = 14 + ihl*4 + doff*4 -- from d_src +
 * d_src_off[i] (any alignment), and its checks are filled as gcs_compute_dev
 * fills them.  Only frames whose headers describe a complete TCP segment (the
 * GCS_TX_OK conditions) are copied; the others get the plain fill.  A source
 * range outside [0, src_bytes) gives GCS_TX_BAD_DESC and leaves the frame
 * untouched.  flags: 0 (the copy is in place by definition). */
int gcs_compute_copy_dev(gcs_ctx *ctx, uint8_t *d_frames, uint64_t frames_bytes,
                         const uint64_t *d_off, const uint16_t *d_len,
                         const uint8_t *d_src, uint64_t src_bytes,
                         const uint64_t *d_src_off, uint32_t n, uint8_t *d_status,
                         uint32_t *d_csums, uint32_t flags, void *stream);

/* ---- software LRO: receive-side segment merge ----------------------------
 * What a NIC's LRO does for mTCP's ENABLELRO builds (dpdk_module.c:44-48,
 * 855-881; tcp_ring_buffer.c:15-21), on the GPU, after the RX verify.  Over
 * windows of `window` (1..256) consecutive descriptors, runs of in-order
 * ACCEPT segments of one flow become one frame: the head's headers with
 * tot_len updated and PSH if any member had it, the payloads in order, IP and
 * TCP checks refilled -- a frame mTCP's own RX checks accept.  The merge rules
 * (Linux GRO's) are listed in oracle/csum_ref.h (ref_gro_batch); a run never
 * exceeds max_len bytes (<= 65535; mTCP's LRO buffers are 16384, dpdk_module.c:45).
 * d_verdict: the frames' GCS_V_* verdicts (gcs_verify_dev / gcs_classify_dev).
 * Output frames of a window are packed from the window's first input offset,
 * 16 B-aligned, into d_out (out_bytes; nothing past it is written): inputs must
 * be packed in increasing offset order, and out_bytes >= in_bytes keeps every
 * frame whole.  Per input frame i: d_head[i] = index of its run's head;
 * d_out_off[i] = the run's output offset; d_out_len[i] = the run's length for
 * a head, 0 for a merged member (and for a bad descriptor). */
int gcs_gro_dev(gcs_ctx *ctx, const uint8_t *d_in, uint64_t in_bytes,
                const uint64_t *d_off, const uint16_t *d_len, const uint8_t *d_verdict,
                uint32_t n, uint32_t window, uint32_t max_len, uint8_t *d_out,
                uint64_t out_bytes, uint64_t *d_out_off, uint16_t *d_out_len,
                uint32_t *d_head, void *stream);

/* ---- RSS steering (rss.c) ----------------------------------------------
 * gcs_ctx_set_rss: the Toeplitz key (key_len >= 16; only the first 16 bytes
 * reach the 96 windows GetRSSHash uses, rss.c:27-40; NULL = the reference's
 * built-in key of 40 x 0x05, rss.c:19-25), the number of RX queues / mTCP
 * cores, and GetRSSCPUCore's endian_check (non-zero: the i40e mapping, 9
 * hash bits + {3,1,-1,-3}[h & 3]; zero: ixgbe / mlx, 7 bits), rss.c:97-115.
 * Until it is called the context uses NULL key, 1 queue, endian_check 0.
 *
 * gcs_classify_*: gcs_verify_* plus, for every ACCEPT frame, the Toeplitz
 * hash of (saddr, daddr, source, dest) taken as host-order integers -- the
 * argument order addr_pool.c:168,251 uses for an incoming packet -- and the
 * queue GetRSSCPUCore maps it to: the mTCP core that owns the flow.  Other
 * verdicts get hash 0 and queue 0xFFFF.  d_hash / d_queue may be NULL.
 *
 * gcs_rss_dev: element-wise GetRSSHash / GetRSSCPUCore over host-order
 * tuples (d_hash or d_queue may be NULL). */
int gcs_ctx_set_rss(gcs_ctx *ctx, const uint8_t *key, uint32_t key_len,
                    uint32_t num_queues, int endian_check);
int gcs_classify_fixed_dev(gcs_ctx *ctx, uint8_t *d_frames, uint64_t stride,
                           uint32_t frame_len, uint32_t n, uint8_t *d_verdict,
                           uint32_t *d_hash, uint16_t *d_queue, uint32_t flags,
                           void *stream);
int gcs_classify_dev(gcs_ctx *ctx, uint8_t *d_frames, uint64_t frames_bytes,
                     const uint64_t *d_off, const uint16_t *d_len, uint32_t n,
                     uint8_t *d_verdict, uint32_t *d_hash, uint16_t *d_queue,
                     uint32_t flags, void *stream);
int gcs_rss_dev(gcs_ctx *ctx, const uint32_t *d_sip, const uint32_t *d_dip,
                const uint16_t *d_sp, const uint16_t *d_dp, uint32_t n,
                uint32_t *d_hash, uint16_t *d_queue, void *stream);

/* ---- host-memory batches (synchronous) --------------------------------
 * frames[off[i] .. off[i]+len[i]) in host memory (any alignment).  The
 * context gathers them into pinned staging at 64 B-aligned slots, copies to
 * HBM, runs the kernel and copies back only verdicts (RX) or the 4 bytes of
 * check fields per frame (TX, scattered back into `frames` on the host). */
int gcs_verify(gcs_ctx *ctx, uint8_t *frames, const uint64_t *off,
               const uint16_t *len, uint32_t n, uint8_t *verdict, uint32_t flags);
int gcs_compute(gcs_ctx *ctx, uint8_t *frames, const uint64_t *off,
                const uint16_t *len, uint32_t n, uint8_t *status, uint32_t *csums);

/* Pointer-vector variants (one pointer per frame, as an I/O module holds
 * them: rte_mbuf data pointers, dpdk_module.c:517-548 / 399-436). */
int gcs_verify_ptrs(gcs_ctx *ctx, uint8_t *const *pkts, const uint16_t *len,
                    uint32_t n, uint8_t *verdict, uint32_t flags);
int gcs_compute_ptrs(gcs_ctx *ctx, uint8_t *const *pkts, const uint16_t *len,
                     uint32_t n, uint8_t *status, uint32_t *csums);

/* Asynchronous TX fill of a host burst (the plugin fills frames as mTCP
 * completes them, tcp_out.c:239-333, instead of all at send_pkts).  With the
 * context's burst server on, the frames are posted to the resident grid and
 * the call returns at once with *ticket != 0; gcs_wait(ctx, *ticket) then
 * completes it: status[] / csums[] written (either may be NULL) and every
 * frame's check fields filled in place.  Until then the frames and the output
 * arrays must stay valid and the frames unmodified.  Frames all in one
 * registered region (gcs_host_register) at 16 B-aligned addresses are read
 * where they are; others are copied into the context's async staging: device
 * memory written over the BAR (default), or pinned host memory
 * (GCS_ASYNC_STAGE=host, or when the device allocation fails).  The checks come
 * back with the results; gcs_wait writes them into the frames.  Without the server, or for a batch larger than one request
 * (512 frames / 256 KiB staged), the fill runs synchronously and *ticket = 0.
 * gcs_wait(ctx, t) completes every async fill posted on ctx up to ticket t;
 * gcs_wait(ctx, 0) does nothing. */
int gcs_compute_ptrs_async(gcs_ctx *ctx, uint8_t *const *pkts, const uint16_t *len,
                           uint32_t n, uint8_t *status, uint32_t *csums, uint64_t *ticket);
/* Asynchronous RX verify of a host burst (the plugin verifies a burst in
 * groups as recv_pkts returns, and mTCP's get_rptr(i) waits only for the group
 * holding frame i, core.c:789-795).  As gcs_compute_ptrs_async: posted to the
 * burst server when it is on (*ticket != 0), verdict[] written -- and, with
 * GCS_VF_ZERO_BAD_TCP_CHECK, tcph->check zeroed in bad frames (tcp_in.c:1237)
 * -- by the gcs_wait that completes it; frames and verdict[] must stay valid
 * and the frames unmodified until then.  Flags other than
 * GCS_VF_ZERO_BAD_TCP_CHECK, no server, or more than one request's frames:
 * verified synchronously, *ticket = 0.  Async fills and verifies share the
 * context's request ring and complete in posting order.
 * A gcs_wait that fails (no answer from the GPU) cancels every pending async
 * request: their outputs and frames are never written.  That failure is the
 * report for the cancelled requests of the kind (fill or verify) of the
 * ticket it waited for, up to that ticket; every other cancelled request (a
 * later one of that kind, or one of the other kind) is reported once, by the
 * first later gcs_wait for a ticket of its kind that covers it -- its own
 * ticket included (GCS_EHIP).  Requests posted after the failure are never
 * reported for it. */
int gcs_verify_ptrs_async(gcs_ctx *ctx, uint8_t *const *pkts, const uint16_t *len,
                          uint32_t n, uint8_t *verdict, uint32_t flags, uint64_t *ticket);
int gcs_wait(gcs_ctx *ctx, uint64_t ticket);

/* Host-memory RX verify + RSS steering (see gcs_classify_dev); hash or queue
 * may be NULL, not both.  The host entry points take GCS_VF_ICMP as well. */
int gcs_classify(gcs_ctx *ctx, uint8_t *frames, const uint64_t *off,
                 const uint16_t *len, uint32_t n, uint8_t *verdict, uint32_t *hash,
                 uint16_t *queue, uint32_t flags);
int gcs_classify_ptrs(gcs_ctx *ctx, uint8_t *const *pkts, const uint16_t *len,
                      uint32_t n, uint8_t *verdict, uint32_t *hash, uint16_t *queue,
                      uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif /* MTCP_GPUCSUM_H */
