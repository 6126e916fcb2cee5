/*
 * csum_ref.h -- CPU ORACLE for mTCP's software checksum path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load or call it, and only as the checker / the timed CPU baseline.  The
 * product path (mtcp_amd/, libmtcp_gpucsum.so) never links or calls it.
 *
 * This is a clean-room C restatement of the reference's algorithm (nothing
 * copied).  Each function cites the reference file:line it follows:
 *
 *   ref_tcp_calc_checksum  mtcp/src/tcp_util.c:244-277   (TCPCalcChecksum)
 *   ref_ip_fast_csum       io_engine/include/ps.h:66-95  (x86 ip_fast_csum,
 *                          including the ihl<=4 early exit at :72-73)
 *   ref_rx_verdict         mtcp/src/eth_in.c:35-47, ip_in.c:21-59,
 *                          tcp_in.c:1208-1241            (RX verify order)
 *   ref_tx_fill            mtcp/src/ip_out.c:143-173, tcp_out.c:244,323-333
 *                          (TX: check fields zero when folded, then stored)
 *   ref_tx_copy_fill       mtcp/src/tcp_out.c:316-333    (payload memcpy + fill)
 *   ref_gro_batch          software LRO merge (rules: this project's, see below)
 *   ref_icmp_checksum      mtcp/src/icmp.c:18-42         (ICMPChecksum, static)
 *   ref_rss_hash/_core     mtcp/src/rss.c:13-41,44-86,97-115 (BuildKeyCache,
 *                          GetRSSHash, GetRSSCPUCore)
 *
 * Parity is pinned: tests/golden/ holds vectors produced by the reference's
 * own compiled objects (oracle/_ref, built from /root/reference sources by
 * oracle/Makefile), and tests/test_oracle_golden.py checks this file against
 * them.  Verdict / status codes are numerically identical to the product's
 * include/mtcp_gpucsum.h (a test asserts that).
 */
#ifndef MTCP_CSUM_REF_H
#define MTCP_CSUM_REF_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* RX verdicts (same numbering as GCS_V_* in include/mtcp_gpucsum.h). */
enum {
	REF_V_ACCEPT = 0,       /* passes IP + TCP checksum: tcp_in.c:1243 onward */
	REF_V_NOT_IPV4 = 1,     /* ethertype != 0x0800 (eth_in.c:35,39-46)        */
	REF_V_DROP_IPLEN = 2,   /* tot_len < 20 (ip_in.c:25-26), ERROR            */
	REF_V_DROP_IPCSUM = 3,  /* ip_fast_csum != 0 (ip_in.c:35-36), ERROR       */
	REF_V_NOT_V4 = 4,       /* version != 4 (ip_in.c:47-50), released         */
	REF_V_NOT_TCP = 5,      /* protocol != TCP (ip_in.c:52-59): IP csum only  */
	REF_V_DROP_TCPLEN = 6,  /* ip_len < (ihl+doff)*4 (tcp_in.c:1221-1222)     */
	REF_V_DROP_TCPCSUM = 7, /* TCPCalcChecksum != 0 (tcp_in.c:1231-1239)      */
	REF_V_DROP_TRUNC = 8,   /* the reference would read past the frame (UB);
	                           defined here as a drop                          */
	REF_V_BAD_DESC = 9,     /* descriptor misuse (offset/len outside buffer)  */
	REF_V_ICMP_OK = 10,     /* REF_VF_ICMP: ICMPChecksum == 0 (icmp.c:89-90)  */
	REF_V_ICMP_BADCSUM = 11 /* REF_VF_ICMP: ICMPChecksum != 0: no echo reply
	                           (icmp.c:89-91); not an error for mTCP          */
};

/* TX fill status (same numbering as GCS_TX_*). */
enum {
	REF_TX_OK = 0,          /* IP and TCP check written                       */
	REF_TX_IP_ONLY = 1,     /* IPv4, not TCP: IP check written (ip_out.c:90)  */
	REF_TX_NOT_IPV4 = 2,    /* untouched                                      */
	REF_TX_BAD_HDR = 3,     /* ihl < 5 or header beyond frame: untouched      */
	REF_TX_BAD_TCPLEN = 4,  /* IP written; TCP segment too short / truncated  */
	REF_TX_ICMP_OK = 5,     /* REF_CF_ICMP: IP and ICMP check written         */
	REF_TX_BAD_ICMPLEN = 6, /* REF_CF_ICMP: IP written; ICMP < 8 B / truncated */
	REF_TX_BAD_DESC = 9
};

#define REF_VF_ZERO_BAD_TCP_CHECK 0x1u  /* tcp_in.c:1237 side effect */
#define REF_VF_ICMP 0x2u                /* classify ICMP frames by ICMPChecksum */
#define REF_CF_ICMP 0x2u                /* TX: also fill ICMP checks (icmp.c:67-69) */

/* TCPCalcChecksum(buf, len, saddr, daddr): buf must be readable for
 * len (+1 if odd: the reference reads the whole last halfword, tcp_util.c:262) */
uint16_t ref_tcp_calc_checksum(const uint8_t *buf, uint16_t len,
                               uint32_t saddr, uint32_t daddr);

/* ip_fast_csum(iph, ihl), x86 semantics (ps.h:66-95). */
uint16_t ref_ip_fast_csum(const uint8_t *iph, unsigned int ihl);

/* One RX frame: verdict (REF_V_*).  May write tcph->check = 0 when flags
 * has REF_VF_ZERO_BAD_TCP_CHECK and the verdict is DROP_TCPCSUM. */
int ref_rx_verdict(uint8_t *frame, uint32_t len, uint32_t flags);

/* One TX frame: fills iph->check / tcph->check in place; returns REF_TX_*.
 * If csums != NULL it receives ip | tcp << 16 of what was written.
 * ref_tx_fill_f with REF_CF_ICMP also fills the ICMP check of ICMP frames
 * (ICMPOutput, icmp.c:44-77: checksum = 0, then ICMPChecksum over the whole
 * ICMP message, tot_len - ihl*4 bytes); csums then holds ip | icmp << 16. */
int ref_tx_fill(uint8_t *frame, uint32_t len, uint32_t *csums);
int ref_tx_fill_f(uint8_t *frame, uint32_t len, uint32_t *csums, uint32_t flags);

/* TX payload copy + fill (SendTCPPacket, tcp_out.c:316-333): when the frame's
 * headers describe a complete TCP segment (IPv4, ihl >= 5, TCP, doff >= 5,
 * tot_len >= (ihl+doff)*4, 14 + tot_len <= len), its payload -- bytes
 * [hl, 14 + tot_len), hl = 14 + ihl*4 + doff*4 -- is copied from src (which
 * must hold that many bytes and not be NULL -- NULL is a source offset past
 * the source buffer -- else REF_TX_BAD_DESC and nothing is written);
 * then ref_tx_fill.  The batch takes per-frame source offsets into one
 * source buffer of src_bytes. */
int ref_tx_copy_fill(uint8_t *frame, uint32_t len, const uint8_t *src, uint64_t src_avail,
                     uint32_t *csums);
void ref_compute_copy_batch(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                            const uint16_t *len, uint32_t n, const uint8_t *src,
                            uint64_t src_bytes, const uint64_t *src_off, uint8_t *status,
                            uint32_t *csums);

/* Receive-side segment merge ("software LRO"): the job a
 * NIC's LRO does for mTCP's ENABLELRO builds (dpdk_module.c:44-48, 855-881;
 * tcp_ring_buffer.c:15-21), done on the host-independent frame batch.  The
 * reference has no software merge, so the RULES are this project's (they are
 * Linux GRO's tcp4_gro_receive conditions); what is pinned to the reference is
 * that every merged frame passes its own RX checks (refx_rx_verdict) and
 * carries exactly the concatenated payloads.
 *
 * Frames are taken in windows of `window` consecutive descriptors (a burst);
 * inside a window, frame c continues frame p = c-1 when both are ACCEPT (the
 * given verdicts), both have ihl == 5, equal tos / frag_off (no MF, offset 0)
 * / ttl / saddr / daddr, c's IP id is p's or p's + 1, equal ports / ack /
 * doff / window / TCP options, zero urgent pointers and reserved bits, p's
 * flags are exactly ACK and c's ACK or ACK|PSH, both carry payload, and
 * seq(c) == seq(p) + payload(p); and the run stays <= max_len bytes.
 * A run of one frame is copied as it is; a longer run becomes one frame: the
 * head's headers with tot_len = the merged length - 14 and PSH if any member
 * has it, the members' payloads in order, and both checks refilled.  Output
 * frames of a window are packed from that window's first input offset, each
 * at a 16 B-aligned offset (inputs must be packed in increasing order, as a
 * PSIO chunk or a staging area is).  head[i] = the run head of frame i;
 * out_off / out_len are set for heads (out_len = 0 for merged members). */
void ref_gro_batch(const uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                   const uint16_t *len, const uint8_t *verdict, uint32_t n,
                   uint32_t window, uint32_t max_len, uint8_t *out, uint64_t out_bytes,
                   uint64_t *out_off, uint16_t *out_len, uint32_t *head);

/* ICMPChecksum(buf, len): LE 16-bit words, an odd final byte added as the
 * low byte of a zero-high-byte word, two-step fold, ~.  The C leaves the high
 * byte of `odd_byte` uninitialised (icmp.c:24,33-34); gcc -O3 compiles it
 * to a zero-extending byte load (movzbl), which tests/golden pins.  len <= 0
 * sums nothing: 0xFFFF. */
uint16_t ref_icmp_checksum(const uint8_t *buf, int len);

/* RSS (rss.c).  key: >= 16 bytes (only the first 16 reach the 96 cached
 * windows, :27-40); NULL = the reference's built-in key (:19-25).  Arguments
 * are host-order integers, as addr_pool.c:168,251 pass them for an incoming
 * packet (source = remote).  ref_rss_core = GetRSSCPUCore: endian_check != 0
 * is the i40e mapping (9 LSBs + {3,1,-1,-3}[h & 3]), else ixgbe/mlx (7 LSBs),
 * then % num_queues. */
extern const uint8_t REF_RSS_DEFAULT_KEY[40];
void     ref_rss_key_cache(const uint8_t *key, uint32_t cache[96]);
uint32_t ref_rss_hash(const uint8_t *key, uint32_t sip, uint32_t dip, uint16_t sp,
                      uint16_t dp);
int      ref_rss_core(const uint8_t *key, uint32_t sip, uint32_t dip, uint16_t sp,
                      uint16_t dp, int num_queues, int endian_check);

/* RX verdict + RSS steering of ACCEPT frames: hash/queue of the frame's
 * (saddr, daddr, source, dest); 0 / 0xFFFF for any other verdict. */
void ref_classify_batch(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                        const uint16_t *len, uint32_t n, uint8_t *verdict,
                        uint32_t *hash, uint16_t *queue, uint32_t flags,
                        const uint8_t *key, int num_queues, int endian_check);
void ref_classify_fixed(uint8_t *buf, uint64_t stride, uint32_t frame_len, uint32_t n,
                        uint8_t *verdict, uint32_t *hash, uint16_t *queue,
                        uint32_t flags, const uint8_t *key, int num_queues,
                        int endian_check);

/* Batches over a buffer with per-frame byte offsets and lengths. */
void ref_verify_batch(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                      const uint16_t *len, uint32_t n, uint8_t *verdict,
                      uint32_t flags);
void ref_compute_batch(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                       const uint16_t *len, uint32_t n, uint8_t *status,
                       uint32_t *csums);
void ref_compute_batch_f(uint8_t *buf, uint64_t buf_bytes, const uint64_t *off,
                         const uint16_t *len, uint32_t n, uint8_t *status,
                         uint32_t *csums, uint32_t flags);

/* Fixed-stride batches (frame i at buf + i*stride, length frame_len). */
void ref_verify_fixed(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                      uint32_t n, uint8_t *verdict, uint32_t flags);
void ref_compute_fixed(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                       uint32_t n, uint8_t *status, uint32_t *csums);

/* Same, split over `threads` pthreads (independent frame shards, like
 * mTCP's per-core threads).  Used by bench.py's cpu_baseline. */
void ref_verify_fixed_mt(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                         uint32_t n, uint8_t *verdict, uint32_t flags,
                         int threads);
void ref_compute_fixed_mt(uint8_t *buf, uint64_t stride, uint32_t frame_len,
                          uint32_t n, uint8_t *status, uint32_t *csums,
                          int threads);

/* Element-wise function batches (one call of the reference function per item). */
void ref_tcp_checksum_batch(const uint8_t *buf, const uint64_t *off,
                            const uint16_t *len, const uint32_t *saddr,
                            const uint32_t *daddr, uint32_t n, uint16_t *out);
void ref_ip_checksum_batch(const uint8_t *buf, const uint64_t *off,
                           const uint8_t *ihl, uint32_t n, uint16_t *out);
void ref_icmp_checksum_batch(const uint8_t *buf, const uint64_t *off,
                             const uint16_t *len, uint32_t n, uint16_t *out);

#ifdef __cplusplus
}
#endif
#endif
