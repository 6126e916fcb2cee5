// gcs_internal.h -- launchers shared between gcs_kernels.hip and gcs_api.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtcp_gpucsum.h"

namespace gcs {

// Kernel-level extension arguments (GCS_VF_ICMP / GCS_CF_ICMP / RSS
// steering); the per-frame view is gcs_device.h's XFrame.
struct Ext {
    uint32_t key[4];           // RSS key bits 0..127 as big-endian words
    uint32_t* hash;            // per-frame outputs (nullable)
    uint16_t* queue;
    uint32_t nq, nq_magic, endian;   // nq_magic = ceil(2^32 / nq) (0 for nq == 1)
};

// Burst server (gcs_api.cpp ServerHub / BurstServer, gcs_kernels.hip
// k_burst_server): ONE short-lived resident grid per process and device that
// takes host batches from the request rings of up to kHubRings contexts (one
// per mTCP thread) in pinned fine-grained memory, instead of one kernel
// launch per batch -- and instead of one resident grid per context, each
// holding a hardware queue of its own (12 per-context grids
// cost the pinned verify 6-15%).  The grid has kServerBlocks blocks per ring
// in use (a ring's group); ring ids of the groups travel in the launch.
//
// A context's ring is kServerSlots request slots.  Request q (a 32-bit
// sequence number; numbers whose low 16 bits are 0 are never used, see
// server_next) lives in slot q % kServerSlots, so the host can post
// requests while earlier ones are still being served (the plugin's TX fill
// posts frames as mTCP completes them).  Every block of the ring's group
// serves its requests in order.  Request q's frames go to the blocks in turn
// starting at block server_rot(q) (kServerFPB frames per block and pass), so
// a run of small requests is served by different blocks at once.
//
// One poll is ONE load instruction of wave 0 of a block: lane 0 reads the
// slot's line A, lane 1 its line B, lanes 2.. the descriptors of the block's
// first frames of that request.  Each 16 B line is read in one piece and
// carries the request number, so a poll that sees seq q in all the lines it
// needs has a consistent request (the host writes each line's fields before
// its seq, and the lines before line A's seq).  Results go to tagged
// per-frame records in the slot; a block that served frames of q then
// releases and writes the ring's ack[b] = q (what the host waits for when the
// frames themselves were written in place).
//
// A block that has seen no request for hot_ticks goes cold: the group's
// block 0 (its leader) then reads only line A per poll and publishes each
// request it claims in HubPub (device memory); the other blocks follow that
// copy instead of polling host memory, and go hot again when a request has
// frames for them.
constexpr int kServerBlocks = 8;
constexpr int kServerFPB = 8;            // frames per block and pass (32 lanes x 3 chunks each)
constexpr int kServerSlots = 8;
constexpr int kSlotFrames = 512;         // frames per request
constexpr int kServerMaxFrames = 4096;   // a larger synchronous batch: several requests
constexpr int kHubRings = 32;            // contexts one grid serves (mTCP threads per GPU)
//
// Each 16 B line goes out as ONE store, but write-combined BAR memory may land
// a partial line as two 8 B halves in either order (Intel SDM 11.3.1), so a
// poll may read one half new and the other from the request that used the
// slot 8 requests earlier.  Every line therefore carries its request in BOTH
// halves: line A the tag (server_tag) beside n, line B and the descriptors
// the tag in the top 16 bits of their 48-bit address / offset (kTagShift).
// A poll takes a line as written only when both halves agree.
struct alignas(16) ServerReqA {
    uint32_t seq;                       // request number (written last)
    uint32_t cmd;                       // unused (0)
    uint32_t n;                         // frames | server_tag(seq) << 16
    uint32_t mode;                      // bit 0: compute (TX fill); bits 1..: flags
};
struct alignas(16) ServerReqB {
    uint64_t frames;                    // device address of the frame buffer (48 bits)
                                        // | server_tag(seq) << kTagShift
    uint32_t bytes16;                   // its size / 16
    uint32_t seq;
};
struct alignas(16) ServerDesc {
    uint64_t off;                       // offset (48 bits) | server_tag(seq) << kTagShift
    uint16_t len;
    uint16_t pad;
    uint32_t seq;
};
constexpr int kTagShift = 48;
constexpr uint64_t kAddrMask = (1ull << kTagShift) - 1;
struct alignas(64) ServerLine {
    uint32_t v;
    uint32_t pad[15];
};
// A request slot's lines: written by the host, read by the grid.  They live
// in HubReqs: uncached device memory the host writes over the BAR (default;
// the grid polls HBM: no PCIe read per poll) or, with
// GCS_SERVER_MAILBOX=host, pinned host memory the grid polls over PCIe.
struct alignas(64) ServerReq {
    ServerReqA a;
    ServerReqB b;
    uint8_t pad0[32];
    ServerDesc desc[kSlotFrames];
};
// A request slot's results (pinned host memory): one record per frame, written
// in ONE 8 B store once the frame is done: csum (ip | tcp << 16) | code << 32
// | (seq & 0xFFFF) << 48.  The host sees a request's results complete when
// every record carries its seq -- without waiting for the blocks' release
// fence and ack.
struct alignas(64) ServerRes {
    uint64_t rec[kSlotFrames];
};
// Phase counters (the k_burst_server<PROF = true> build, GCS_SERVER_COUNTERS=1
// or GCS_SERVER_PROF; the plain build by default): per block,
// running sums over the requests it served (HubReqs::prof, next to the
// request lines: in device memory they cost the PCIe link nothing), and the
// marks of its last request (ServerMailbox::mark, host memory: the host waits
// for them per request).
enum ServerProf {
    kProfN = 0,         // requests with frames in this block
    kProfSeenRtt = 1,   // sum: issue -> return of the poll that saw a request
    kProfAcq = 2,       // sum: the acquire after the poll
    kProfFrames = 3,    // sum: frame loads, folds, record stores issued
    kProfRecs = 4,      // sum: the record stores' acknowledgement
    kProfPolls = 5,     // sum: polls (all)
    kProfPollRtt = 6,   // sum: issue -> return, all polls
    kProfRel = 7,       // sum: release fence + ack (requests that wrote frames)
    kProfCold = 8,      // sum: requests the block was cold for when they came
    kProfSlow2 = 9,     // polls whose round trip took over 2 us
    kProfSlow5 = 10,    // ... over 5 us
    kProfMaxRtt = 11,   // the longest poll round trip (ticks)
    kProfTorn = 12,     // polls that saw line A of the request but not all its lines
    kProfWords = 16
};
// One context's ring (pinned host memory).
struct ServerMailbox {
    ServerLine ack[kServerBlocks];       // device: the last request each block served frames of
    ServerLine state[kServerBlocks];     // device: 1 serving, 2 exited (this launch's group)
    // device, counters: ONE 16 B store per request {seen lo, seen hi, rec -
    // seen, q} (u32 each): the clock when the poll that saw request q
    // returned, and how long after that its records were stored
    // (acknowledged) -- one store, so no fence orders the marks before their tag
    uint64_t mark[kServerBlocks][2];
    ServerRes res[kServerSlots];
};
struct HubMailbox {
    ServerMailbox ring[kHubRings];
};
// Written by the host, read by the grid (and the profile sums the other way):
// uncached device memory over the BAR by default, else pinned host memory.
struct HubReqs {
    ServerLine cmd;                      // host: 1 = leave now (the group leaders poll it)
    ServerReq req[kHubRings][kServerSlots];
    uint64_t prof[kHubRings][kServerBlocks][kProfWords];   // device: phase counter sums
};

// Device memory.  ent[r][q % kServerSlots] = q << 32 | n for each request q
// of ring r its group's leader claimed (n = 0 for one it skipped); exit[r] =
// that leader left.  prog[r][b] = the last request of ring r that block b
// finished: a fresh grid resumes there, so no block serves a request twice.
// The host sets a ring's entries (to the ring's start: "done") when a context
// joins, and clears exit[] before each launch.
struct alignas(16) PubFlag {
    uint32_t v;
    uint32_t pad[3];
};
struct HubPub {
    uint64_t ent[kHubRings][kServerSlots];
    PubFlag exit[kHubRings];
    uint32_t prog[kHubRings][kServerBlocks];
    uint32_t ring_of[kHubRings];         // host, before each launch: group g serves ring_of[g]
};

// The request number after q: q + 1, skipping numbers whose 16-bit record tag
// would be 0 (a cleared record reads as tag 0).  Host and kernel both use it.
__host__ __device__ inline uint32_t server_next(uint32_t q)
{
    q += 1;
    return (q & 0xFFFFu) == 0 ? q + 1 : q;
}

// Request q's 16-bit tag (its records and the second half of each request
// line carry it; never 0, see server_next).
__host__ __device__ inline uint32_t server_tag(uint32_t q)
{
    return q & 0xFFFFu;
}

// Request q starts at block 2q mod kServerBlocks and goes out kServerFPB
// frames per block: four consecutive requests of <= 16 frames (the plugin's
// RX and TX groups) land on disjoint blocks and are served side by side.  (A
// start of q mod 8 put consecutive 16-frame groups on overlapping blocks, so
// each group waited for the one before: ~3 us per group, round 4.)
constexpr uint32_t kServerRot = 2;
__host__ __device__ inline uint32_t server_rot(uint32_t q)
{
    return (kServerRot * q) % kServerBlocks;
}
// Block holding frame i of request q.
__host__ __device__ inline int server_block(uint32_t q, uint32_t i)
{
    return (int)((server_rot(q) + i / kServerFPB) % kServerBlocks);
}

// groups rings (group g serves ring pub->ring_of[g]); the grid is groups *
// kServerBlocks blocks.  A block stays hot for hot_ticks after a request, or
// for 3 x the gap between its last two requests when that is <= hot_max_ticks
// (a thread bursting every 50 us keeps its ring hot; one bursting every 200 us
// does not).
hipError_t launch_burst_server(HubMailbox* mb, HubReqs* rq, HubPub* pub, int groups,
                               uint64_t idle_ticks,
                               uint64_t life_ticks, uint64_t hot_ticks, uint64_t hot_max_ticks,
                               uint32_t max_polls, uint32_t naps, uint32_t opts, bool prof,
                               hipStream_t s);
// launch_burst_server opts, the acquire after a poll (A/B knobs,
// GCS_SERVER_ACQUIRE): by default a request whose frames are in device
// memory (ServerReqA::mode bit kModeDevFrames: device staging, which the
// host writes over the BAR and the XCD L2s keep coherent) takes an
// agent-scope acquire (the CU's L1 only), one whose frames are in host memory
// a system-scope one (which also invalidates the L2's non-coherent lines: a
// registered mbuf pool), and one in an uncached registered region
// (kModeUncachedFrames) the CU's L1 invalidate alone.  kServerAcqAgent: agent
// scope always; kServerAcqNone: no acquire for device or uncached frames.
constexpr uint32_t kServerAcqAgent = 1u;
constexpr uint32_t kServerAcqNone = 2u;

constexpr uint32_t kModeDevFrames = 1u << 31;
// ... and a request whose frames are in a region registered uncached
// (gcs_host_register: hipExtHostRegisterUncached, MTYPE UC) takes only a
// workgroup-scope invalidate (the CU's L1): no L2 or Infinity Cache line
// holds that memory, so there is nothing older to miss it in (RX bursts from
// an mbuf pool: the L2 invalidate was ~1 us of each).
constexpr uint32_t kModeUncachedFrames = 1u << 30;

hipError_t launch_verify_fixed(uint8_t* frames, uint64_t stride, uint32_t frame_len, uint32_t n,
                               uint8_t* verdict, uint32_t flags, hipStream_t s);
hipError_t launch_compute_fixed(uint8_t* frames, uint64_t stride, uint32_t frame_len, uint32_t n,
                                uint8_t* status, uint32_t* csums, uint32_t flags, hipStream_t s);
// A TX fill and an RX verify of two fixed-stride batches in one launch
// (k_fixed_step), or the two launches when their kernel shapes differ.
hipError_t launch_step_fixed(uint8_t* tx, uint64_t tx_stride, uint32_t tx_len, uint32_t ntx,
                             uint8_t* tx_code, uint32_t* tx_csum, uint32_t tx_flags, uint8_t* rx,
                             uint64_t rx_stride, uint32_t rx_len, uint32_t nrx, uint8_t* rx_code,
                             uint32_t rx_flags, hipStream_t s);
constexpr uint32_t kDescFrames = 256;    // frames per k_desc_stream block
hipError_t launch_verify_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                              const uint16_t* len, uint32_t n, uint8_t* verdict, uint32_t flags,
                              hipStream_t s);
hipError_t launch_compute_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                               const uint16_t* len, uint32_t n, uint8_t* status, uint32_t* csums,
                               uint32_t flags, hipStream_t s);
// Direct-mode host batch with its results as 8 B records (csum | code << 32)
// into pinned host memory, one 64 B line per block of 8 frames (k_desc_rec).
hipError_t launch_desc_rec(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                           const uint16_t* len, uint32_t n, uint64_t* rec, bool compute,
                           uint32_t flags, hipStream_t s);
hipError_t launch_classify_fixed(uint8_t* frames, uint64_t stride, uint32_t frame_len,
                                 uint32_t n, uint8_t* verdict, uint32_t flags, const Ext& ext,
                                 hipStream_t s);
hipError_t launch_classify_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                                const uint16_t* len, uint32_t n, uint8_t* verdict,
                                uint32_t flags, const Ext& ext, hipStream_t s);
hipError_t launch_copy_fill(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                            const uint16_t* len, const uint8_t* src, uint64_t src_bytes,
                            const uint64_t* src_off, uint32_t n, uint8_t* status,
                            uint32_t* csums, uint32_t flags, hipStream_t s);
hipError_t launch_gro(const uint8_t* in, uint64_t in_bytes, const uint64_t* off,
                      const uint16_t* len, const uint8_t* verdict, uint32_t n, uint32_t window,
                      uint32_t max_len, uint8_t* out, uint64_t out_bytes, uint64_t* out_off,
                      uint16_t* out_len, uint32_t* head, hipStream_t s);
hipError_t launch_icmp_fn(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off,
                          const uint16_t* len, uint32_t n, uint16_t* out, hipStream_t s);
hipError_t launch_rss_fn(const uint32_t* sip, const uint32_t* dip, const uint16_t* sp,
                         const uint16_t* dp, uint32_t n, const Ext& ext, hipStream_t s);
hipError_t launch_tcp_fn(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off,
                         const uint16_t* len, const uint32_t* saddr, const uint32_t* daddr,
                         uint32_t n, uint16_t* out, hipStream_t s);
hipError_t launch_ip_fn(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off,
                        const uint8_t* ihl, uint32_t n, uint16_t* out, hipStream_t s);

}  // namespace gcs
