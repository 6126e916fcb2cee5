// gcs_kernels.hip -- gfx950 (CDNA4) kernels + launchers for mTCP's software
// checksum path.  The per-frame device code (and the derivation of why the
// lane-split sums are bit-exact) is in gcs_device.h.
#include "gcs_device.h"
#include "gcs_internal.h"

#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace gcs {

constexpr int kBlock = 256;

// Launch-time choices, fixed by the A/B runs recorded in DESIGN.md App. A
// (tools/kbench.hip): non-temporal loads for the once-read frame stream
// (verify 250 -> 236 us per 1M x 1500 B), and check fields written back as
// whole 64 B sectors with sc1 stores (no partial-line writes; the TX+RX step
// 531 -> 515 us against 2-byte stores).
constexpr bool kNT = true;
constexpr int kWM = WM_SECTOR_SC1;
// XCD-contiguous frame ranges (xcd_block below): TX+RX step 491 -> 485 us.
constexpr bool kXCD = true;
// k_desc_mixed register budget: 6 waves per SIMD (80 VGPRs; one 8-byte value goes to
// scratch around the list passes: a store and a reload per thread, outside the loops).
// 4M IMIX frames: verify 349 -> 316 us against the unbounded 89-94 VGPRs (5
// waves); 8 waves spills and takes 385 us.
constexpr int kDescOcc = 6;

// Fixed stride: frame i at frames + i*stride, length frame_len,
// 16*ceil(frame_len/16) <= stride.  One frame per G-lane group, 256/G frames
// per workgroup, one workgroup per 256/G frames (no grid-stride loop: the
// short-lived waves keep more bytes in flight than a persistent grid did).
// XCD-aware block order (cdna_hip_programming.md T1): workgroups are dealt
// round-robin over the 8 XCDs, so block b runs on the XCD of b % 8.  Remap b
// to a logical block such that every XCD owns ONE contiguous range of frames:
// the per-frame outputs (verdict bytes, csums) of neighbouring frames are then
// written through the same XCD L2 and leave it as whole sectors instead of
// partial ones from eight L2s.  Bijective for any grid size; speed only.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb)
{
    const uint32_t q = nb / 8, r = nb % 8, x = b % 8, k = b / 8;
    return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}

// The extension outputs of frame i (EXT kernels only).
__device__ __forceinline__ XFrame xframe(const Ext& x, uint64_t i)
{
    return XFrame{{x.key[0], x.key[1], x.key[2], x.key[3]}, x.hash ? x.hash + i : nullptr,
                  x.queue ? x.queue + i : nullptr, x.nq, x.nq_magic, x.endian, nullptr};
}

// K > 1: each group takes K frames, FPB apart (so every load instruction of a
// wave still reads one contiguous range), and issues the loads of all K before
// folding any: small frames give a lane only U*16 bytes each, too few bytes in
// flight per wave to cover HBM latency.
// bid / nb: this block's index in, and the size of, the grid (or the part of
// a grid, k_fixed_step) that takes this batch.
template <int G, int U, bool COMPUTE, bool LOOP, bool NT, int WM, bool XCD, bool EXT, int K = 1>
__device__ __forceinline__ void fixed_frame(uint8_t* __restrict__ frames, uint64_t stride,
                                            u32 frame_len, u32 n, uint8_t* __restrict__ out_code,
                                            uint32_t* __restrict__ out_csum, u32 flags,
                                            const Ext& ext, uint32_t bid, uint32_t nb)
{
    constexpr int FPB = kBlock / G;                    // frames per block and batch
    const int sub = threadIdx.x & (G - 1);
    const uint32_t blk = XCD ? xcd_block(bid, nb) : bid;
    const uint64_t i0 = (uint64_t)blk * FPB * K + threadIdx.x / G;
    if (i0 >= n)
        return;                                        // whole group leaves together
    if constexpr (K == 1) {
        do_frame<G, U, COMPUTE, LOOP, false, NT, WM, EXT>(frames + i0 * stride, frame_len,
                                                          (int64_t)stride, true, sub, flags,
                                                          out_code ? out_code + i0 : nullptr,
                                                          out_csum ? out_csum + i0 : nullptr,
                                                          true, EXT ? xframe(ext, i0) : XFrame{});
    } else {
        static_assert(!LOOP, "K > 1 is for frames that fit one batch");
        const int nch = (int)((frame_len + 15) >> 4);
        uint4 v[K][U];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = i0 + (uint64_t)k * FPB;
            if (i < n) {
                load_first<G, U, false, NT>(frames + i * stride, nch, (int64_t)stride, sub, v[k]);
            } else {
#pragma unroll
                for (int j = 0; j < U; j++)
                    v[k][j] = make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = i0 + (uint64_t)k * FPB;
            if (i >= n)
                break;                                 // group-uniform, and so are later k
            uint8_t* f = frames + i * stride;
            frame_body<G, U, COMPUTE, false, false, NT, WM, EXT>(
                v[k], f, f, frame_len, (int64_t)stride, true, sub, flags,
                out_code ? out_code + i : nullptr, out_csum ? out_csum + i : nullptr, true,
                EXT ? xframe(ext, i) : XFrame{});
        }
    }
}

template <int G, int U, bool COMPUTE, bool LOOP, bool NT, int WM, bool XCD = false, int K = 1>
__global__ void __launch_bounds__(kBlock)
k_fixed(uint8_t* __restrict__ frames, uint64_t stride, u32 frame_len, u32 n,
        uint8_t* __restrict__ out_code, uint32_t* __restrict__ out_csum, u32 flags)
{
    fixed_frame<G, U, COMPUTE, LOOP, NT, WM, XCD, false, K>(frames, stride, frame_len, n,
                                                            out_code, out_csum, flags, Ext{},
                                                            blockIdx.x, gridDim.x);
}

// One launch for a TX fill and an RX verify of two fixed-stride batches
// (gcs_step_fixed_dev: mTCP's loop folds both every iteration, core.c:761-877):
// blocks [0, tx_blocks) fill the TX batch, the rest verify the RX batch, so
// the verify's first blocks run in the fill's tail instead of behind a
// kernel boundary.  tx_blocks is a multiple of 8: both parts keep the
// XCD-contiguous block order (xcd_block).
template <int G, int U, bool LOOP, int WMA, int WMB>
__global__ void __launch_bounds__(kBlock)
k_fixed_step(uint8_t* __restrict__ tx, uint64_t tx_stride, u32 tx_len, u32 ntx,
             uint8_t* __restrict__ tx_code, uint32_t* __restrict__ tx_csum, u32 tx_flags,
             uint8_t* __restrict__ rx, uint64_t rx_stride, u32 rx_len, u32 nrx,
             uint8_t* __restrict__ rx_code, u32 rx_flags, u32 tx_blocks, u32 tx_split,
             u32 rx_blocks, u32 order)
{
    // which part this block serves, and its index in that part: order 0 =
    // the TX blocks first, 1 = the RX blocks first, 2 = 8-block groups of
    // the two alternating (both block counts are multiples of 8, so a block
    // keeps its XCD, b % 8, in its part)
    uint32_t b = blockIdx.x;
    bool is_tx;
    if (order == 0) {
        is_tx = b < tx_blocks;
        b = is_tx ? b : b - tx_blocks;
    } else if (order == 1) {
        is_tx = b >= rx_blocks;
        b = is_tx ? b - rx_blocks : b;
    } else {
        const uint32_t g = b / 8, gt = tx_blocks / 8, gr = rx_blocks / 8;
        const uint32_t both = gt < gr ? gt : gr;
        if (g < 2 * both) {
            is_tx = (g & 1) == 0;
            b = (g / 2) * 8 + b % 8;
        } else {
            is_tx = gt > gr;
            b = (both + g - 2 * both) * 8 + b % 8;
        }
    }
    // the fill's write-back as launch_fixed picks it (k_fixed_tx2): WMA for
    // its logical blocks [0, tx_split), WMB after
    if (is_tx) {
        const uint32_t blk = xcd_block(b, tx_blocks);
        if (blk < tx_split)
            fixed_frame<G, U, true, LOOP, kNT, WMA, false, false>(tx, tx_stride, tx_len, ntx,
                                                                  tx_code, tx_csum, tx_flags,
                                                                  Ext{}, blk, tx_blocks);
        else
            fixed_frame<G, U, true, LOOP, kNT, WMB, false, false>(tx, tx_stride, tx_len, ntx,
                                                                  tx_code, tx_csum, tx_flags,
                                                                  Ext{}, blk, tx_blocks);
    } else {
        fixed_frame<G, U, false, LOOP, kNT, kWM, kXCD, false>(rx, rx_stride, rx_len, nrx, rx_code,
                                                              nullptr, rx_flags, Ext{}, b,
                                                              rx_blocks);
    }
}

// k_fixed with the extensions (ICMP fold, RSS steering): a separate
// instantiation so the plain path carries none of their registers.
template <int G, int U, bool COMPUTE, bool LOOP, bool NT, int WM, bool XCD, int K = 1>
__global__ void __launch_bounds__(kBlock)
k_fixed_x(uint8_t* __restrict__ frames, uint64_t stride, u32 frame_len, u32 n,
          uint8_t* __restrict__ out_code, uint32_t* __restrict__ out_csum, u32 flags, Ext ext)
{
    fixed_frame<G, U, COMPUTE, LOOP, NT, WM, XCD, true, K>(frames, stride, frame_len, n, out_code,
                                                           out_csum, flags, ext, blockIdx.x,
                                                           gridDim.x);
}

// Small frames (<= 64 B, C1): ONE LANE PER FRAME.  A lane loads its frame's
// (up to) four 16 B chunks itself, so there is no cross-lane reduction, the
// ihl == 5 word masks are compile-time constants per register, and the 64
// verdict bytes of a wave are one coalesced 64 B store.  (The G-lane kernels
// spend most of their instructions on reductions and a per-group epilogue at
// this size: tools/kbench.hip, DESIGN.md App. A.)
__device__ __forceinline__ XFrame small_xframe(const Ext& x, uint64_t i, const u32* nib)
{
    XFrame f = xframe(x, i);
    f.nib = nib;
    return f;
}

template <bool COMPUTE, bool NT, bool XCD, bool EXT>
__device__ __forceinline__ void small_frame(uint8_t* __restrict__ frames, uint64_t stride,
                                            u32 frame_len, u32 n, uint8_t* __restrict__ out_code,
                                            uint32_t* __restrict__ out_csum, u32 flags,
                                            const Ext& ext)
{
    __shared__ u32 nib[EXT ? kNibEntries : 1];
    const bool rss = EXT && !COMPUTE && (ext.hash || ext.queue);   // kernel-uniform
    if (rss)
        rss_nibble_tables(ext.key, nib);
    const uint32_t blk = XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint64_t i = (uint64_t)blk * kBlock + threadIdx.x;
    if (i >= n)
        return;
    uint8_t* f = frames + i * stride;
    const int nch = (int)((frame_len + 15) >> 4);      // <= 4, uniform
    uint4 v[4];
#pragma unroll
    for (int c = 0; c < 4; c++)
        v[c] = c < nch ? ldg16<NT>(f + 16 * c) : make_uint4(0, 0, 0, 0);
    Hdr h = {v[0].w, v[1].x, v[1].y};
    const int ts = 14 + 4 * (int)((h.d3 >> 16) & 15u);
    const int te = 14 + (int)bswap16(h.d4 & 0xFFFFu);
    Acc a = {0u, 0u, 0u};
    if (ts == 34) {
        // ihl == 5: constant masks (see masks5); only the chunk holding te is cut
#pragma unroll
        for (int c = 0; c < 4; c++)
            accum_fast5<COMPUTE, true>(v[c], c, te, masks5<COMPUTE>(c), a);
    } else {
#pragma unroll
        for (int c = 0; c < 4; c++)
            accum_chunk<COMPUTE>(v[c], 16 * c, ts, te, a);
    }
    // one-lane "group": epilogue<1, 4> finishes the frame (no reduction steps)
    epilogue<1, 4, COMPUTE, kWM, EXT>(h, a, f, frame_len, (int64_t)stride, true, 0, flags,
                                      out_code ? out_code + i : nullptr,
                                      out_csum ? out_csum + i : nullptr, true, v,
                                      EXT ? small_xframe(ext, i, nib) : XFrame{});
}

template <bool COMPUTE, bool NT, bool XCD>
__global__ void __launch_bounds__(kBlock)
k_small(uint8_t* __restrict__ frames, uint64_t stride, u32 frame_len, u32 n,
        uint8_t* __restrict__ out_code, uint32_t* __restrict__ out_csum, u32 flags)
{
    small_frame<COMPUTE, NT, XCD, false>(frames, stride, frame_len, n, out_code, out_csum, flags,
                                         Ext{});
}

template <bool COMPUTE, bool NT, bool XCD>
__global__ void __launch_bounds__(kBlock)
k_small_x(uint8_t* __restrict__ frames, uint64_t stride, u32 frame_len, u32 n,
          uint8_t* __restrict__ out_code, uint32_t* __restrict__ out_csum, u32 flags, Ext ext)
{
    small_frame<COMPUTE, NT, XCD, true>(frames, stride, frame_len, n, out_code, out_csum, flags,
                                        ext);
}

// Descriptor batch: frame i at frames + off[i], length len[i], one frame per
// G-lane group (longer frames in further batches of G*U chunks).  Device
// batches with the rooms hint
// (GCS_VF_ROOMS / GCS_CF_ROOMS: frames one per mbuf room, which the packed
// stream cannot stream; XCD-contiguous blocks, and for a fill of lines that
// fit the Infinity Cache the whole-line write-back of k_fixed).
template <int G, int U, bool COMPUTE, bool NT, int WM, bool XCD = false>
__global__ void __launch_bounds__(kBlock)
k_desc(uint8_t* __restrict__ frames, uint64_t frames_bytes, const uint64_t* __restrict__ off,
       const uint16_t* __restrict__ lens, u32 n, uint8_t* __restrict__ out_code,
       uint32_t* __restrict__ out_csum, u32 flags)
{
    constexpr int FPB = kBlock / G;
    const int sub = threadIdx.x & (G - 1);
    const uint32_t blk = XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint64_t i = (uint64_t)blk * FPB + threadIdx.x / G;
    if (i >= n)
        return;
    const uint64_t o = off[i];
    const u32 len = lens[i];
    const bool ok = (o & 15) == 0 && o <= frames_bytes && len <= frames_bytes - o;
    uint8_t* f = frames + (ok ? o : 0);
    do_frame<G, U, COMPUTE, true, true, NT, WM>(f, len, ok ? (int64_t)(frames_bytes - o) : 0,
                                                ok, sub, flags,
                                                out_code ? out_code + i : nullptr,
                                                out_csum ? out_csum + i : nullptr);
}

// Direct-mode host batch (gcs_api.cpp run_host_batch: a small batch whose
// results go straight into pinned host memory, without the burst server):
// k_desc's one frame per 32-lane group, 8 frames per block, but each block
// stages its frames' results in LDS and writes them as ONE 64 B line of 8 B
// records (csum | code << 32), the burst server's record format: every
// partial-line write into host memory is a fabric write of its own (round 5:
// eight 8 B record stores per block made the server's way back grow 1.6 ->
// 24 us at 16 threads), and the plain k_desc wrote a 1 B verdict and a 4 B
// check per frame.
template <int G, int U, bool COMPUTE>
__global__ void __launch_bounds__(kBlock)
k_desc_rec(uint8_t* __restrict__ frames, uint64_t frames_bytes, const uint64_t* __restrict__ off,
           const uint16_t* __restrict__ lens, u32 n, uint64_t* __restrict__ out_rec, u32 flags)
{
    constexpr int FPB = kBlock / G;
    static_assert(FPB == 8, "one 64 B line of records per block");
    __shared__ uint8_t s_code[FPB];
    __shared__ uint32_t s_csum[FPB];
    const int sub = threadIdx.x & (G - 1), grp = threadIdx.x / G;
    const uint64_t i = (uint64_t)blockIdx.x * FPB + grp;
    const bool here = i < n;                           // group-uniform
    if (sub == 0)
        s_csum[grp] = 0;
    if (here) {
        const uint64_t o = off[i];
        const u32 len = lens[i];
        const bool ok = (o & 15) == 0 && o <= frames_bytes && len <= frames_bytes - o;
        uint8_t* f = frames + (ok ? o : 0);
        do_frame<G, U, COMPUTE, true, true, kNT, kWM>(f, len,
                                                      ok ? (int64_t)(frames_bytes - o) : 0, ok,
                                                      sub, flags, s_code + grp,
                                                      COMPUTE ? s_csum + grp : nullptr);
    }
    __syncthreads();                                   // the block's results in LDS
    if (threadIdx.x < FPB / 2) {
        const int t = threadIdx.x;
        const uint64_t j = (uint64_t)blockIdx.x * FPB + 2 * t;
        const uint64_t r0 = (uint64_t)s_csum[2 * t] | ((uint64_t)s_code[2 * t] << 32);
        const uint64_t r1 = (uint64_t)s_csum[2 * t + 1] | ((uint64_t)s_code[2 * t + 1] << 32);
        if (j + 1 < n) {
            const u32x4 w = {(u32)r0, (u32)(r0 >> 32), (u32)r1, (u32)(r1 >> 32)};
            asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1"
                         : : "v"(&out_rec[j]), "v"(w) : "memory");
        } else if (j < n) {
            __hip_atomic_store(&out_rec[j], r0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

hipError_t launch_desc_rec(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                           const uint16_t* len, uint32_t n, uint64_t* rec, bool compute,
                           uint32_t flags, hipStream_t s)
{
    constexpr int G = 32, U = 3, FPB = kBlock / G;
    const dim3 grid((n + FPB - 1) / FPB);
    if (compute)
        hipLaunchKernelGGL((k_desc_rec<G, U, true>), grid, dim3(kBlock), 0, s, frames,
                           frames_bytes, off, len, n, rec, flags);
    else
        hipLaunchKernelGGL((k_desc_rec<G, U, false>), grid, dim3(kBlock), 0, s, frames,
                           frames_bytes, off, len, n, rec, flags);
    return hipGetLastError();
}

// Burst server: a grid of kServerBlocks blocks per ring in use that stays
// resident for at most life_ticks (wall clock) and serves the host batches
// posted in the contexts' request rings (gcs_internal.h HubMailbox) -- each
// batch with the per-frame work of k_desc<G,U> (frames in pinned host memory,
// read and written over PCIe), without a kernel launch and event wait per
// batch.  Group g (blocks 8g..8g+7) serves ring pub->ring_of[g]: each of
// its blocks serves every request in order (q = server_next(last)); its
// frames of request q are i = kServerFPB * ((b - q) mod kServerBlocks) + grp,
// then + 64 per pass.
//
// Every block ends: on the host's exit command (which each group's leader
// polls and publishes), after idle_ticks without a request, after life_ticks
// in total, or after max_polls polls -- whichever comes first, so the grid
// always drains.  All decisions are taken by wave 0 from the poll's lines
// and broadcast through LDS (block-uniform control flow: no wave leaves the
// loop while another waits at a barrier).
// Phase counters (PROF): the wall clock once every vector-memory access of this
// wave issued so far has completed (loads returned, stores acknowledged).
__device__ __forceinline__ uint64_t clock_after_vmem()
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return __builtin_amdgcn_s_memrealtime();
}

template <int G, int U, bool PROF, int BT = kBlock>
__global__ void __launch_bounds__(BT)
k_burst_server(HubMailbox* mb, HubReqs* rq, HubPub* pub, uint64_t idle_ticks, uint64_t life_ticks,
               uint64_t hot_ticks, uint64_t hot_max_ticks, uint32_t max_polls, uint32_t naps,
               uint32_t opts)
{
    enum { IDLE = 0, WORK = 1, EXIT = 2, SKIP = 3 };
    constexpr int FPB = BT / G;
    static_assert(FPB == kServerFPB, "the mailbox's frames per block and pass");
    constexpr int kPass = kServerBlocks * FPB;          // frames of one request per pass
    constexpr int kLanes = 2 + FPB;                     // lines of a poll
    constexpr int kAhead = kServerSlots - 1;            // + line A of the next requests
    __shared__ uint4 s_line[kLanes];
    __shared__ uint32_t s_claim, s_last;
    __shared__ uint8_t s_code[FPB];          // a frame's results, packed into its record
    __shared__ uint32_t s_csum[FPB];
    const int t = threadIdx.x, sub = t & (G - 1), grp = t / G;
    const int wave = t >> 6, lane = t & 63;
    const int blk = blockIdx.x % kServerBlocks;
    const int r = (int)(pub->ring_of[blockIdx.x / kServerBlocks] % kHubRings);
    const bool leader = blk == 0;
    ServerMailbox* rm = &mb->ring[r];
    ServerReq* rr = rq->req[r];
    uint32_t last = pub->prog[r][blk], polls = 0;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint64_t t_last = t_start;               // this block's last request (hot window, idle exit)
    // adaptive hot window: 3 x the gap between this block's last two
    // requests when that is <= hot_max_ticks, at least hot_ticks
    uint64_t win = hot_ticks, t_claim = t_start;
    // PROF (thread 0): this launch's additions to the block's sums
    uint64_t p_issue = 0, p_seen = 0, p_rtt = 0, p_sum[kProfWords] = {};
    uint64_t* const psum = rq->prof[r][blk];
    uint64_t p_polls0 = 0, p_rtt0 = 0, p_slow2 = 0, p_slow5 = 0, p_maxrtt = 0, p_torn = 0;
    bool p_cold = false;                     // a cold poll since the last request
    // ack[blk] must stay within 2^31 of the ring's requests (the host reads
    // it as a 32-bit serial number): a block acks each request that wrote
    // frames in place, and otherwise refreshes it at the start and every 2^30
    // requests.  Acking q without a fence is sound: every earlier in-place
    // request was acked behind its own release (a previous grid's ended with
    // its kernel), and q itself wrote nothing.
    uint32_t acked = last;
    if (t == 0) {
        s_claim = IDLE;
        if (PROF)                            // the sums go on from the block's last launch
            for (int k = 0; k < kProfWords; k++)
                p_sum[k] = __hip_atomic_load(&psum[k], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&rm->ack[blk].v, last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&rm->state[blk].v, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    p_polls0 = p_sum[kProfPolls];
    p_rtt0 = p_sum[kProfPollRtt];
    p_slow2 = p_sum[kProfSlow2];
    p_slow5 = p_sum[kProfSlow5];
    p_maxrtt = p_sum[kProfMaxRtt];
    p_torn = p_sum[kProfTorn];
    __syncthreads();
    for (;;) {
        const uint32_t q = server_next(last);            // the request this block serves next
        ServerReq* sl = &rr[q % kServerSlots];
        const uint32_t first = (uint32_t)FPB * ((blk + kServerBlocks - server_rot(q)) %
                                                kServerBlocks);   // this block's first frame of q
        if (wave == 0) {
            for (;;) {
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                const bool hot = now - t_last <= win;
                // ONE load per lane, all in flight together: the lines of q
                // when hot (the leader reads line A when cold too), the
                // leader's entry for q's slot for a cold follower (the 16 B
                // pair holding it), and in lane 63 the exit flag (the host's
                // command for the leader; the leader's exit, every 8th poll,
                // for the others)
                const bool follow = !hot && !leader && lane == 0;
                // hot, lanes kLanes..: line A of requests q_1..q_kAhead after
                // q, so that one poll claims a run of requests none of whose
                // frames are here (the plugin's small groups, posted together)
                const bool ahead = hot && lane >= kLanes && lane < kLanes + kAhead;
                uint32_t qk = q;
                if (ahead)
                    for (int j = kLanes; j <= lane; j++)
                        qk = server_next(qk);
                const volatile u32x4* src = nullptr;
                if (ahead)
                    src = reinterpret_cast<const volatile u32x4*>(&rr[qk % kServerSlots].a);
                else if ((hot && lane < kLanes) || (leader && lane == 0))
                    src = lane == 0   ? reinterpret_cast<const volatile u32x4*>(&sl->a)
                          : lane == 1 ? reinterpret_cast<const volatile u32x4*>(&sl->b)
                                      : reinterpret_cast<const volatile u32x4*>(&sl->desc[first + lane - 2]);
                else if (follow)
                    src = reinterpret_cast<const volatile u32x4*>(
                        &pub->ent[r][(q % kServerSlots) & ~1u]);
                else if (lane == 63 && (leader || (polls & 7) == 0))
                    src = leader ? reinterpret_cast<const volatile u32x4*>(&rq->cmd.v)
                                 : reinterpret_cast<const volatile u32x4*>(&pub->exit[r].v);
                u32x4 v = {0, 0, 0, 0};
                if (src)                         // global_load (the lines are never LDS)
                    v = *(const volatile __attribute__((address_space(1))) u32x4*)src;
                // Whole lines only (gcs_internal.h: the host's 16 B lines may
                // land as two 8 B halves).  A line A whose halves name
                // different requests reads as the request before the one
                // expected (look again); n loses its tag.  Line B and the
                // descriptors keep their tag for the torn test below, and
                // lose it from the address / offset.
                const bool line_a = ahead || (lane == 0 && !follow);
                const bool line_bd = !ahead && hot && lane >= 1 && lane < kLanes;
                const bool bd_whole = (v.y >> 16) == server_tag(q);
                if (line_a) {
                    if ((v.z >> 16) != server_tag(v.x))
                        v.x = (ahead ? qk : q) - 1u;
                    v.z &= 0xFFFFu;
                } else if (line_bd) {
                    v.y &= 0xFFFFu;
                }
                if (PROF) {
                    const uint64_t back = clock_after_vmem();
                    p_issue = now;
                    p_seen = back;
                    p_rtt += back - now;
                    p_cold |= !hot;
                    p_slow2 += back - now > 200 ? 1 : 0;     // 100 MHz clock
                    p_slow5 += back - now > 500 ? 1 : 0;
                    p_maxrtt = back - now > p_maxrtt ? back - now : p_maxrtt;
                }
                // line A's (seq, n), or the leader's entry's (q, n)
                uint32_t dq = v.x, dn = v.z;
                if (follow) {
                    dq = (q & 1u) ? v.w : v.y;
                    dn = (q & 1u) ? v.z : v.x;
                }
                const uint32_t x0 = __shfl(dq, 0), z0 = __shfl(dn, 0);
                // a consistent poll has request q whole in line B and in the
                // descriptor lines of the block's frames: each lane checks its
                // own line, both halves
                const bool torn = line_bd && first + (lane >= 2 ? lane - 2 : 0) < z0 &&
                                  (v.w != q || !bd_whole);
                const bool ok = __ballot(torn) == 0;
                uint32_t act = IDLE;
                if (hot) {
                    if (PROF && x0 == q && !ok)
                        p_torn++;
                    if (x0 == q)
                        act = ok ? WORK : IDLE;  // torn poll: look again
                    else if ((int32_t)(x0 - q) > 0)
                        act = SKIP;             // q is done and its slot reused: this block
                                                // had no frames in it (the host reuses a slot
                                                // only after its request completed)
                } else if (leader) {
                    if (x0 == q && first >= z0) {
                        act = WORK;             // out, none of its frames here: publish n
                    } else if (x0 == q) {
                        // out: publish it now, so the other blocks start their
                        // polls of it while this one reads its lines
                        if (lane == 0)
                            __hip_atomic_store(&pub->ent[r][q % kServerSlots],
                                               ((uint64_t)q << 32) | z0, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        t_last = now;
                    } else if ((int32_t)(x0 - q) > 0) {
                        act = SKIP;
                    }
                } else {
                    // the leader's entry for q's slot: q itself (skip it unless
                    // it has frames here), a newer request (q is done), or older
                    if (x0 == q && first < z0)
                        t_last = now;
                    else if ((int32_t)(x0 - q) >= 0)
                        act = SKIP;
                }
                if (__shfl(v.x, 63) != 0 || now - t_start > life_ticks || ++polls >= max_polls ||
                    (act == IDLE && now - t_last > idle_ticks))
                    act = EXIT;
                if (act == IDLE) {
                    // naps: extra ~4k-cycle naps between polls, the low 16 bits
                    // for a cold block, the high 16 for a hot one
                    __builtin_amdgcn_s_sleep(2);
                    for (uint32_t k = 0, m = hot ? naps >> 16 : naps & 0xFFFFu; k < m; k++)
                        __builtin_amdgcn_s_sleep(63);
                    continue;
                }
                // a WORK claim of q without frames here also claims the posted
                // requests right after it that have none here either
                int run = 0;
                {
                    const uint32_t fk = (uint32_t)FPB * ((blk + kServerBlocks - server_rot(qk)) %
                                                         kServerBlocks);
                    const uint64_t okm = __ballot(ahead && v.x == qk && fk >= v.z) >> kLanes;
                    if (act == WORK && first >= z0)
                        run = __builtin_ctzll(~okm);
                    run = run < kAhead ? run : kAhead;
                }
                const uint32_t qlast = run ? (uint32_t)__shfl((int)qk, kLanes + run - 1) : q;
                if (leader && ahead && lane < kLanes + run)
                    __hip_atomic_store(&pub->ent[r][qk % kServerSlots], ((uint64_t)qk << 32) | v.z,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (lane == 0) {
                    s_claim = act;
                    s_last = qlast;
                }
                if (act == WORK && lane < kLanes)
                    s_line[lane] = make_uint4(v.x, v.y, v.z, v.w);
                break;
            }
        }
        __syncthreads();
        const uint32_t act = s_claim;
        const uint32_t qend = s_last;        // q, or the last request of a claimed run
        if (act == EXIT) {
            if (leader && t == 0)
                __hip_atomic_store(&pub->exit[r].v, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        if (leader && t == 0) {
            // the leader publishes what it claimed before serving it: one
            // self-describing 8 B entry (no ordering against other stores)
            const uint64_t e = ((uint64_t)q << 32) | (act == WORK ? s_line[0].z : 0u);
            __hip_atomic_store(&pub->ent[r][q % kServerSlots], e, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        bool mine = false;
        uint64_t t_acq = 0, t_frames = 0, t_rec = 0;
        bool writes = false;
        if (act == WORK) {
            // a request: its lines were written before its seq (fence-acquire
            // after observing it: later loads see everything the host wrote)
            const uint4 a = s_line[0], b = s_line[1];
            const bool dev = (a.w & kModeDevFrames) != 0;   // block-uniform
            const bool unc = (a.w & kModeUncachedFrames) != 0;
            if ((dev || unc) && (opts & kServerAcqNone))
                ;
            else if (unc && !(opts & kServerAcqAgent))
                asm volatile("buffer_inv sc0" ::: "memory");   // the CU's L1 only
            else if (dev || (opts & kServerAcqAgent))
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            else
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            if (PROF)
                t_acq = clock_after_vmem();
            const uint32_t n = a.z, compute = a.w & 1u, flags = (a.w & ~(kModeDevFrames | kModeUncachedFrames)) >> 1;
            // frames written in place: a fill's check fields, or a verify's
            // tcp_in.c:1237 side effect
            writes = compute ? !(flags & GCS_CF_NO_INPLACE)
                             : (flags & GCS_VF_ZERO_BAD_TCP_CHECK) != 0;
            uint8_t* frames = reinterpret_cast<uint8_t*>((uint64_t)b.x |
                                                         ((uint64_t)(b.y & 0xFFFFu) << 32));
            const uint64_t bytes = (uint64_t)b.z * 16;
            const uint4 d0 = s_line[2 + grp];
            uint64_t* rec = rm->res[q % kServerSlots].rec;
            mine = first < n;                            // block-uniform: frames of q here
            // the block's frames of q in passes of FPB (one per group); each
            // pass's records leave as ONE 64 B line (four lanes x 16 B), not
            // as eight 8 B writes: every partial-line write to host memory is
            // a fabric write of its own, and at 8-16 rings the records' way
            // back grew from 1.6 to 10-24 us
            const uint32_t npass = mine ? (n - first + kPass - 1) / kPass : 0;   // block-uniform
            for (uint32_t pass = 0; pass < npass; pass++) {
                const uint32_t base = first + pass * kPass, i = base + grp;
                const bool here = i < n;                 // group-uniform
                uint4 d = d0;
                if (pass != 0 && here) {
                    // written before line A's fence: whole once A was seen
                    const u32x4 w = *(const volatile __attribute__((address_space(1))) u32x4*)
                                         &sl->desc[i];
                    d = make_uint4(w.x, w.y, w.z, w.w);
                }
                const uint64_t o = (uint64_t)d.x | ((uint64_t)(d.y & 0xFFFFu) << 32);
                const u32 len = d.z & 0xFFFFu;
                const bool ok = (o & 15) == 0 && o <= bytes && len <= bytes - o;
                uint8_t* f = frames + (ok ? o : 0);
                const int64_t avail = ok ? (int64_t)(bytes - o) : 0;
                if (sub == 0)
                    s_csum[grp] = 0;
                if (compute)
                    do_frame<G, U, true, true, true, kNT, kWM>(f, len, avail, ok, sub, flags,
                                                               s_code + grp, s_csum + grp, here);
                else
                    do_frame<G, U, false, true, true, kNT, kWM>(f, len, avail, ok, sub, flags,
                                                                s_code + grp, nullptr, here);
                __syncthreads();                         // the pass's results in LDS
                if (t < FPB / 2) {
                    const uint32_t j = base + 2 * t;
                    const uint64_t tag = (uint64_t)(q & 0xFFFFu) << 48;
                    const uint64_t r0 = (uint64_t)s_csum[2 * t] |
                                        ((uint64_t)s_code[2 * t] << 32) | tag;
                    const uint64_t r1 = (uint64_t)s_csum[2 * t + 1] |
                                        ((uint64_t)s_code[2 * t + 1] << 32) | tag;
                    if (j + 1 < n) {
                        const u32x4 w = {(u32)r0, (u32)(r0 >> 32), (u32)r1, (u32)(r1 >> 32)};
                        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1"
                                     : : "v"(&rec[j]), "v"(w) : "memory");
                    } else if (j < n) {
                        __hip_atomic_store(&rec[j], r0, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
                __syncthreads();                         // s_code / s_csum free again
            }
            if (PROF && mine) {
                __syncthreads();
                t_frames = __builtin_amdgcn_s_memrealtime();
                (void)clock_after_vmem();        // every wave's record stores acknowledged
                __syncthreads();
                t_rec = __builtin_amdgcn_s_memrealtime();
            }
            // frames written in place reach host memory before the ack; the
            // records are system-scope stores of their own, so a request that
            // writes no frame needs neither the release (an L2 write-back of
            // the whole XCD) nor the ack
            if (mine && writes)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        }
        __syncthreads();                     // every wave done with s_line / s_claim
        if (t == 0) {
            if (mine && writes) {
                __hip_atomic_store(&rm->ack[blk].v, q, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                acked = q;
            } else if (qend - acked >= (1u << 30)) {
                __hip_atomic_store(&rm->ack[blk].v, qend, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                acked = qend;
            }
            if (PROF && mine) {
                const uint64_t t_rel = clock_after_vmem();
                p_sum[kProfN] += 1;
                p_sum[kProfSeenRtt] += p_seen - p_issue;
                p_sum[kProfAcq] += t_acq - p_seen;
                p_sum[kProfFrames] += t_frames - t_acq;
                p_sum[kProfRecs] += t_rec - t_frames;
                p_sum[kProfRel] += writes ? t_rel - t_rec : 0;
                p_sum[kProfPolls] = p_polls0 + polls;
                p_sum[kProfPollRtt] = p_rtt0 + p_rtt;
                p_sum[kProfCold] += p_cold ? 1 : 0;
                p_sum[kProfSlow2] = p_slow2;
                p_sum[kProfSlow5] = p_slow5;
                p_sum[kProfMaxRtt] = p_maxrtt;
                p_sum[kProfTorn] = p_torn;
                // relaxed stores only (a release here would write back the
                // XCD's L2 per request and perturb what it measures), the sums
                // next to the request lines (device memory: no PCIe traffic)
                for (int k = 0; k < kProfWords; k++)
                    __hip_atomic_store(&psum[k], p_sum[k], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                const u32x4 mk = {(u32)p_seen, (u32)(p_seen >> 32), (u32)(t_rec - p_seen), q};
                asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1"
                             : : "v"(&rm->mark[blk][0]), "v"(mk) : "memory");
            }
            __hip_atomic_store(&pub->prog[r][blk], qend, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            s_claim = IDLE;
        }
        last = qend;
        if (PROF && act == WORK)
            p_cold = false;
        t_last = __builtin_amdgcn_s_memrealtime();
        if (act == WORK && hot_ticks != ~0ull) {
            const uint64_t gap = t_last - t_claim;
            t_claim = t_last;
            // 3 x the gap when that is within hot_max (gaps <= hot_max / 3),
            // else the fixed window: a ring kept alive by one burst every
            // 200 us still goes cold between them (the idle-poll cost, DESIGN App. A)
            win = 3 * gap <= hot_max_ticks ? (3 * gap < hot_ticks ? hot_ticks : 3 * gap)
                                           : hot_ticks;
        }
        __syncthreads();                     // s_claim reset before anyone polls again
    }
    __threadfence_system();
    __syncthreads();
    if (t == 0)
        __hip_atomic_store(&rm->state[blk].v, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kLdsMaxGroups = 24;

hipError_t launch_burst_server(HubMailbox* mb, HubReqs* rq, HubPub* pub, int groups,
                               uint64_t idle_ticks, uint64_t life_ticks, uint64_t hot_ticks,
                               uint64_t hot_max_ticks, uint32_t max_polls, uint32_t naps,
                               uint32_t opts, bool prof, hipStream_t s)
{
    if (groups < 1 || groups > kHubRings)
        return hipErrorInvalidValue;
    const dim3 grid(kServerBlocks * groups);
    // ONE server block per CU: 96 KiB of dynamic LDS per block (unused; a CU
    // has 160 KiB), so the dispatcher cannot stack up to four of them (117
    // VGPRs, four waves) on a CU whose memory pipeline they then share.  With
    // 8-24 rings, per-call times varied 1.5x from grid to grid without it
    // (DESIGN.md §5).  The reservation leaves 64 KiB of those CUs' LDS to
    // other kernels while the grid lives, so it is made only while the grid
    // covers at most kLdsMaxGroups x 8 CUs (3/4 of the chip); a larger grid
    // stacks.  GCS_SERVER_LDS_KB overrides the size (0: none),
    // GCS_SERVER_LDS_GROUPS the group bound.
    static const size_t lds_kb = [] {
        const char* e = std::getenv("GCS_SERVER_LDS_KB");
        return e ? (size_t)std::strtoul(e, nullptr, 10) : (size_t)96;
    }();
    static const int lds_groups = [] {
        const char* e = std::getenv("GCS_SERVER_LDS_GROUPS");
        return e ? std::atoi(e) : kLdsMaxGroups;
    }();
    const size_t lds = groups <= lds_groups ? lds_kb << 10 : 0;
    // (a 512-thread shape, 64 lanes x 2 chunks per frame, measured no faster:
    // RX frame phase 4.16-4.20 vs 4.01-4.02 us per 64 x 1500 B)
    if (lds > 65536) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_burst_server<32, 3, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_burst_server<32, 3, false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    if (prof)
        hipLaunchKernelGGL((k_burst_server<32, 3, true>), grid, dim3(kBlock), lds, s, mb, rq, pub,
                           idle_ticks, life_ticks, hot_ticks, hot_max_ticks, max_polls, naps,
                           opts);
    else
        hipLaunchKernelGGL((k_burst_server<32, 3, false>), grid, dim3(kBlock), lds, s, mb, rq,
                           pub, idle_ticks, life_ticks, hot_ticks, hot_max_ticks, max_polls, naps,
                           opts);
    return hipGetLastError();
}

// Mixed-size descriptor batch (IMIX, plugin bursts): a block takes 256
// consecutive frames, keeps their validated descriptors in LDS, sorts them
// into three LDS lists by size, and runs each list on a group shape that fits
// it (DescShape: class 0 = frames <= 16*G0*U0 B on G0 lanes x U0 chunks, class
// 1 <= 16*G1*U1 B on G1 x U1, class 2 the rest on G2 x U2 with further
// batches; WM = the TX write-back mode).  Each list is walked by a
// block-uniform loop so every cross-lane step sees its whole group.
// Verdicts / statuses / checks are staged in LDS and leave as one coalesced
// store per block.  Keeping the descriptors in LDS saves each list iteration
// a dependent global load before its frame loads: 4M IMIX frames, verify
// 316 -> 269 us, fill 407 -> 364 us.  Wider shapes (U = 6 or 9 per lane)
// spill at 6 waves per SIMD and lose (kbench imix).
// F = descriptors per block: <= kBlock (one per thread) or R * kBlock (R per
// thread).  256 measured best on C3 (128: verify 319-336 us, 512: 273 us but
// the fill's LDS stage then allows 3 blocks per CU; kbench_imix_F*_blocked.log).
// ORDERED: the class lists keep frame order (wave ballot + prefix count)
// instead of atomicAdd arrival order, so the groups of one list instruction
// work on neighbouring frames: a wave's 64 B-class loads and sector stores
// then cover runs of adjacent frames (two frames per 128 B line) instead of
// frames scattered over the block's whole range.
// K0 / K1: frames per group per list iteration for classes 0 / 1, all their
// loads issued before the first is folded (as k_fixed<4,1,K> does).  Measured
// on C3 (K0 = 3, K1 = 2): verify 278 vs 280 us, fill 388 vs 390 us -- the
// list passes' memory waits are not what bounds it -- so the shipped shape
// keeps K = 1 (profiles/r02/kbench_imix_K.log; other class shapes:
// kbench_imix_shapes2.log).
template <int G0_, int U0_, int G1_, int U1_, int G2_, int U2_, int WM_ = kWM, int F_ = kBlock,
          bool ORDERED_ = true, int K0_ = 1, int K1_ = 1, bool STAGE_ = false, bool NT_ = kNT>
struct DescShape {
    static constexpr bool NT = NT_;
    static constexpr int G0 = G0_, U0 = U0_, G1 = G1_, U1 = U1_, G2 = G2_, U2 = U2_, WM = WM_;
    static constexpr int F = F_;
    static constexpr bool ORDERED = ORDERED_;
    static constexpr int K0 = K0_, K1 = K1_;
    static constexpr bool STAGE = STAGE_;
    static constexpr int R = (F + kBlock - 1) / kBlock;   // descriptors per thread
    static_assert(F <= kBlock || F % kBlock == 0, "whole descriptors per thread");
    static constexpr int T0 = 16 * G0 * U0, T1 = 16 * G1 * U1;
};

// The shipped shapes (A/B in tools/kbench.hip imix).  The fill
// stages each frame's sector 0 in LDS and stores the block's sectors together
// at its end, in frame order, non-temporal: 4M IMIX 390 -> 377-379 us (in the
// epilogues: sc1 390, nt 411; staged: sc1 409, sc0 sc1 410;
// profiles/r02/kbench_imix_stage*.log).  The fill loads its frames with the
// default (temporal) policy, 377-379 -> 371-373 us; the verify keeps NT loads
// (temporal: 319-320 vs 276-279 us; kbench_imix_temporal*.log).
template <bool COMPUTE>
using DescShip = DescShape<4, 1, 16, 3, 32, 3, COMPUTE ? WM_SECTOR_NT : kWM, kBlock, true, 1, 1,
                           COMPUTE, !COMPUTE>;

template <int G, int U, bool COMPUTE, bool LOOP, bool EXT, int WM, int K = 1, bool NT = kNT,
          int NTH = kBlock>
__device__ __forceinline__ void desc_class(uint8_t* __restrict__ frames, uint64_t frames_bytes,
                                           const uint64_t* soff, const uint16_t* slen,
                                           const uint16_t* list, int count, u32 flags,
                                           uint8_t* codes, uint32_t* csums, const Ext& ext,
                                           uint32_t* hashes, uint16_t* queues, uint4* stage)
{
    static_assert(K == 1 || !LOOP, "K > 1 is for frames that fit one batch");
    constexpr int GPB = NTH / G;                       // groups per block (NTH threads)
    const int g = threadIdx.x / G, sub = threadIdx.x & (G - 1);
    auto xframe_of = [&](int t) {
        return EXT ? XFrame{{ext.key[0], ext.key[1], ext.key[2], ext.key[3]},
                            hashes ? hashes + t : nullptr, queues ? queues + t : nullptr, ext.nq,
                            ext.nq_magic, ext.endian, nullptr}
                   : XFrame{};
    };
    for (int base = 0; base < count; base += GPB * K) {   // block-uniform trip count
        uint4 v[K][U];
        int tk[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int idx = base + k * GPB + g;
            const bool active = idx < count;
            const int t = active ? list[idx] : list[0];  // list[0] exists: count > 0
            tk[k] = active ? t : -1;
            const uint64_t o = soff[t];                  // LDS: no dependent global load
            const int nch = active ? (int)((slen[t] + 15u) >> 4) : 0;
            load_first<G, U, true, NT>(frames + o, nch, (int64_t)(frames_bytes - o), sub, v[k]);
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const bool active = tk[k] >= 0;
            const int t = active ? tk[k] : list[0];
            const uint64_t o = soff[t];                  // descriptor validated in phase 0
            uint8_t* f = frames + o;
            frame_body<G, U, COMPUTE, LOOP, true, NT, WM, EXT>(
                v[k], f, f, slen[t], (int64_t)(frames_bytes - o), true, sub, flags, codes + t,
                COMPUTE ? csums + t : nullptr, active, xframe_of(t),
                stage ? reinterpret_cast<uint8_t*>(stage + 4 * t) : nullptr);
        }
    }
}

// End of a descriptor block: the staged sector-0 write-backs, then the block's
// per-frame outputs from LDS as coalesced stores.
template <class S, bool COMPUTE, bool EXT, int NTH = kBlock>
__device__ __forceinline__ void desc_tail(uint8_t* __restrict__ frames, uint64_t frames_bytes,
                                          uint64_t f0, u32 n, const uint64_t* soff,
                                          const uint16_t* slen, const uint8_t* codes,
                                          const uint32_t* csums, const uint32_t* hashes,
                                          const uint16_t* queues, const uint4* stage,
                                          uint8_t* __restrict__ out_code,
                                          uint32_t* __restrict__ out_csum, u32 flags,
                                          const Ext& ext)
{
    constexpr int F = S::F, NR = 4 * ((F + NTH - 1) / NTH);            // stage rounds: 4 chunks per frame
    const int t = threadIdx.x;
    if (COMPUTE && S::STAGE && !(flags & GCS_CF_NO_INPLACE)) {
        // STAGE: the frames' sector-0 write-backs leave together, in frame
        // order, 16 B per lane: four lanes per sector, so adjacent sectors
        // (two packed 64 B frames) are one whole 128 B line of one store
        // instruction.  A chunk goes out under exactly the epilogue's
        // conditions: a status that fills, inside the frame and the buffer.
        bool go[NR];
        uint64_t ob[NR];
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const int q = r * NTH + t, ft = q >> 2, c = q & 3;
            go[r] = false;
            ob[r] = 0;
            if (ft >= F || f0 + ft >= n)
                continue;
            const u32 st = codes[ft];
            const bool wip = st == GCS_TX_OK || st == GCS_TX_IP_ONLY || st == GCS_TX_BAD_TCPLEN ||
                             (EXT && (st == GCS_TX_ICMP_OK || st == GCS_TX_BAD_ICMPLEN));
            if (!wip || 16 * c >= (int)slen[ft])
                continue;
            ob[r] = soff[ft] + 16 * c;
            go[r] = ob[r] + 16 <= frames_bytes;
        }
#pragma unroll
        for (int r = 0; r < NR; r++)
            if (go[r])
                stg16<S::WM>(frames + ob[r], stage[r * NTH + t]);
    }
#pragma unroll
    for (int r = 0; r < (F + NTH - 1) / NTH; r++) {
        const int ft = r * NTH + t;
        const uint64_t i = f0 + ft;
        if (ft < F && i < n) {
            if (out_code)
                out_code[i] = codes[ft];
            if (COMPUTE && out_csum)
                out_csum[i] = csums[ft];
            if (EXT && !COMPUTE) {
                if (ext.hash)
                    ext.hash[i] = hashes[ft];
                if (ext.queue)
                    ext.queue[i] = queues[ft];
            }
        }
    }
}

template <class S, bool COMPUTE, bool EXT>
__device__ __forceinline__ void desc_mixed(uint8_t* __restrict__ frames, uint64_t frames_bytes,
                                           const uint64_t* __restrict__ off,
                                           const uint16_t* __restrict__ lens, u32 n,
                                           uint8_t* __restrict__ out_code,
                                           uint32_t* __restrict__ out_csum, u32 flags,
                                           const Ext& ext, uint32_t blk)
{
    constexpr int F = S::F;
    __shared__ uint64_t soff[F];
    __shared__ uint16_t slen[F];
    __shared__ uint16_t list[3][F];
    __shared__ int cnt[3];
    constexpr int R = S::R, NW = kBlock / 64;
    __shared__ int wcnt[3][R * NW];
    __shared__ uint8_t codes[F];
    __shared__ uint32_t csums[COMPUTE ? F : 1];
    __shared__ uint32_t hashes[EXT && !COMPUTE ? F : 1];
    __shared__ uint16_t queues[EXT && !COMPUTE ? F : 1];
    __shared__ uint4 stage[COMPUTE && S::STAGE ? 4 * F : 1];   // sector 0 of each frame
    const uint64_t f0 = (uint64_t)blk * F;
    const int t = threadIdx.x;
    if (t < 3)
        cnt[t] = 0;
    __syncthreads();
    // phase 0: validate and classify (R descriptors per thread: frames t, t+256, ..)
    int cls[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int ft = r * kBlock + t;
        const uint64_t i = f0 + ft;
        cls[r] = -1;
        if (ft < F && i < n) {
            const uint64_t o = off[i];
            const u32 len = lens[i];
            const bool ok = (o & 15) == 0 && o <= frames_bytes && len <= frames_bytes - o;
            if (!ok) {
                codes[ft] = COMPUTE ? GCS_TX_BAD_DESC : GCS_V_BAD_DESC;
                if (COMPUTE)
                    csums[ft] = 0;
                if (EXT && !COMPUTE) {
                    hashes[ft] = 0;
                    queues[ft] = 0xFFFF;
                }
            } else {
                soff[ft] = o;
                slen[ft] = (uint16_t)len;
                cls[r] = len <= (u32)S::T0 ? 0 : (len <= (u32)S::T1 ? 1 : 2);
                if (!S::ORDERED)
                    list[cls[r]][atomicAdd(&cnt[cls[r]], 1)] = (uint16_t)ft;
            }
        }
    }
    if (S::ORDERED) {
        // per (descriptor round, wave) and class: ballot, then the lane's rank
        // among its class; lists come out in frame order
        const int lane = t & 63, w = t >> 6;
        const uint64_t below = (1ull << lane) - 1;
        int rank[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            rank[r] = 0;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const uint64_t m = __ballot(cls[r] == c);
                if (lane == 0)
                    wcnt[c][r * NW + w] = __popcll(m);
                if (cls[r] == c)
                    rank[r] = __popcll(m & below);
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (cls[r] >= 0) {
                int base = 0;
                for (int k = 0; k < r * NW + w; k++)
                    base += wcnt[cls[r]][k];
                list[cls[r]][base + rank[r]] = (uint16_t)(r * kBlock + t);
            }
        }
        if (t < 3) {
            int tot = 0;
            for (int k = 0; k < R * NW; k++)
                tot += wcnt[t][k];
            cnt[t] = tot;
        }
    }
    __syncthreads();
    {
        const int n0 = cnt[0], n1 = cnt[1], n2 = cnt[2];
        uint32_t* hl = EXT && !COMPUTE ? hashes : nullptr;
        uint16_t* ql = EXT && !COMPUTE ? queues : nullptr;
        uint4* stg = COMPUTE && S::STAGE ? stage : nullptr;
        if (n0) desc_class<S::G0, S::U0, COMPUTE, false, EXT, S::WM, S::K0, S::NT>(frames, frames_bytes, soff, slen, list[0], n0, flags, codes, csums, ext, hl, ql, stg);
        if (n1) desc_class<S::G1, S::U1, COMPUTE, false, EXT, S::WM, S::K1, S::NT>(frames, frames_bytes, soff, slen, list[1], n1, flags, codes, csums, ext, hl, ql, stg);
        if (n2) desc_class<S::G2, S::U2, COMPUTE, true, EXT, S::WM, 1, S::NT>(frames, frames_bytes, soff, slen, list[2], n2, flags, codes, csums, ext, hl, ql, stg);
    }
    __syncthreads();
    desc_tail<S, COMPUTE, EXT>(frames, frames_bytes, f0, n, soff, slen, codes, csums, hashes, queues,
                               stage, out_code, out_csum, flags, ext);
}

template <class S, bool COMPUTE, bool XCD, int OCC = 1>
__global__ void __launch_bounds__(kBlock, OCC)
k_desc_mixed(uint8_t* __restrict__ frames, uint64_t frames_bytes,
             const uint64_t* __restrict__ off, const uint16_t* __restrict__ lens, u32 n,
             uint8_t* __restrict__ out_code, uint32_t* __restrict__ out_csum, u32 flags)
{
    desc_mixed<S, COMPUTE, false>(frames, frames_bytes, off, lens, n, out_code, out_csum, flags,
                                  Ext{}, XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x);
}

template <class S, bool COMPUTE, bool XCD, int OCC = 1>
__global__ void __launch_bounds__(kBlock, OCC)
k_desc_mixed_x(uint8_t* __restrict__ frames, uint64_t frames_bytes,
               const uint64_t* __restrict__ off, const uint16_t* __restrict__ lens, u32 n,
               uint8_t* __restrict__ out_code, uint32_t* __restrict__ out_csum, u32 flags,
               Ext ext)
{
    desc_mixed<S, COMPUTE, true>(frames, frames_bytes, off, lens, n, out_code, out_csum, flags,
                                 ext, XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x);
}

// ---------------------------------------------------------------------------
// Packed descriptor batches as a prefix-sum stream (IMIX, C3).
//
// A frame's TCP fold over [ts, te) is a difference of two prefix sums of the
// block region's 16-bit words: sum[a, b) = Q(b) - Q(a), exact in u32 because
// one frame's words sum to < 2^32 (len < 64 KiB) and wrap-around cancels in
// the difference.  So the block's packed region is read ONCE, as four plain
// streams (one per wave, 1 KiB per load instruction, no per-frame group
// shapes, no class passes): each lane folds its chunk to one word sum, a DPP
// wave scan turns the sums into chunk prefixes, and the lanes holding a
// frame's first chunks or its chunk NH or its last chunk park what the
// per-frame step needs in LDS -- chunks 0..NH-1 (the headers; for TX the
// sector that is written back) and Q(len) - Q(16 NH), the frame's words past
// the stash, accumulated by two LDS adds.  Then one lane per frame parses its
// headers from LDS, folds the stashed chunks with the group kernels' exact
// masks and adds the words [16 NH, te) from the stash-less tail, then runs
// the shared epilogue (verdict, or fill into the staged sector).  Per-frame
// results are identical as integers to the group kernels' (the same words,
// the same u32 sums).
//
// A block streams when its frames are valid, non-empty, in offset order,
// chunk-disjoint with gaps <= 64 B, the region (<= RMAX chunks) ends inside
// the buffer, and every frame is "fast": ihl <= 8 (TX, NH = 4: IP header,
// doff byte and tcph->check inside chunks 0..3) or ihl == 5 (RX, NH = 3), and
// te <= 16 NH or te == len (the segment ends at the frame's end, as every
// frame mTCP builds).  Any other block has written nothing and runs its frames
// one wave per frame instead (desc_fallback_block).  Keeping desc_mixed's
// class passes (and their 80 VGPRs) out of this kernel is what lets it run 8
// waves per SIMD (round 4; before: 6 waves for the fill, 7 for the verify).  Reference
// layout: PSIO's packed chunk (pslib.c:132-156, ps.h:181-213).
template <int U_, int RMAX_, int OCC_, int NH_, int FG_ = 64, int FU_ = 1>
struct StreamShape {
    static constexpr int FG = FG_;        // a non-streaming block: lanes per frame ...
    static constexpr int FU = FU_;        // ... and chunks per lane per trip
    static constexpr int U = U_;          // chunks per lane per trip (64 * U per wave)
    static constexpr int RMAX = RMAX_;    // region chunks a streaming block may span
    static constexpr int OCC = OCC_;      // waves per SIMD asked of the compiler
    static constexpr int NH = NH_;        // header chunks stashed per frame
    static_assert(RMAX % 64 == 0 && RMAX <= 65536, "start chunks fit 16 bits");
    static_assert(NH == 3 || NH == 4, "stash: chunks 0..2 (RX, ihl = 5) or 0..3 (TX sector)");
};

// A block of a descriptor launch that k_desc_stream does not stream runs its
// frames here, inside the same kernel: one wave per frame, 64 lanes x 1 chunk
// per trip until the frame ends (k_fixed<64,1>'s shape, and its exact
// per-frame results).  It is the lightest per-frame shape there is (desc_mixed's
// class passes cost 80 VGPRs, a 32 x 3 loop 87-96), so it fits the stream
// path's 64 VGPRs and the kernel keeps 8 waves per SIMD.  Round 4 first put
// these blocks on a list for a second kernel: its launch alone cost 6 us on
// every batch, and the list's head serialised an all-fallback batch (1M x
// 1500 B: 22 ms).  Rare in mTCP traffic: misordered or sparse descriptors,
// regions over RMAX (256 frames of ~1500 B), IP options, frames padded past a
// segment that ends beyond byte 48/64.
template <int G, int U, bool COMPUTE>
__device__ __forceinline__ void
desc_fallback_block(uint8_t* __restrict__ frames, uint64_t frames_bytes,
                    const uint64_t* __restrict__ off, const uint16_t* __restrict__ lens,
                    uint64_t f0, int nf, uint8_t* __restrict__ out_code,
                    uint32_t* __restrict__ out_csum, u32 flags)
{
    const int sub = threadIdx.x & (G - 1);
    for (int k = threadIdx.x / G; k < nf; k += kBlock / G) {     // group-uniform
        const uint64_t i = f0 + k;
        const uint64_t o = off[i];
        const u32 len = lens[i];
        const bool ok = (o & 15) == 0 && o <= frames_bytes && len <= frames_bytes - o;
        uint8_t* f = frames + (ok ? o : 0);
        do_frame<G, U, COMPUTE, true, true, kNT, WM_SECTOR_SC1>(
            f, len, ok ? (int64_t)(frames_bytes - o) : 0, ok, sub, flags,
            // RX: the verdict array is never null (every C-ABI entry checks it),
            // so the store is a global one; a TX status array may be absent
            COMPUTE ? (out_code ? out_code + i : nullptr) : out_code + i,
            out_csum ? out_csum + i : nullptr);
    }
}

template <class T, bool COMPUTE, int WM, bool XCD>
__global__ void __launch_bounds__(kBlock, T::OCC)
k_desc_stream(uint8_t* __restrict__ frames, uint64_t frames_bytes,
              const uint64_t* __restrict__ off, const uint16_t* __restrict__ lens, u32 n,
              uint8_t* __restrict__ out_code, uint32_t* __restrict__ out_csum, u32 flags)
{
    constexpr int F = kBlock, NW = kBlock / 64, RW = T::RMAX / 64, U = T::U, NH = T::NH;
    constexpr int HB = 16 * NH;            // header bytes stashed per frame
    static_assert(!COMPUTE || NH == 4, "TX stages sector 0 (chunks 0..3) in hdr");
    __shared__ uint4 hdr[NH * F];          // chunks 0..NH-1 per frame; TX: the staged sector 0
    __shared__ u32 meta[F];                // pass-relative start chunk << 16 | len
    __shared__ u32 tail[F];                // wave-local Q(len) - Q(HB): words [HB, len)
    __shared__ uint64_t bm[RW];            // bit c: a frame starts at region chunk c
    __shared__ uint16_t rbase[RW];         // frames starting before chunk 64 * row
    __shared__ u32 wtot[NW];
    __shared__ uint8_t codes[F];           // TX statuses (the write-back's test)
    __shared__ u32 nchunks_s, pbase_s;     // the pass region's chunks; its first, in the block's

    const uint32_t blk = XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint64_t f0 = (uint64_t)blk * F;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int nf = (int)((n - f0) < (uint64_t)F ? (n - f0) : (uint64_t)F);

    // A long block region is streamed in passes of at most RMAX chunks, one
    // workgroup per pass (blockIdx.y; straight-line code: a pass loop around
    // the stream made the compiler spill 23-38 VGPRs).  Pass p's frames are
    // [p0, p1): greedily, the frames from p0 whose end lies within RMAX chunks
    // of frame p0's start (in order, so contiguous).  An IMIX block is one
    // pass (~91 KiB), and its pass-1.. workgroups leave after two loads; 256
    // packed 1500 B frames are three passes.
    const int pass = blockIdx.y;
    const uint64_t r0 = off[f0];
    if (pass > 0) {
        const uint64_t ol = off[f0 + nf - 1];
        if (ol >= r0 && ol - r0 + lens[f0 + nf - 1] <= 16ull * T::RMAX)
            return;                        // block-uniform: a one-pass region
    }

    // phase 0: validate; streamability (in order, chunk-disjoint, gaps <= 64 B,
    // the last frame's chunks inside the buffer); each frame's place in the
    // block's region (chunks from frame 0's start): its first chunk, its end,
    // the next frame's first chunk
    u32 len = 0, start = 0, snext = 0;
    bool sok = true;
    if (t < nf) {
        const uint64_t o = off[f0 + t];
        len = lens[f0 + t];
        sok = (o & 15) == 0 && o <= frames_bytes && len <= frames_bytes - o && len > 0 &&
              o >= r0 && o - r0 < (1ull << 35);
        const uint64_t e = o + 16ull * ((len + 15) >> 4);
        start = (u32)((o - r0) >> 4);
        if (sok && t + 1 < nf) {
            const uint64_t on = off[f0 + t + 1];
            sok = on >= e && on - e <= 64;
            snext = (u32)((on - r0) >> 4);
        } else if (sok) {
            sok = e <= frames_bytes;
        }
    }
    const u32 nch = (len + 15) >> 4, end = start + nch;
    for (int r = t; r < RW; r += kBlock)
        bm[r] = 0;
    if (!__syncthreads_and(sok)) {         // block-uniform: nothing written
        if (pass == 0)
            desc_fallback_block<T::FG, T::FU, COMPUTE>(frames, frames_bytes, off, lens, f0, nf,
                                                       out_code, out_csum, flags);
        return;
    }
    int p0 = 0, p1 = 0;
    u32 pb = 0;
    for (int k = 0; k <= pass; k++) {      // block-uniform
        p0 = p1;
        if (p0 >= nf)
            return;                        // no pass p here
        if (t == p0)
            pbase_s = start;
        __syncthreads();
        pb = pbase_s;
        p1 = p0 + __syncthreads_count(t >= p0 && t < nf && end - pb <= (u32)T::RMAX);
    }
    const bool in = t >= p0 && t < p1;
    // frames past the last pass a launch has (PMAX) go to the per-frame path
    const int fb_hi = pass + 1 == (int)gridDim.y ? nf : p1;
    const u32 rs = start - pb;         // pass-relative first chunk

    // phase 1: the pass region's first-chunk bitmap, per-frame metadata,
    // and per 64-chunk row the frame owning its first chunk, minus one
    // for the mbcnt below (frame t owns the rows r with rs_t < 64 r <=
    // rs_t+1; rbase[0] = p0: block frame indices throughout)
    if (in) {
        meta[t] = rs << 16 | len;
        tail[t] = 0;
#pragma unroll
        for (int k = 0; k < NH; k++)
            if ((u32)k >= nch)
                hdr[NH * t + k] = make_uint4(0, 0, 0, 0);
        atomicOr((unsigned long long*)&bm[rs >> 6], 1ull << (rs & 63));
        const bool last = t == p1 - 1;
        const u32 rhi = last ? ((end - pb + 63) >> 6) - 1 : (snext - pb) >> 6;
        for (u32 r = (rs >> 6) + 1; r <= rhi; r++)
            rbase[r] = (uint16_t)(t + 1);
        if (last)
            nchunks_s = end - pb;
    }
    if (t == p0)
        rbase[0] = (uint16_t)p0;
    __syncthreads();

    // phase 2: wave w streams chunks [w*QW, (w+1)*QW) of the pass region
    const u32 NCH = nchunks_s;
    const u32 QW = ((NCH + 4 * 64 - 1) / (4 * 64)) * 64;
    uint8_t* const reg = frames + r0 + 16ull * pb;
    {
        const u32 lo = w * QW, hi = (lo + QW < NCH) ? lo + QW : NCH;
        u32 run = 0;
        for (u32 base = lo; base < hi; base += 64 * U) {
            uint4 v[U];
#pragma unroll
            for (int j = 0; j < U; j++) {
                const u32 c = base + 64 * j + lane;
                v[j] = c < hi ? ldg16<true>(reg + 16ull * c) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < U; j++) {
                const u32 row = (base >> 6) + j;
                if (64 * row >= hi)           // wave-uniform
                    break;
                const u32 c = 64 * row + lane;
                const u32 s4 = hsum4(v[j]);
                const u32 incl = wave_incl_scan(s4);
                const u32 excl = run + incl - s4;
                run += (u32)__builtin_amdgcn_readlane((int)incl, 63);
                const uint64_t bits = bm[row];
                const u32 below = __builtin_amdgcn_mbcnt_hi((u32)(bits >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((u32)bits, 0u));
                const int f = (int)rbase[row] + (int)below + (int)((bits >> lane) & 1u) - 1;
                if (c < hi) {
                    const u32 m = meta[f], fl = m & 0xFFFFu;
                    const u32 k = c - (m >> 16), fn = (fl + 15) >> 4;
                    if (k < (u32)NH && k < fn)
                        hdr[NH * f + k] = v[j];
                    if (fn > (u32)NH) {       // words [HB, len): Q(len) - Q(HB)
                        if (k == (u32)NH)
                            __hip_atomic_fetch_add(&tail[f], 0u - excl, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (k + 1 == fn)
                            __hip_atomic_fetch_add(&tail[f],
                                                   excl + chunk_prefix_sum(v[j], (int)(fl - 16 * k)),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
        }
        if (lane == 0)
            wtot[w] = run;
    }
    __syncthreads();

    // phase 3: one lane per frame of the pass
    const int tf = in ? t : p0;
    const uint4 h4[4] = {hdr[NH * tf], hdr[NH * tf + 1], hdr[NH * tf + 2],
                         NH == 4 ? hdr[NH * tf + 3] : make_uint4(0, 0, 0, 0)};
    Hdr h;
    h.d3 = h4[0].w;
    h.d4 = h4[1].x;
    h.d5 = h4[1].y;
    const int ihl = (int)((h.d3 >> 16) & 15u);
    const int ts = 14 + 4 * ihl;
    const int te = 14 + (int)bswap16(h.d4 & 0xFFFFu);
    // NH = 3 (RX): doff (byte ts + 12) must lie in chunk 2: ihl == 5
    const bool fast = !in || ((NH == 4 ? ihl <= 8 : ihl == 5) && (te <= HB || te == (int)len));
    if (!__syncthreads_and(fast)) {    // block-uniform: this pass wrote nothing yet
        desc_fallback_block<T::FG, T::FU, COMPUTE>(frames, frames_bytes, off, lens, f0 + p0,
                                                   fb_hi - p0, out_code, out_csum, flags);
        return;
    }
    // wave-uniform: every frame of the wave has ihl == 5, so the stash's
    // word masks are constants (masks5, as the group kernels); and when
    // every one also has te >= HB, no segment end lies in the stash
    const bool all5 = NH == 3 || __all(!in || ihl == 5);
    const bool endh = __all(!in || te >= HB);
    if (in) {
        Acc a = {0u, 0u, 0u};
        if (all5 && endh) {
#pragma unroll
            for (int c = 0; c < NH; c++)
                accum_fast5<COMPUTE, true>(h4[c], c, HB, masks5<COMPUTE>(c), a);
        } else if (all5) {
#pragma unroll
            for (int c = 0; c < NH; c++)
                accum_fast5<COMPUTE, true>(h4[c], c, te < HB ? te : HB, masks5<COMPUTE>(c), a);
        } else if constexpr (NH == 4) {
#pragma unroll
            for (int j = 0; j < NH; j++)
                accum_chunk<COMPUTE>(h4[j], 16 * j, ts, te < HB ? te : HB, a);
        }
        if (te > HB) {
            // Q is wave-local: add the chunk's wave base at both ends
            auto wbase = [&](u32 c) {
                const u32 q = c / QW;
                u32 b = 0;
#pragma unroll
                for (int k = 0; k < NW - 1; k++)
                    b += (u32)k < q ? wtot[k] : 0u;
                return b;
            };
            a.tcp += tail[t] + wbase(rs + nch - 1) - wbase(rs + NH);
        }
        const uint64_t o = r0 + 16ull * (pb + rs);
        epilogue<1, 4, COMPUTE, WM, false>(
            h, a, frames + o, len, (int64_t)(frames_bytes - o), true, 0, flags,
            COMPUTE ? codes + t : out_code + f0 + t,        // RX: never null (C ABI)
            COMPUTE && out_csum ? out_csum + f0 + t : nullptr, true, h4, XFrame{},
            COMPUTE ? reinterpret_cast<uint8_t*>(hdr + 4 * t) : nullptr);
    }
    if constexpr (COMPUTE) {
        // the staged sectors leave together, in frame order, 16 B per
        // lane: four lanes per sector, so two packed 64 B frames are one
        // 128 B line of one store instruction.  A chunk goes out under
        // exactly the epilogue's conditions: a status that fills, inside
        // the frame (the region ends inside the buffer: phase 0).
        __syncthreads();
        if (!(flags & GCS_CF_NO_INPLACE)) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int q = r * kBlock + t, ft = q >> 2, c = q & 3;
                if (ft < p0 || ft >= p1)
                    continue;
                const u32 st = codes[ft], m = meta[ft];
                const bool wip = st == GCS_TX_OK || st == GCS_TX_IP_ONLY || st == GCS_TX_BAD_TCPLEN;
                if (wip && (u32)(16 * c) < (m & 0xFFFFu))
                    stg16<WM>(reg + 16ull * ((m >> 16) + c), hdr[q]);
            }
        }
        if (out_code && in)
            out_code[f0 + t] = codes[t];
    }
    if (fb_hi > p1) {
        __syncthreads();                   // every wave done with the pass
        desc_fallback_block<T::FG, T::FU, COMPUTE>(frames, frames_bytes, off, lens, f0 + p1,
                                                   fb_hi - p1, out_code, out_csum, flags);
    }
}

// ---------------------------------------------------------------------------
// TX payload copy + fill (SendTCPPacket, tcp_out.c:316-333:
// memcpy of the payload behind the TCP header, then TCPCalcChecksum over
// header + payload, then IPOutput's ip_fast_csum, ip_out.c:172).  One pass:
// the payload is read once from the source, folded while in registers and
// written once into the frame; only the header chunks are read from the frame.
// A frame is copied when its headers describe a complete TCP segment (the
// conditions under which the fill returns GCS_TX_OK); any other frame gets the
// plain fill.  Payload bytes [hl, te) of the frame come from src + pay_off[i]
// (any alignment: unaligned 16 B loads), hl = 14 + 4*ihl + 4*doff, te = 14 +
// tot_len; bytes past te are left as they are.

typedef u32x4 u32x4_u __attribute__((aligned(1)));

__device__ __forceinline__ uint4 ldg16u(const uint8_t* p)
{
    const u32x4 r = *reinterpret_cast<const u32x4_u*>(p);
    return make_uint4(r.x, r.y, r.z, r.w);
}

__device__ __forceinline__ u32 chunk_byte(const uint4& v, int k)
{
    return (pick(v, k >> 2) >> (8 * (k & 3))) & 0xFFu;
}

// Chunk byte j of the result = byte j - k of v (0 below k), k in [0, 16].
__device__ __forceinline__ uint4 bytes_up(uint4 v, int k)
{
    const uint64_t lo = v.x | ((uint64_t)v.y << 32), hi = v.z | ((uint64_t)v.w << 32);
    const int sh = 8 * k;
    uint64_t nlo, nhi;
    if (sh == 0) {
        nlo = lo;
        nhi = hi;
    } else if (sh < 64) {
        nlo = lo << sh;
        nhi = (hi << sh) | (lo >> (64 - sh));
    } else if (sh < 128) {
        nlo = 0;
        nhi = lo << (sh - 64);
    } else {
        nlo = nhi = 0;
    }
    return make_uint4((u32)nlo, (u32)(nlo >> 32), (u32)nhi, (u32)(nhi >> 32));
}

// Bytes [a, b) of a chunk set, 0 <= a <= b <= 16.
__device__ __forceinline__ uint4 byte_mask(int a, int b)
{
    return make_uint4(low_mask(b) & ~low_mask(a), low_mask(b - 4) & ~low_mask(a - 4),
                      low_mask(b - 8) & ~low_mask(a - 8), low_mask(b - 12) & ~low_mask(a - 12));
}

// x where m is clear, y where it is set
__device__ __forceinline__ uint4 blend(uint4 x, uint4 y, uint4 m)
{
    return make_uint4((x.x & ~m.x) | (y.x & m.x), (x.y & ~m.y) | (y.y & m.y),
                      (x.z & ~m.z) | (y.z & m.z), (x.w & ~m.w) | (y.w & m.w));
}

// Chunk assembly plans (k_copy_fill, k_gro): which loads a destination chunk
// needs and how they combine.  All loads of a batch are issued before any is
// consumed, so a wave waits once per batch.
enum { AS_ZERO = 0, AS_FRAME, AS_ONE, AS_UP, AS_TAIL, AS_TWO, AS_BYTES };

// k_copy_fill: the plan and loads of one batch of destination chunks (base +
// j*G + sub) for headers ending at hl and a segment ending at te; payload byte
// p of the frame comes from ps[p - hl], with src_room readable bytes from ps.
// Every source load stays inside [ps, ps + src_room): AS_ONE needs
// cb - hl + 16 <= te - hl, which the caller has checked against src_room.
// Frame chunks (headers, bytes past te, the plain fill) are loaded from f,
// except batch 0's chunk `sub` < hv_lanes, already loaded as hv.
template <int G, int U>
__device__ __forceinline__ void cf_issue(int base, int sub, int nchunks, bool copy, int hl, int te,
                                         const uint8_t* ps, int64_t src_room,
                                         const uint8_t* f, int64_t avail, const uint4& hv,
                                         int hv_lanes, uint4 (&fr)[U], uint4 (&pv)[U],
                                         int (&plan)[U])
{
    const uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < U; j++) {
        const int c = base + j * G + sub;
        const int cb = 16 * c;
        int pl = AS_ZERO;
        fr[j] = z;
        pv[j] = z;
        if (c < nchunks) {
            if (!copy || cb + 16 <= hl || cb >= te) {
                pl = AS_FRAME;                           // header / past the segment
            } else if (cb >= hl && cb + 16 <= te) {
                pl = AS_ONE;                             // payload only
                pv[j] = ldg16u(ps + (cb - hl));
            } else if (cb < hl && cb + 16 <= te && src_room >= 16) {
                pl = AS_UP;                              // headers, then the payload start
                pv[j] = ldg16u(ps);
            } else if (cb >= hl && src_room >= (int64_t)(cb - hl) + 16) {
                pl = AS_TAIL;                            // the payload end, then frame bytes
                pv[j] = ldg16u(ps + (cb - hl));
            } else {
                pl = AS_BYTES;                           // tiny payload / source end
            }
            if (pl != AS_ONE) {
                if (base == 0 && j == 0 && sub < hv_lanes)
                    fr[j] = hv;
                else
                    fr[j] = load_chunk<true, false>(f + cb, avail - cb);
            }
        }
        plan[j] = pl;
    }
}

// Assemble destination chunks from a batch's loads (cf_issue's plans), in
// place: x[j] becomes chunk base + j*G + sub of the filled frame.
template <int G, int U>
__device__ __forceinline__ void cf_assemble(int base, int sub, int hl, int te, const uint8_t* ps,
                                            uint4 (&x)[U], const uint4 (&pv)[U],
                                            const int (&plan)[U])
{
    const uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < U; j++) {
        const int cb = 16 * (base + j * G + sub);
        switch (plan[j]) {
        case AS_FRAME: break;
        case AS_ONE: x[j] = pv[j]; break;
        case AS_UP: x[j] = blend(x[j], bytes_up(pv[j], hl - cb), byte_mask(hl - cb, 16)); break;
        case AS_TAIL: x[j] = blend(x[j], pv[j], byte_mask(0, te - cb)); break;
        case AS_BYTES: {
            u32 w[4] = {0u, 0u, 0u, 0u};
            for (int k = 0; k < 16; k++) {
                const int p = cb + k;
                const u32 b = (p >= hl && p < te) ? (u32)ps[p - hl] : chunk_byte(x[j], k);
                w[k >> 2] |= b << (8 * (k & 3));
            }
            x[j] = make_uint4(w[0], w[1], w[2], w[3]);
            break;
        }
        default: x[j] = z; break;
        }
    }
}

// Frame chunks read up front: 0..5, enough to parse (the doff byte of the
// longest IP header, ts + 12 <= 86, lies in chunk 5).  Further frame chunks are
// read only where the plan keeps frame bytes; the rest of the frame's old
// contents is overwritten by the payload (PMC: 2.2 -> 1.6 GB read per 1M x
// 1500 B).  Speculation: mTCP's data segments carry ihl 5 and doff 8
// (ip_out.c:143, tcp_out.c:22-61 with timestamps), so headers end at 66 and
// tot_len covers the frame; batch 0's payload loads are issued for that layout
// together with the header loads and re-issued only if the parsed headers
// differ -- one memory round trip per frame instead of two.
// Registers: batch 0 (the frame's first G*U chunks, the whole frame up to
// 16*G*U bytes) is assembled IN the registers its loads landed in, folded
// there and handed to the epilogue as it is; no copy of it is kept across a
// batch loop.  Frames longer than one batch build their later batches first
// (no speculation for them), then batch 0.  ihl = 5 waves fold with the
// constant-mask path (accum_fast5).  1M x 1500 B: 706-711 -> 576-624 us
// against the earlier form (88 VGPRs, first batch copied; kbench copy,
// profiles/r02/kbench_copy_fill2*.log).
template <int G, int U, int OCC = 1, int CWM = WM_SECTOR>
__global__ void __launch_bounds__(kBlock, OCC)
k_copy_fill(uint8_t* __restrict__ frames, uint64_t frames_bytes,
             const uint64_t* __restrict__ off, const uint16_t* __restrict__ lens,
             const uint8_t* __restrict__ src, uint64_t src_bytes,
             const uint64_t* __restrict__ src_off, u32 n, uint8_t* __restrict__ out_code,
             uint32_t* __restrict__ out_csum, u32 flags)
{
    static_assert(G >= 16, "the first G chunks must hold the longest header (134 B)");
    constexpr int kHdrLanes = 6, kSpecHl = 66, CAP = G * U, FPB = kBlock / G;
    const int sub = threadIdx.x & (G - 1);
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x);
    const uint64_t i = (uint64_t)blk * FPB + threadIdx.x / G;
    if (i >= n)
        return;
    const uint64_t o = off[i];
    const u32 len = lens[i];
    const uint64_t po_any = src_off[i];
    const bool ok = (o & 15) == 0 && o <= frames_bytes && len <= frames_bytes - o;
    uint8_t* f = frames + (ok ? o : 0);
    const int64_t avail = ok ? (int64_t)(frames_bytes - o) : 0;
    const int nchunks = ok ? (int)((len + 15) >> 4) : 0;
    const uint4 hv = (sub < kHdrLanes && sub < nchunks)
                         ? load_chunk<true, false>(f + 16 * sub, avail - 16 * sub)
                         : make_uint4(0, 0, 0, 0);
    const bool single = nchunks <= CAP;                // group-uniform
    const int te_g = (int)len;
    const bool copy_g = single && ok && te_g >= kSpecHl && po_any <= src_bytes &&
                        (uint64_t)(te_g - kSpecHl) <= src_bytes - po_any;
    uint4 x[U], pv[U];
    int plan[U];
    if (single)
        cf_issue<G, U>(0, sub, nchunks, copy_g, kSpecHl, te_g, src + (copy_g ? po_any : 0),
                       copy_g ? (int64_t)(src_bytes - po_any) : 0, f, avail, hv, kHdrLanes, x, pv,
                       plan);
    Hdr h;
    h.d3 = group_bcast<G, 0>(hv.w);
    h.d4 = group_bcast<G, 1>(hv.x);
    h.d5 = group_bcast<G, 1>(hv.y);
    const int ihl = (int)((h.d3 >> 16) & 15u);
    const int ts = 14 + 4 * ihl;
    const int tot = (int)bswap16(h.d4 & 0xFFFFu);
    const int te = 14 + tot;
    const int pd = ts + 12;
    const u32 db = group_sum<G>(sub == (pd >> 4) ? chunk_byte(hv, pd & 15) : 0u);
    const int doff = (int)(db >> 4);
    const int hl = ts + 4 * doff;
    const bool copy = ok && len >= 34 && (h.d3 & 0xFFFFu) == 0x0008u && ihl >= 5 &&
                      (h.d5 >> 24) == 6 && doff >= 5 && tot >= 4 * (ihl + doff) &&
                      te <= (int)len;
    const uint64_t plen = copy ? (uint64_t)(te - hl) : 0;
    const uint64_t po = copy ? po_any : 0;
    if (copy && !(po <= src_bytes && plen <= src_bytes - po)) {   // group-uniform
        if (sub == 0) {
            if (out_code)
                out_code[i] = GCS_TX_BAD_DESC;
            if (out_csum)
                out_csum[i] = 0;
        }
        return;
    }
    const uint8_t* ps = src + po;
    const int64_t src_room = copy ? (int64_t)(src_bytes - po) : 0;
    Acc a = {0u, 0u, 0u};
    // later batches of a frame longer than CAP chunks, last first
    for (int base = CAP * ((nchunks - 1) / CAP); base > 0; base -= CAP) {   // group-uniform
        cf_issue<G, U>(base, sub, nchunks, copy, hl, te, ps, src_room, f, avail, hv, kHdrLanes, x,
                       pv, plan);
        cf_assemble<G, U>(base, sub, hl, te, ps, x, pv, plan);
#pragma unroll
        for (int j = 0; j < U; j++)
            accum_chunk<true>(x[j], 16 * (base + j * G + sub), ts, te, a);
        if (copy) {
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int c = base + j * G + sub, cb = 16 * c;
                if (c >= nchunks || cb >= te)
                    continue;
                if (cb + 16 <= avail) {
                    stg16<CWM>(f + cb, x[j]);
                } else {
                    for (int k = 0; k < 16 && cb + k < te; k++)
                        f[cb + k] = (uint8_t)chunk_byte(x[j], k);
                }
            }
        }
    }
    // batch 0: loaded above unless the frame is long or the guess was wrong
    if (!single || copy != copy_g || (copy && (hl != kSpecHl || te != te_g)))
        cf_issue<G, U>(0, sub, nchunks, copy, hl, te, ps, src_room, f, avail, hv, kHdrLanes, x, pv,
                       plan);
    cf_assemble<G, U>(0, sub, hl, te, ps, x, pv, plan);
    if (__all(ts == 34)) {                            // wave-uniform: ihl == 5 everywhere
        const Mask5 m = masks5<true>(sub);
        accum_fast5<true, true>(x[0], sub, te, m, a);
#pragma unroll
        for (int j = 1; j < U; j++)
            accum_fast5<true, false>(x[j], j * G + sub, te, m, a);
    } else {
#pragma unroll
        for (int j = 0; j < U; j++)
            accum_chunk<true>(x[j], 16 * (j * G + sub), ts, te, a);
    }
    if (copy) {
        // chunks 8.. go out now; the first line (with the check fields) in the epilogue
#pragma unroll
        for (int j = 0; j < U; j++) {
            const int c = j * G + sub, cb = 16 * c;
            if (c < 8 || c >= nchunks || cb >= te)
                continue;
            if (cb + 16 <= avail) {
                stg16<CWM>(f + cb, x[j]);
            } else {
                for (int k = 0; k < 16 && cb + k < te; k++)
                    f[cb + k] = (uint8_t)chunk_byte(x[j], k);
            }
        }
    }
    epilogue<G, U, true, WM_LINE_SC1>(h, a, f, len, avail, ok, sub, flags & ~GCS_CF_NO_INPLACE,
                                      out_code ? out_code + i : nullptr,
                                      out_csum ? out_csum + i : nullptr, true, x);
}

// ---------------------------------------------------------------------------
// Software LRO (the merge a NIC's LRO does for mTCP's
// ENABLELRO builds, dpdk_module.c:855-881).  Rules: oracle/csum_ref.h
// ref_gro_batch.  One block per window of <= kGroW frames:
//   A  thread t parses frame t's first 96 B into LDS;
//   B  thread t decides whether frame t continues frame t-1;
//   C  each chain's first thread cuts its chain into runs (length limit);
//      a block scan numbers the runs and gives their output offsets;
//   D  each wave builds whole runs: a single frame is copied as it is, a
//      longer run is assembled destination-chunk by destination-chunk (head
//      headers with tot_len / PSH patched, then the members' payloads through
//      unaligned 16 B loads), folded on the way (accum_chunk) and written,
//      with the checks filled by the TX epilogue -- the merged frame is read
//      once and written once.

constexpr int kGroW = 256;      // frames per window (one per thread)
constexpr int kGroWideThreads = 1024;   // block of the FLAT form for windows > 64
constexpr int kGroHdr = 96;     // header bytes kept per frame (14 + 20 + 60 + 2)

__device__ __forceinline__ u32 lds_be16(const uint8_t* p) { return ((u32)p[0] << 8) | p[1]; }
__device__ __forceinline__ u32 lds_be32(const uint8_t* p)
{
    return ((u32)p[0] << 24) | ((u32)p[1] << 16) | ((u32)p[2] << 8) | p[3];
}

// gro_continues of oracle/csum_ref.c over two frames' header bytes
__device__ bool gro_cont(const uint8_t* p, const uint8_t* c, int pp, int pc)
{
    if (pp <= 0 || pc <= 0)
        return false;
    if (p[15] != c[15] || lds_be16(p + 20) != lds_be16(c + 20) || (lds_be16(p + 20) & 0x3FFFu) ||
        p[22] != c[22])
        return false;
    for (int k = 26; k < 34; k++)
        if (p[k] != c[k])
            return false;
    const u32 idp = lds_be16(p + 18), idc = lds_be16(c + 18);
    if (idc != idp && idc != ((idp + 1) & 0xFFFFu))
        return false;
    for (int k = 34; k < 38; k++)
        if (p[k] != c[k])
            return false;
    for (int k = 42; k < 46; k++)
        if (p[k] != c[k])
            return false;
    if (c[46] != p[46] || (p[46] & 0x0F) || lds_be16(p + 48) != lds_be16(c + 48) ||
        lds_be16(p + 52) || lds_be16(c + 52))
        return false;
    if (p[47] != 0x10 || (c[47] != 0x10 && c[47] != 0x18))
        return false;
    const int hl = 34 + 4 * (p[46] >> 4);
    for (int k = 54; k < hl; k++)
        if (p[k] != c[k])
            return false;
    return lds_be32(c + 38) == lds_be32(p + 38) + (u32)pp;
}

// gro_cont on 32-bit LDS words (rows are 16 B-aligned): the same tests as
// gro_cont, ~30 dword reads instead of ~80 byte reads per pair.
__device__ bool gro_cont32(const uint8_t* p, const uint8_t* c, int pp, int pc)
{
    if (pp <= 0 || pc <= 0)
        return false;
    const u32* P = reinterpret_cast<const u32*>(p);
    const u32* C = reinterpret_cast<const u32*>(c);
    if ((P[3] ^ C[3]) & 0xFF000000u)                   // byte 15 (tos)
        return false;
    if (((P[5] ^ C[5]) & 0x00FFFFFFu) || (P[5] & 0xFF3Fu))   // bytes 20-22; frag bits
        return false;
    if (((P[6] ^ C[6]) & 0xFFFF0000u) || P[7] != C[7] || P[8] != C[8])   // 26..35
        return false;
    const u32 idp = bswap16(P[4] >> 16), idc = bswap16(C[4] >> 16);
    if (idc != idp && idc != ((idp + 1) & 0xFFFFu))
        return false;
    if (((P[9] ^ C[9]) & 0x0000FFFFu) || ((P[10] ^ C[10]) & 0xFFFF0000u))   // 36-37, 42-43
        return false;
    if (((P[11] ^ C[11]) & 0x00FFFFFFu) || ((P[11] >> 16) & 0x0Fu))   // 44-46; 46's low nibble
        return false;
    if (((P[12] ^ C[12]) & 0x0000FFFFu) || (P[13] & 0xFFFFu) || (C[13] & 0xFFFFu))   // 48-49; 52-53
        return false;
    const u32 fp = P[11] >> 24, fc = C[11] >> 24;      // byte 47 (flags)
    if (fp != 0x10u || (fc != 0x10u && fc != 0x18u))
        return false;
    const int hl = 34 + 4 * (int)((P[11] >> 20) & 0x0Fu);
#pragma unroll
    for (int d = 13; d < 24; d++) {                    // options: bytes [54, hl)
        const int a = 4 * d < 54 ? 54 : 4 * d, b = 4 * d + 4 < hl ? 4 * d + 4 : hl;
        if (a < b && ((P[d] ^ C[d]) & (low_mask(b - 4 * d) & ~low_mask(a - 4 * d))))
            return false;
    }
    const u32 sp = __builtin_bswap32((P[9] >> 16) | (P[10] << 16));
    const u32 sc = __builtin_bswap32((C[9] >> 16) | (C[10] << 16));
    return sc == sp + (u32)pp;
}

// W = the largest window the instantiation takes (LDS is sized by it): W = 64
// needs ~9 KiB of LDS per block instead of ~36 KiB, so a CU holds twice the
// blocks (8 instead of 4) and twice the run-building waves.
// FLAT: phase D as one stream over the window's output instead of one wave
// per run -- see the comment at phase D2.  W <= 64: the window's frames sit in
// wave 0.  W > 64 (WIDE, round 5): every wave parses frames; chains and the
// segment list are block scans, the merged heads' header chunks are read from
// the input in D2, and the stash of each merged run's first chunks takes the
// header rows' LDS once D1 is done with them.
enum { SEG_HDR = 0, SEG_PAY = 1, SEG_WHOLE = 2 };

template <int U, int W = kGroW, int OCC = 1, bool FLAT = false, int FWM = WM_SECTOR,
          bool ACX = false, int PF = 0, int BT = kBlock>
__global__ void __launch_bounds__(BT, OCC)
k_gro(const uint8_t* __restrict__ in, uint64_t in_bytes, const uint64_t* __restrict__ off,
      const uint16_t* __restrict__ lens, const uint8_t* __restrict__ verdict, u32 n, u32 window,
      u32 max_len, uint8_t* __restrict__ out, uint64_t out_bytes, uint64_t* __restrict__ out_off,
      uint16_t* __restrict__ out_len, uint32_t* __restrict__ head)
{
    static_assert(W <= BT, "one frame per thread");
    constexpr int G = 64;
    constexpr bool WIDE = FLAT && W > 64;
    __shared__ __attribute__((aligned(16))) uint8_t hdr[W][kGroHdr];
    __shared__ int pay[W];         // TCP payload bytes of a mergeable frame, else -1
    __shared__ uint8_t cont[W];
    __shared__ uint8_t dok[W];     // descriptor inside the input buffer
    __shared__ uint32_t pref[W];   // payload offset of a member within its run
    __shared__ uint16_t rhead[W];  // run head (window index) of each frame
    __shared__ uint16_t run_t[W];  // runs: head index, member count, length, offset
    __shared__ uint16_t run_n[W];
    __shared__ uint32_t run_len[W];
    __shared__ uint64_t run_off[W];
    __shared__ int nruns;
    __shared__ uint64_t soff[W];   // the window's descriptors: no dependent global loads in D
    __shared__ uint16_t rn_at[W];  // per run head (window index): members, length, run index
    __shared__ uint32_t rl_at[W];
    __shared__ uint16_t ridx[W];
    __shared__ uint32_t wsum[BT / 64][2];
    __shared__ uint32_t nout_s;     // the window's output bytes (runs at 16 B-aligned offsets)
    constexpr int NS = FLAT ? 2 * W : 1, NRF = FLAT ? W : 1;
    __shared__ uint32_t sg_st[NS];  // FLAT: segments of the output, in output order
    __shared__ uint32_t sg_len[NS];
    __shared__ uint64_t sg_src[NS]; // input offset (SEG_HDR: the head's window index)
    __shared__ uint8_t sg_kind[NS];
    __shared__ uint8_t sg_run[NS];
    __shared__ int nseg_s;
    constexpr int NROW = FLAT ? 1024 : 1;   // 64-chunk output rows with a start entry (1 MiB)
    using SgIdx = std::conditional_t<(NS > 256), uint16_t, uint8_t>;
    __shared__ SgIdx sg_row[NROW];     // FLAT: the segment holding each row's first byte
    // FLAT: chunks 0..3 of each merged run (WIDE: in hdr's rows, dead after D1)
    static_assert(!WIDE || NRF * 64 <= W * kGroHdr, "the stash fits the header rows");
    __shared__ uint4 rstash_own[WIDE ? 1 : NRF][4];
    uint4 (*const rstash)[4] = WIDE ? reinterpret_cast<uint4 (*)[4]>(&hdr[0][0]) : rstash_own;
    __shared__ uint32_t rpf[NRF], rqe[NRF], wtot[BT / 64];
    constexpr int WW = WIDE ? W : 1;
    __shared__ uint8_t rpsh[WW];       // WIDE: each merged run's PSH bit (read before D2)
    __shared__ uint32_t cincl[WW], cexcl[WW], cwt[BT / 64];   // WIDE: block scans
    __shared__ uint64_t smask[BT / 64];   // WIDE: chain starts, per wave

    const int t = threadIdx.x;
    const uint64_t w0 = (uint64_t)blockIdx.x * window;
    const int cnt = (int)min<uint64_t>(window, n - w0);
    const uint4 z = make_uint4(0, 0, 0, 0);

    // A: parse.  PF (A/B, FLAT windows in wave 0): waves 1-3, idle until D,
    // read the window's input region meanwhile with cached loads, so that D2's
    // payload loads find it in L2 / the Infinity Cache.
    if constexpr (PF > 0) {
        if (t >= 64 && cnt > 0) {
            const uint64_t a = off[w0] & ~15ull, l = off[w0 + cnt - 1] + lens[w0 + cnt - 1];
            uint64_t b = l < in_bytes ? l : in_bytes;
            if (b > a && b - a > 64ull * 4096)         // not a packed window: no prefetch
                b = a;
            u32 x = 0;
            for (uint64_t base = a + 16ull * (t - 64); base < b; base += 16ull * (BT - 64) * PF) {
                uint4 v[PF];
#pragma unroll
                for (int k = 0; k < PF; k++) {
                    const uint64_t q = base + 16ull * (BT - 64) * k;
                    v[k] = q + 16 <= b ? ldg16<false>(in + q) : z;
                }
#pragma unroll
                for (int k = 0; k < PF; k++)
                    x ^= v[k].x ^ v[k].w;
            }
            if (x == 0x9E3779B9u && t == 64 && cnt == 1 && w0 == (uint64_t)-1)
                head[0] = x;                               // never: keeps the loads alive
        }
    }
    if (t < cnt) {
        const uint64_t o = off[w0 + t];
        const u32 L = lens[w0 + t];
        soff[t] = o;
        const bool ok = (o & 15) == 0 && o <= in_bytes && L <= in_bytes - o;
        const bool acc = ok && verdict[w0 + t] == GCS_V_ACCEPT;
        dok[t] = ok;
#pragma unroll
        for (int c = 0; c < kGroHdr / 16; c++) {
            const uint4 v = acc ? load_chunk<true, false>(in + o + 16 * c,
                                                          (int64_t)(in_bytes - o) - 16 * c)
                                : z;
            uint32_t* d = reinterpret_cast<uint32_t*>(&hdr[t][16 * c]);
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
        const uint8_t* h = hdr[t];
        int p = -1;
        if (acc && (h[14] & 0x0F) == 5)
            p = (int)lds_be16(h + 16) - 20 - 4 * (h[46] >> 4);
        pay[t] = p;
    }
    __syncthreads();
    // B: continuation
    if (t < cnt)
        cont[t] = t > 0 && (ACX ? gro_cont32(hdr[t - 1], hdr[t], pay[t - 1], pay[t])
                                : gro_cont(hdr[t - 1], hdr[t], pay[t - 1], pay[t]));
    __syncthreads();
    // C: runs.  A chain is a maximal sequence of frames that each continue the
    // previous one (cont); every frame of a chain is mergeable, so runs are
    // chains cut greedily at max_len -- ref_gro_batch's walk, done by each
    // chain's first thread over its own chain, in parallel.  Then one block
    // scan gives every run its index and its 16 B-aligned output offset.
    // (One thread walking the whole window took ~1/3 of the kernel.)
    uint32_t rl = 0;                                   // this thread's run length if it heads one
    bool rs = false;                                   // ... and whether it does
    bool walk = true;                                  // this chain needs the sequential walk
    if constexpr (ACX && WIDE) {
        // the same over the block: chain heads and ends from the waves' start
        // masks, payload prefixes from a block scan
        const int lane = t & 63, wv = t >> 6;
        const bool valid = t < cnt, start = !valid || t == 0 || !cont[t];
        const uint64_t sm = __ballot(start);
        const u32 pv = valid && pay[t] > 0 ? (u32)pay[t] : 0u;
        const u32 winc = wave_incl_scan(pv);
        if (lane == 63) {
            smask[wv] = sm;
            cwt[wv] = winc;
        }
        __syncthreads();
        u32 base = 0;
        for (int q = 0; q < wv; q++)
            base += cwt[q];
        const u32 incl = base + winc, excl = incl - pv;
        if (t < WW) {
            cincl[t] = incl;
            cexcl[t] = excl;
        }
        const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
        int sh = 0;                                    // the last start at or below t
        if (sm & upto) {
            sh = 64 * wv + 63 - __clzll(sm & upto);
        } else {
            for (int q = wv - 1; q >= 0; q--)
                if (smask[q]) {
                    sh = 64 * q + 63 - __clzll(smask[q]);
                    break;
                }
        }
        const uint64_t above = sm & ~upto;
        int se = BT - 1;                           // the frame before the next start
        if (above) {
            se = 64 * wv + __ffsll((long long)above) - 2;
        } else {
            for (int q = wv + 1; q < BT / 64; q++)
                if (smask[q]) {
                    se = 64 * q + __ffsll((long long)smask[q]) - 2;
                    break;
                }
        }
        __syncthreads();                               // cincl / cexcl complete
        if (valid) {
            const u32 hx = cexcl[sh];
            const u32 tot = cincl[se] - hx;            // the chain's payload
            const u32 hhl = 34 + 4 * (hdr[sh][46] >> 4);
            const bool fits = pay[sh] > 0 && hhl + tot <= max_len;
            walk = !fits;
            if (fits) {
                pref[t] = excl - hx;
                rhead[t] = (uint16_t)sh;
                if (t == sh) {
                    rn_at[t] = (uint16_t)(se - sh + 1);
                    rl_at[t] = hhl + tot;
                }
            }
        }
    } else if constexpr (ACX) {
        static_assert(W <= 64, "a window's frames sit in wave 0");
        // A chain whose whole payload fits max_len is one run: its members'
        // payload offsets are a segmented scan of the wave, no walk.
        if (t < 64) {
            const bool valid = t < cnt, start = !valid || t == 0 || !cont[t];
            const uint64_t sm = __ballot(start);
            const uint64_t upto = t == 63 ? ~0ull : ((2ull << t) - 1);
            const int sh = 63 - __clzll(sm & upto);                 // chain head
            const uint64_t above = sm & ~upto;
            const int se = above ? __ffsll((long long)above) - 2 : 63;   // chain's last lane
            const u32 pv = valid && pay[t] > 0 ? (u32)pay[t] : 0u;
            const u32 incl = wave_incl_scan(pv), excl = incl - pv;
            const u32 hx = (u32)__shfl((int)excl, sh, 64);
            const u32 tot = (u32)__shfl((int)incl, se, 64) - hx;      // the chain's payload
            const int hp = __shfl(valid ? pay[t] : -1, sh, 64);
            const u32 hhl = 34 + 4 * (hdr[sh][46] >> 4);
            const bool fits = hp > 0 && hhl + tot <= max_len;
            walk = !fits;
            if (valid && fits) {
                pref[t] = excl - hx;
                rhead[t] = (uint16_t)sh;
                if (t == sh) {
                    rn_at[t] = (uint16_t)(se - sh + 1);
                    rl_at[t] = hhl + tot;
                }
            }
        }
    }
    if (walk && t < cnt && (t == 0 || !cont[t])) {
        int cur = t;
        u32 mlen = pay[t] > 0 ? 34 + 4 * (hdr[t][46] >> 4) + (u32)pay[t]
                              : (dok[t] ? (u32)lens[w0 + t] : 0u);     // a bad descriptor: nothing
        pref[t] = 0;
        rhead[t] = (uint16_t)t;
        rn_at[t] = 1;
        for (int k = t + 1; k < cnt && cont[k]; k++) {
            if (mlen + (u32)pay[k] <= max_len) {
                pref[k] = mlen - (34 + 4 * (hdr[cur][46] >> 4));
                mlen += (u32)pay[k];
                rhead[k] = (uint16_t)cur;
                rn_at[cur]++;
                continue;
            }
            rl_at[cur] = mlen;                         // max_len cut: k heads a new run
            cur = k;
            mlen = 34 + 4 * (hdr[k][46] >> 4) + (u32)pay[k];
            pref[k] = 0;
            rhead[k] = (uint16_t)k;
            rn_at[k] = 1;
        }
        rl_at[cur] = mlen;
    }
    __syncthreads();
    if (t < cnt && rhead[t] == t) {
        rs = true;
        rl = rl_at[t];
    }
    // exclusive scans of (run starts, aligned run lengths) over the window
    u32 xs = rs ? 1u : 0u, xl = rs ? (rl + 15u) & ~15u : 0u;
    {
        const int lane = t & 63, w = t >> 6;
        u32 is = xs, il = xl;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u32 os = __shfl_up(is, d, 64), ol = __shfl_up(il, d, 64);
            if (lane >= d) {
                is += os;
                il += ol;
            }
        }
        if (lane == 63) {
            wsum[w][0] = is;
            wsum[w][1] = il;
        }
        __syncthreads();
        u32 bs = 0, bl = 0;
        for (int q = 0; q < w; q++) {
            bs += wsum[q][0];
            bl += wsum[q][1];
        }
        xs = bs + is - xs;                             // exclusive
        xl = bl + il - xl;
        if (t == BT - 1) {
            nruns = (int)(bs + is);
            nout_s = bl + il;
        }
    }
    const uint64_t o0 = cnt ? soff[0] : 0;
    if (rs) {
        run_t[xs] = (uint16_t)t;
        run_n[xs] = (uint16_t)rn_at[t];
        run_len[xs] = rl;
        run_off[xs] = o0 + xl;
        ridx[t] = (uint16_t)xs;
    }
    __syncthreads();
    if (t < cnt) {
        const int hk = rhead[t];
        const int r = ridx[hk];
        head[w0 + t] = (uint32_t)(w0 + hk);
        out_off[w0 + t] = run_off[r];
        out_len[w0 + t] = hk == t ? (uint16_t)run_len[r] : (uint16_t)0;
    }

    if constexpr (FLAT) {
        if constexpr (WIDE) {
            // each merged run's PSH bit for D3, before the stash takes hdr's rows
            if (t < nruns && run_n[t] > 1) {
                uint8_t p = 0;
                for (int k = run_t[t]; k < run_t[t] + run_n[t]; k++)
                    p |= hdr[k][47] & 0x08;
                rpsh[t] = p;
            }
        }
        // D1: the output as segments: a merged run's head headers (from LDS;
        // WIDE: from the input), each member's payload, or a single frame as it is
        if (WIDE || t < 64) {                        // WIDE: every thread (a block scan)
            int ns = 0, k0 = SEG_HDR;
            u32 st0 = 0, ln0 = 0, ln1 = 0;
            uint64_t sr0 = 0, sr1 = 0;
            int rr = 0;
            if (t < cnt) {
                const int hk = rhead[t];
                rr = ridx[hk];
                const int nm = run_n[rr];
                const u32 rel = (u32)(run_off[rr] - o0);
                if (nm == 1) {
                    if (run_len[rr] > 0) {
                        ns = 1;
                        k0 = SEG_WHOLE;
                        st0 = rel;
                        ln0 = run_len[rr];
                        sr0 = soff[t];
                    }
                } else {
                    const u32 hl = 34 + 4 * (hdr[hk][46] >> 4);
                    if (t == hk) {
                        ns = 2;
                        k0 = SEG_HDR;
                        st0 = rel;
                        ln0 = hl;
                        sr0 = WIDE ? soff[hk] : (uint64_t)hk;
                        ln1 = (u32)pay[t];
                        sr1 = soff[t] + hl;
                    } else {
                        ns = 1;
                        k0 = SEG_PAY;
                        st0 = rel + hl + pref[t];
                        ln0 = (u32)pay[t];
                        sr0 = soff[t] + hl;
                    }
                }
            }
            const u32 winc = wave_incl_scan((u32)ns);
            u32 base = 0;
            if constexpr (WIDE) {
                if ((t & 63) == 63)
                    cwt[t >> 6] = winc;
                __syncthreads();
                for (int q = 0; q < (t >> 6); q++)
                    base += cwt[q];
            }
            const u32 incl = base + winc;
            const int e = (int)(incl - (u32)ns);
            if (ns >= 1) {
                sg_st[e] = st0;
                sg_len[e] = ln0;
                sg_src[e] = sr0;
                sg_kind[e] = (uint8_t)k0;
                sg_run[e] = (uint8_t)rr;
            }
            if (ns == 2) {
                sg_st[e + 1] = st0 + ln0;
                sg_len[e + 1] = ln1;
                sg_src[e + 1] = sr1;
                sg_kind[e + 1] = SEG_PAY;
                sg_run[e + 1] = (uint8_t)rr;
            }
            if (t == (WIDE ? BT - 1 : 63))
                nseg_s = (int)incl;
        }
        __syncthreads();
        {
            // per 64-chunk row of the output, the segment holding its first byte
            // (one binary search per row here instead of one per chunk in D2)
            const int nsg = nseg_s;
            const u32 nrow = ((nout_s >> 4) + 63) >> 6;
            for (u32 rw = t; rw < nrow && rw < (u32)NROW; rw += BT) {
                const u32 p = rw << 10;
                int sgi = 0;
#pragma unroll
                for (int step = NS / 2; step > 0; step >>= 1)
                    if (sgi + step < nsg && sg_st[sgi + step] <= p)
                        sgi += step;
                sg_row[rw] = (SgIdx)sgi;
            }
        }
        __syncthreads();
        // D2: the window's output chunks as one stream, wave w a quarter of
        // them, 64 * U per trip.  A chunk finds its segment by binary search
        // (7 steps over <= 128 starts in LDS) and is one unaligned load, or
        // two at a segment boundary, or (tiny payloads, the input's end) a
        // byte loop.  Each lane folds its chunk to one word sum and a DPP
        // wave scan makes prefixes; a merged run's checks are then
        // Q(end) - Q(start) plus its header chunks (D3), as in
        // k_desc_stream.  Chunks 0..3 of merged runs wait in LDS for D3.
        const int nseg = nseg_s, wave = t >> 6, lane = t & 63;
        const u32 NOUT = nout_s >> 4;
        const u32 QW = ((NOUT + BT - 1) / BT) * 64;        // BT / 64 waves
        const u32 lo = wave * QW, hi = lo + QW < NOUT ? lo + QW : NOUT;
        uint8_t* ob = out + o0;
        const int64_t wl_all = o0 <= out_bytes ? (int64_t)(out_bytes - o0) : 0;
        const uint8_t* in_end = in + in_bytes;
        u32 run = 0;
        for (u32 base = lo; base < hi; base += 64 * U) {
            uint4 x[U], y[U];
            int sj[U], pl[U];
#pragma unroll
            for (int j = 0; j < U; j++) {
                const u32 c = base + 64 * j + lane, p = 16 * c;
                // from the row's first segment: a row (1 KiB) spans few segments
                const u32 rw = (c < hi ? c : hi - 1) >> 6;
                int sgi = rw < (u32)NROW ? sg_row[rw] : 0;   // past the table: search
#pragma unroll
                for (int k = 0; k < 3; k++)
                    if (sgi + 1 < nseg && sg_st[sgi + 1] <= p)
                        sgi++;
                if (sgi + 1 < nseg && sg_st[sgi + 1] <= p) {   // tiny segments: search on
                    int lo2 = sgi + 1, hi2 = nseg - 1;
                    while (lo2 < hi2) {
                        const int mid = (lo2 + hi2 + 1) >> 1;
                        if (sg_st[mid] <= p) lo2 = mid; else hi2 = mid - 1;
                    }
                    sgi = lo2;
                }
                sj[j] = sgi;
                x[j] = z;
                y[j] = z;
                int plan = AS_ZERO;
                if (c < hi) {
                    const u32 ss = sg_st[sgi], sl = sg_len[sgi], kd = sg_kind[sgi];
                    const int r = sg_run[sgi];
                    const u32 rend = (u32)(run_off[r] - o0) + run_len[r];
                    const u32 offs = p - ss, rem = sl - offs;
                    const u32 need = rend - p < 16u ? rend - p : 16u;
                    const uint8_t* pa = in + sg_src[sgi] + offs;
                    if (!WIDE && kd == SEG_HDR && offs + 16 <= (u32)kGroHdr) {
                        x[j] = *reinterpret_cast<const uint4*>(&hdr[sg_src[sgi]][offs]);
                        plan = AS_ONE;
                    } else if ((WIDE || kd != SEG_HDR) && pa + 16 <= in_end) {
                        x[j] = ldg16u(pa);
                        plan = AS_ONE;
                    } else {
                        plan = AS_BYTES;
                    }
                    if (plan == AS_ONE && rem < need) {
                        const int s2 = sgi + 1;
                        const uint8_t* pb = in + sg_src[s2];
                        if (s2 < nseg && sg_run[s2] == r && sg_st[s2] == ss + sl &&
                            sg_kind[s2] == SEG_PAY && sg_len[s2] >= need - rem && pb + 16 <= in_end) {
                            y[j] = ldg16u(pb);
                            plan = AS_TWO;
                        } else {
                            plan = AS_BYTES;
                        }
                    }
                }
                pl[j] = plan;
            }
#pragma unroll
            for (int j = 0; j < U; j++) {
                const u32 c = base + 64 * j + lane, p = 16 * c;
                const int sgi = sj[j], r = sg_run[sgi];
                const u32 ss = sg_st[sgi], sl = sg_len[sgi];
                const u32 rrel = (u32)(run_off[r] - o0), rend = rrel + run_len[r];
                const bool merged = sg_kind[sgi] != SEG_WHOLE;
                if (pl[j] == AS_TWO) {
                    x[j] = blend(x[j], bytes_up(y[j], (int)(ss + sl - p)),
                                 byte_mask((int)(ss + sl - p), 16));
                } else if (pl[j] == AS_BYTES) {
                    u32 wv[4] = {0u, 0u, 0u, 0u};
                    int s2 = sgi;
                    for (int k = 0; k < 16; k++) {
                        const u32 q = p + k;
                        if (q >= rend)
                            break;
                        while (s2 + 1 < nseg && q >= sg_st[s2] + sg_len[s2])
                            s2++;
                        if (q < sg_st[s2] || q >= sg_st[s2] + sg_len[s2])
                            continue;
                        const u32 b = !WIDE && sg_kind[s2] == SEG_HDR
                                          ? (u32)hdr[sg_src[s2]][q - sg_st[s2]]
                                          : (in + sg_src[s2] + (q - sg_st[s2]) < in_end
                                                 ? (u32)in[sg_src[s2] + (q - sg_st[s2])] : 0u);
                        wv[k >> 2] |= b << (8 * (k & 3));
                    }
                    x[j] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                }
                if (merged && pl[j] != AS_ZERO && rend - p < 16u)       // nothing past the run
                    x[j] = blend(z, x[j], byte_mask(0, (int)(rend - p)));
                const u32 sum = pl[j] != AS_ZERO ? hsum4(x[j]) : 0u;
                const u32 incl = wave_incl_scan(sum);
                const u32 excl = run + incl - sum;
                run += (u32)__builtin_amdgcn_readlane((int)incl, 63);
                if (pl[j] == AS_ZERO)
                    continue;
                const u32 kr = (p - rrel) >> 4;
                if (merged) {
                    if (kr == 0)
                        rpf[r] = excl;
                    if (p + 16 >= rend)
                        rqe[r] = excl + sum;                   // Q at the run's end
                    if (kr < 4) {
                        rstash[r][kr] = x[j];
                        continue;
                    }
                }
                if ((int64_t)p + 16 <= wl_all) {
                    stg16<FWM>(ob + p, x[j]);
                } else {
                    for (int k = 0; k < 16 && (int64_t)(p + k) < wl_all && (!merged || p + k < rend); k++)
                        ob[p + k] = (uint8_t)chunk_byte(x[j], k);
                }
            }
        }
        if (lane == 0)
            wtot[wave] = run;
        __syncthreads();
        // D3: one thread per merged run: tot_len and PSH into the head's
        // headers, the checks from chunks 0..3 and the prefix difference, then
        // chunks 0..3 out
        if (t < nruns && run_n[t] > 1) {
            const int r = t, k0 = run_t[r], nm = run_n[r];
            const u32 mlen = run_len[r], rrel = (u32)(run_off[r] - o0);
            uint4 sc[4] = {rstash[r][0], rstash[r][1], rstash[r][2], rstash[r][3]};
            const u32 raw = hsum4(sc[0]) + hsum4(sc[1]) + hsum4(sc[2]) + hsum4(sc[3]);
            uint8_t psh = 0;
            if constexpr (WIDE) {
                psh = rpsh[r];
            } else {
                for (int k = k0; k < k0 + nm; k++)
                    psh |= hdr[k][47] & 0x08;
            }
            sc[1].x = (sc[1].x & 0xFFFF0000u) | bswap16((mlen - 14) & 0xFFFFu);
            sc[2].w |= (u32)psh << 24;
            Hdr h;
            h.d3 = sc[0].w;
            h.d4 = sc[1].x;
            h.d5 = sc[1].y;
            const int te = (int)mlen;
            Acc a = {0u, 0u, 0u};
#pragma unroll
            for (int c = 0; c < 4; c++)
                accum_fast5<true, true>(sc[c], c, te, masks5<true>(c), a);
            if (te > 64) {
                auto wbase = [&](u32 ch) {
                    const u32 q = ch / QW;
                    u32 b = 0;
#pragma unroll
                    for (int k = 0; k < BT / 64 - 1; k++)
                        b += (u32)k < q ? wtot[k] : 0u;
                    return b;
                };
                const u32 p0 = rpf[r] + wbase(rrel >> 4);
                const u32 p1 = rqe[r] + wbase((rrel + mlen - 1) >> 4);
                a.tcp += (p1 - p0) - raw;
            }
            uint8_t st = 0;
            uint32_t cs = 0;
            epilogue<1, 4, true, WM_SECTOR, false>(h, a, ob + rrel, mlen, 0, true, 0,
                                                   GCS_CF_NO_INPLACE, &st, &cs, true, sc);
            if (st == GCS_TX_OK || st == GCS_TX_IP_ONLY || st == GCS_TX_BAD_TCPLEN)
                sc[1].z = (sc[1].z & 0xFFFF0000u) | (cs & 0xFFFFu);          // bytes 24-25
            if (st == GCS_TX_OK)
                sc[3].x = (sc[3].x & 0x0000FFFFu) | (cs & 0xFFFF0000u);      // bytes 50-51
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const u32 p = rrel + 16 * c;
                if (16 * c >= (int)mlen)
                    break;
                if ((int64_t)p + 16 <= wl_all) {
                    stg16<FWM>(ob + p, sc[c]);
                } else {
                    for (int k = 0; k < 16 && (int64_t)(p + k) < wl_all && 16 * c + k < (int)mlen; k++)
                        ob[p + k] = (uint8_t)chunk_byte(sc[c], k);
                }
            }
        }
        return;
    }

    // D: build the runs, one wave per run
    const int wave = t >> 6, sub = t & 63, nwaves = BT / 64;
    for (int r = wave; r < nruns; r += nwaves) {       // wave-uniform
        const int k0 = run_t[r], nm = run_n[r];
        const u32 mlen = run_len[r];
        const uint64_t oo = run_off[r];
        uint8_t* m = out + oo;
        const int64_t wlim = oo <= out_bytes ? (int64_t)(out_bytes - oo) : 0;
        const uint64_t io = soff[k0];
        const int nchunks = (int)((mlen + 15) >> 4);
        if (nm == 1) {                                 // as it is
            const int64_t avail = (int64_t)(in_bytes - io);
            for (int c = sub; c < nchunks; c += G) {
                const uint4 v = load_chunk<true, false>(in + io + 16 * c, avail - 16 * c);
                if (16 * c + 16 <= wlim) {
                    stg16<WM_SECTOR>(m + 16 * c, v);
                } else {
                    for (int k = 0; k < 16 && 16 * c + k < (int)mlen && 16 * c + k < wlim; k++)
                        m[16 * c + k] = (uint8_t)chunk_byte(v, k);
                }
            }
            continue;
        }
        const uint8_t* hh = hdr[k0];
        const int hl = 34 + 4 * (hh[46] >> 4);
        uint8_t psh = 0;
        for (int k = k0; k < k0 + nm; k++)
            psh |= hdr[k][47] & 0x08;
        const int ts = 34, te = (int)mlen;
        Acc a = {0u, 0u, 0u};
        uint4 first[U];
        const uint8_t* in_end = in + in_bytes;
        for (int base = 0; base < nchunks; base += G * U) {
            uint4 v[U], pa[U], pb[U];
            int plan[U], cut[U];
            // 1: issue the loads of every chunk of the batch
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int c = base + j * G + sub;
                const int cb = 16 * c;
                int pl = AS_ZERO, ct = 0, sg = k0;
                pa[j] = z;
                pb[j] = z;
                if (c < nchunks && cb + 16 <= hl) {
                    pl = AS_FRAME;                                 // head's headers (LDS)
                } else if (c < nchunks && cb < hl) {
                    const uint8_t* p0 = in + soff[k0] + hl;
                    ct = hl - cb;                                  // header bytes in the chunk
                    if (cb + 16 <= te && pay[k0] >= 16 - ct && p0 + 16 <= in_end) {
                        pl = AS_UP;
                        pa[j] = ldg16u(p0);
                    } else {
                        pl = AS_BYTES;
                    }
                } else if (c < nchunks) {
                    const u32 q = (u32)(cb - hl);                  // merged payload offset
                    int lo2 = k0, hi2 = k0 + nm - 1;
                    while (lo2 < hi2) {
                        const int mid = (lo2 + hi2 + 1) >> 1;
                        if (pref[mid] <= q) lo2 = mid; else hi2 = mid - 1;
                    }
                    sg = lo2;
                    const int rem = (int)(pref[sg] + (u32)pay[sg] - q);   // bytes left in sg
                    const int need = min(16, te - cb);
                    const uint8_t* pq = in + soff[sg] + hl + (q - pref[sg]);
                    if (rem >= need && pq + 16 <= in_end) {
                        pl = AS_ONE;                               // one member (masked at te)
                        pa[j] = ldg16u(pq);
                    } else if (sg + 1 < k0 + nm && pay[sg + 1] >= need - rem &&
                               pq + 16 <= in_end && in + soff[sg + 1] + hl + 16 <= in_end) {
                        pl = AS_TWO;                               // the end of sg, then sg+1
                        ct = rem;
                        pa[j] = ldg16u(pq);
                        pb[j] = ldg16u(in + soff[sg + 1] + hl);
                    } else {
                        pl = AS_BYTES;
                    }
                }
                plan[j] = pl;
                cut[j] = ct;
            }
            // 2: assemble
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int c = base + j * G + sub;
                const int cb = 16 * c;
                uint4 x = z;
                switch (plan[j]) {
                case AS_FRAME:
                    x = *reinterpret_cast<const uint4*>(&hh[cb]);
                    break;
                case AS_UP:
                    x = blend(*reinterpret_cast<const uint4*>(&hh[cb]), bytes_up(pa[j], cut[j]),
                              byte_mask(cut[j], 16));
                    break;
                case AS_ONE:
                    x = pa[j];
                    break;
                case AS_TWO:
                    x = blend(pa[j], bytes_up(pb[j], cut[j]), byte_mask(cut[j], 16));
                    break;
                case AS_BYTES: {
                    u32 w[4] = {0u, 0u, 0u, 0u};
                    int s2 = k0;
                    for (int k = 0; k < 16; k++) {
                        const int p = cb + k;
                        u32 b = 0;
                        if (p < hl) {
                            b = hh[p];
                        } else if (p < te) {
                            const u32 qq = (u32)(p - hl);
                            while (qq >= pref[s2] + (u32)pay[s2])
                                s2++;
                            b = in[soff[s2] + hl + (qq - pref[s2])];
                        }
                        w[k >> 2] |= b << (8 * (k & 3));
                    }
                    x = make_uint4(w[0], w[1], w[2], w[3]);
                    break;
                }
                default:
                    break;
                }
                if (c < nchunks && cb + 16 > te)                    // nothing past the frame
                    x = blend(z, x, byte_mask(0, te - cb));
                if (c == 1)                                        // tot_len (bytes 16-17)
                    x.x = (x.x & 0xFFFF0000u) | bswap16((mlen - 14) & 0xFFFFu);
                if (c == 2)                                        // flags (byte 47): PSH of any member
                    x.w |= (u32)psh << 24;
                v[j] = x;
            }
#pragma unroll
            for (int j = 0; j < U; j++)
                accum_chunk<true>(v[j], 16 * (base + j * G + sub), ts, te, a);
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int c = base + j * G + sub;
                const int cb = 16 * c;
                if (c < 8 || c >= nchunks)
                    continue;
                if (cb + 16 <= wlim) {
                    stg16<WM_SECTOR>(m + cb, v[j]);
                } else {
                    for (int k = 0; k < 16 && cb + k < te && cb + k < wlim; k++)
                        m[cb + k] = (uint8_t)chunk_byte(v[j], k);
                }
            }
            if (base == 0) {
#pragma unroll
                for (int j = 0; j < U; j++)
                    first[j] = v[j];
            }
        }
        Hdr h;
        h.d3 = group_bcast<G, 0>(first[0].w);
        h.d4 = group_bcast<G, 1>(first[0].x);
        h.d5 = group_bcast<G, 1>(first[0].y);
        epilogue<G, U, true, WM_LINE_SC1>(h, a, m, mlen, wlim, true, sub, 0u, nullptr, nullptr,
                                          true, first);
    }
}

// TCPCalcChecksum(buf + off[i], len[i], saddr[i], daddr[i]), G lanes per item;
// PSEUDO = false: ICMPChecksum(buf + off[i], len[i]) (icmp.c:18-42), the same
// word loop and odd-byte rule without the pseudo header.
template <int G, bool PSEUDO = true>
__global__ void __launch_bounds__(kBlock)
k_tcp_fn(const uint8_t* __restrict__ buf, uint64_t buf_bytes, const uint64_t* __restrict__ off,
         const uint16_t* __restrict__ lens, const uint32_t* __restrict__ saddr,
         const uint32_t* __restrict__ daddr, u32 n, uint16_t* __restrict__ out)
{
    constexpr int FPB = kBlock / G;
    const int sub = threadIdx.x & (G - 1);
    const uint64_t i = (uint64_t)blockIdx.x * FPB + threadIdx.x / G;
    if (i >= n)
        return;
    const uint64_t o = off[i];
    const u32 len = lens[i];
    const bool ok = (o & 1) == 0 && o <= buf_bytes && len <= buf_bytes - o;
    const uint64_t base = ok ? (o & ~15ull) : 0;
    const int a = (int)(o - base);                     // even
    const int b = a + (int)len;
    const int nchunks = ok ? (b + 15) >> 4 : 0;
    const int64_t avail = (int64_t)(buf_bytes - base);
    u32 s = 0;
    for (int c = sub; c < nchunks; c += G) {
        uint4 v = load_chunk<true, false>(buf + base + 16 * c, avail - 16 * c);
        int p = 16 * c;
        if (p >= a && p + 16 <= b)
            s += hsum4(v);
        else
            s += region_sum(v.x, p, a, b) + region_sum(v.y, p + 4, a, b) +
                 region_sum(v.z, p + 8, a, b) + region_sum(v.w, p + 12, a, b);
    }
    s = group_sum<G>(s);
    if (sub != 0)
        return;
    if (!ok) {
        out[i] = 0;
        return;
    }
    if (PSEUDO) {
        const u32 sa = saddr[i], da = daddr[i];
        s += (sa & 0xFFFFu) + (sa >> 16) + (da & 0xFFFFu) + (da >> 16);   // tcp_util.c:266-267
        s += bswap16(len) + 0x0600u;                                       // :268-269
    }
    out[i] = (uint16_t)csum16(s);
}

// GetRSSHash / GetRSSCPUCore (rss.c:44-115) of host-order tuples, one lane
// per item (the same hash as the fused path, with a one-lane "group").
__global__ void __launch_bounds__(kBlock)
k_rss_fn(const uint32_t* __restrict__ sip, const uint32_t* __restrict__ dip,
         const uint16_t* __restrict__ sp, const uint16_t* __restrict__ dp, u32 n, Ext ext)
{
    __shared__ u32 nib[kNibEntries];
    rss_nibble_tables(ext.key, nib);
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const XFrame xf = xframe(ext, i);
    const u32 h = rss_hash<1>(xf.key, sip[i], dip[i], ((u32)sp[i] << 16) | dp[i], 0, nib);
    if (xf.hash)
        *xf.hash = h;
    if (xf.queue)
        *xf.queue = (uint16_t)rss_queue(xf, h);
}

// ip_fast_csum(buf + off[i], ihl[i]), one lane per item (<= 60 bytes each).
__global__ void __launch_bounds__(kBlock)
k_ip_fn(const uint8_t* __restrict__ buf, uint64_t buf_bytes, const uint64_t* __restrict__ off,
        const uint8_t* __restrict__ ihls, u32 n, uint16_t* __restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t o = off[i];
    const u32 ihl = ihls[i] & 15u;
    const u32 need = ihl <= 4 ? 4u : 4u * ihl;
    if ((o & 1) || o > buf_bytes || need > buf_bytes - o) {
        out[i] = 0;
        return;
    }
    const uint16_t* w = reinterpret_cast<const uint16_t*>(buf + o);
    if (ihl <= 4) {                                // ps.h:72-73: raw low 16 bits of word 0
        out[i] = w[0];
        return;
    }
    u32 s = 0;
    for (u32 k = 0; k < 2 * ihl; k++)
        s += w[k];
    out[i] = (uint16_t)csum16(s);
}

// ---------------------------------------------------------------------------
// launchers (called from gcs_api.cpp)

// TX write-back of a fixed-stride frame: the 64 B sector holding both check
// fields, or its whole first 128 B line.  The line lies inside the frame's own
// slot (16 * chunks <= stride), so no other frame shares it, and at a 128 B-
// multiple stride it is one aligned line.  A whole line drains cheaper than a
// partial one while the written lines stay in the Infinity Cache, but it is
// twice the bytes once they spill to HBM: C2 1M x 1500 B 260.6 -> 254.6 us,
// 2M 524.9 -> 563.7 us, 4M 1114 -> 1178 us (profiles/r02/pmc_configs.csv,
// kbench_tx_nt.log).  So lines up to kLineWbBytes of them per launch, sectors
// beyond.  (Descriptor batches keep the sector: a packed frame's line can hold
// its neighbour's bytes.)
constexpr uint64_t kLineWbBytes = 128ull << 20;

// GCS_TX_LINE_WB_MB overrides kLineWbBytes (MB of lines per launch; 0 = sector
// write-back only): an A/B knob for the bench step, read once.
static uint64_t line_wb_bytes()
{
    static const uint64_t v = [] {
        const char* e = std::getenv("GCS_TX_LINE_WB_MB");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) << 20 : kLineWbBytes;
    }();
    return v;
}

template <int G, int U, bool COMPUTE, bool LOOP, bool EXT, int K = 1, int WM = kWM>
static hipError_t launch_fixed_wm(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                                  uint8_t* code, uint32_t* csum, u32 flags, const Ext& ext,
                                  hipStream_t s)
{
    constexpr int FPB = kBlock / G * K;                // frames per block
    dim3 grid((n + FPB - 1) / FPB);
    if (EXT)
        hipLaunchKernelGGL((k_fixed_x<G, U, COMPUTE, LOOP, kNT, WM, kXCD, K>), grid, dim3(kBlock),
                           0, s, frames, stride, frame_len, n, code, csum, flags, ext);
    else
        hipLaunchKernelGGL((k_fixed<G, U, COMPUTE, LOOP, kNT, WM, kXCD, K>), grid, dim3(kBlock),
                           0, s, frames, stride, frame_len, n, code, csum, flags);
    return hipGetLastError();
}

// A fill too large for whole-line write-back (C4: 4M frames) writes whole
// lines for its first line_wb_bytes() / 128 frames -- their dirty lines fit
// the Infinity Cache -- and the 64 B sectors with non-temporal stores for the
// rest, in ONE launch (k_fixed_tx2): 4M x 1500 B fill 1,093-1,096 us (0.719-
// 0.721 of 8 TB/s) as two launches against 1,104-1,137 us with sc1 sectors
// for the whole batch, 1,117-1,120 us with nt sectors alone, 1,215-1,223 us
// with sc1 sectors after the lines (profiles/r06/r06{d,e}).  GCS_TX_HYBRID
// (read once): nt (default), sc1, off (sc1 sectors for the whole batch, as
// before round 6).
static int tx_hybrid()
{
    static const int v = [] {
        const char* e = std::getenv("GCS_TX_HYBRID");
        if (!e || std::strcmp(e, "nt") == 0) return 2;
        if (std::strcmp(e, "sc1") == 0) return 1;
        return 0;
    }();
    return v;
}

// The TX write-back of a plain fixed-stride fill of n frames (G >= 8 lanes
// per frame): WMA for the frames of logical blocks [0, split), WMB after.
struct TxWb {
    int mode;      // 0: kWM whole batch; 1: lines whole batch; 2: lines then nt; 3: lines then sc1
    u32 split;     // logical blocks written with lines (modes 2, 3)
};

static TxWb tx_wb(uint64_t stride, u32 n, u32 flags, u32 fpb)
{
    if (stride % 128 != 0 || (flags & GCS_CF_SECTOR_WB))
        return {0, 0};
    if ((uint64_t)n * 128 <= line_wb_bytes())
        return {1, 0};
    const int hy = tx_hybrid();
    const u32 m = (u32)(line_wb_bytes() / 128) / fpb;
    if (!hy)
        return {0, 0};
    return {hy == 2 ? 2 : 3, m};
}

template <int G, int U, bool LOOP, int WMA, int WMB>
__global__ void __launch_bounds__(kBlock)
k_fixed_tx2(uint8_t* __restrict__ frames, uint64_t stride, u32 frame_len, u32 n,
            uint8_t* __restrict__ out_code, uint32_t* __restrict__ out_csum, u32 flags, u32 split)
{
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x);    // block-uniform choice below
    if (blk < split)
        fixed_frame<G, U, true, LOOP, kNT, WMA, false, false>(frames, stride, frame_len, n,
                                                              out_code, out_csum, flags, Ext{},
                                                              blk, gridDim.x);
    else
        fixed_frame<G, U, true, LOOP, kNT, WMB, false, false>(frames, stride, frame_len, n,
                                                              out_code, out_csum, flags, Ext{},
                                                              blk, gridDim.x);
}

template <int G, int U, bool COMPUTE, bool LOOP, bool EXT, int K = 1>
static hipError_t launch_fixed(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                               uint8_t* code, uint32_t* csum, u32 flags, const Ext& ext,
                               hipStream_t s)
{
    if constexpr (COMPUTE && G >= 8) {
        constexpr u32 FPB = kBlock / G * K;
        const TxWb wb = tx_wb(stride, n, flags, FPB);
        if (wb.mode == 1)
            return launch_fixed_wm<G, U, COMPUTE, LOOP, EXT, K, WM_LINE_SC1>(
                frames, stride, frame_len, n, code, csum, flags, ext, s);
        if constexpr (!EXT && K == 1) {
            if (wb.mode >= 2) {
                const dim3 grid((n + FPB - 1) / FPB);
                if (wb.mode == 2)
                    hipLaunchKernelGGL((k_fixed_tx2<G, U, LOOP, WM_LINE_SC1, WM_SECTOR_NT>), grid,
                                       dim3(kBlock), 0, s, frames, stride, frame_len, n, code,
                                       csum, flags, wb.split);
                else
                    hipLaunchKernelGGL((k_fixed_tx2<G, U, LOOP, WM_LINE_SC1, kWM>), grid,
                                       dim3(kBlock), 0, s, frames, stride, frame_len, n, code,
                                       csum, flags, wb.split);
                return hipGetLastError();
            }
        }
    }
    return launch_fixed_wm<G, U, COMPUTE, LOOP, EXT, K>(frames, stride, frame_len, n, code, csum,
                                                        flags, ext, s);
}

// (G, U) by frame size: G*16 B per load instruction of a group, U loads per lane.
constexpr u32 kSmallMaxFrames = 4u << 20;   // RX <= 64 B: one lane per frame up to here
template <bool COMPUTE, bool EXT>
static hipError_t dispatch_fixed(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                                 uint8_t* code, uint32_t* csum, u32 flags, const Ext& ext,
                                 hipStream_t s)
{
    const u32 chunks = (frame_len + 15) / 16;
    if (chunks <= 4) {
        // <= 64 B.  TX: 4 lanes per frame, whose sector write-back is one coalesced
        // 1 KiB store per wave, where one lane per frame scatters 64 sectors per
        // store instruction (74 us per 1M frames vs 21.8 us); more frames per group
        // only adds to the write tail (K = 2: 22.4 us, 8M frames 151 -> 161 us).
        if (COMPUTE)
            return launch_fixed<4, 1, COMPUTE, false, EXT>(frames, stride, frame_len, n, code,
                                                           csum, flags, ext, s);
        // Plain RX up to 4M frames: one lane per frame, plain loads (k_small):
        // 14.0 / 22.9 / 40.3 us per 1M / 2M / 4M frames after a cache scrub
        // against 16.2 / 31.2 / 51.6 us for 4 lanes and 2 frames per group
        // (round 4, tools/kbench 64, KB_SCRUB; warm the same).  Beyond 4M the
        // 64-B-strided loads of one lane per frame fall behind (8M: 108 vs
        // 94 us), so larger batches take the 4-lane, 2-frame groups.
        if (!EXT && n <= kSmallMaxFrames) {
            hipLaunchKernelGGL((k_small<false, false, kXCD>), dim3((n + kBlock - 1) / kBlock),
                               dim3(kBlock), 0, s, frames, stride, frame_len, n, code, csum,
                               flags);
            return hipGetLastError();
        }
        if (!EXT)
            return launch_fixed<4, 1, COMPUTE, false, EXT, 2>(frames, stride, frame_len, n, code,
                                                              csum, flags, ext, s);
        // RX with the extensions: one lane per frame (k_small_x), whose RSS hash
        // is 24 lookups in LDS nibble tables instead of a 4-lane bit split.
        hipLaunchKernelGGL((k_small_x<COMPUTE, kNT, kXCD>), dim3((n + kBlock - 1) / kBlock),
                           dim3(kBlock), 0, s, frames, stride, frame_len, n, code, csum, flags,
                           ext);
        return hipGetLastError();
    }
    if (chunks <= 8)   return launch_fixed<8, 1, COMPUTE, false, EXT>(frames, stride, frame_len, n, code, csum, flags, ext, s);
    if (chunks <= 16)  return launch_fixed<16, 1, COMPUTE, false, EXT>(frames, stride, frame_len, n, code, csum, flags, ext, s);
    if (chunks <= 32)  return launch_fixed<32, 1, COMPUTE, false, EXT>(frames, stride, frame_len, n, code, csum, flags, ext, s);
    if (chunks <= 64)  return launch_fixed<32, 2, COMPUTE, false, EXT>(frames, stride, frame_len, n, code, csum, flags, ext, s);
    if (chunks <= 96)  return launch_fixed<32, 3, COMPUTE, false, EXT>(frames, stride, frame_len, n, code, csum, flags, ext, s);
    if (chunks <= 128) return launch_fixed<64, 2, COMPUTE, false, EXT>(frames, stride, frame_len, n, code, csum, flags, ext, s);
    return launch_fixed<64, 4, COMPUTE, true, EXT>(frames, stride, frame_len, n, code, csum, flags, ext, s);
}

template <int G, int U, bool LOOP>
static hipError_t launch_step_gu(uint8_t* tx, uint64_t tx_stride, u32 tx_len, u32 ntx,
                                 uint8_t* tx_code, uint32_t* tx_csum, u32 tx_flags, uint8_t* rx,
                                 uint64_t rx_stride, u32 rx_len, u32 nrx, uint8_t* rx_code,
                                 u32 rx_flags, hipStream_t s)
{
    constexpr u32 FPB = kBlock / G;
    const u32 txb = ((ntx + FPB - 1) / FPB + 7) & ~7u;   // multiples of 8 (XCD order)
    const u32 rxb = ((nrx + FPB - 1) / FPB + 7) & ~7u;
    const dim3 grid(txb + rxb);
    const TxWb wb = tx_wb(tx_stride, ntx, tx_flags, FPB);
    // GCS_STEP_ORDER (A/B knob, read once): tx (default), rx, mix
    static const u32 order = [] {
        const char* e = std::getenv("GCS_STEP_ORDER");
        return !e ? 0u : std::strcmp(e, "rx") == 0 ? 1u : std::strcmp(e, "mix") == 0 ? 2u : 0u;
    }();
#define GCS_STEP_K(A_, B_, SPLIT_)                                                            \
    hipLaunchKernelGGL((k_fixed_step<G, U, LOOP, A_, B_>), grid, dim3(kBlock), 0, s, tx,       \
                       tx_stride, tx_len, ntx, tx_code, tx_csum, tx_flags, rx, rx_stride,     \
                       rx_len, nrx, rx_code, rx_flags, txb, SPLIT_, rxb, order)
    switch (wb.mode) {
    case 1: GCS_STEP_K(WM_LINE_SC1, WM_LINE_SC1, txb); break;
    case 2: GCS_STEP_K(WM_LINE_SC1, WM_SECTOR_NT, wb.split); break;
    case 3: GCS_STEP_K(WM_LINE_SC1, kWM, wb.split); break;
    default: GCS_STEP_K(kWM, kWM, 0u); break;
    }
#undef GCS_STEP_K
    return hipGetLastError();
}

// The (G, U) shape dispatch_fixed picks for frames of `chunks` 16 B chunks
// (0: <= 64 B, the one-lane / 4-lane kernels).
static int fixed_shape(u32 chunks)
{
    return chunks <= 4 ? 0 : chunks <= 8 ? 1 : chunks <= 16 ? 2 : chunks <= 32 ? 3
         : chunks <= 64 ? 4 : chunks <= 96 ? 5 : chunks <= 128 ? 6 : 7;
}

hipError_t launch_step_fixed(uint8_t* tx, uint64_t tx_stride, u32 tx_len, u32 ntx,
                             uint8_t* tx_code, uint32_t* tx_csum, u32 tx_flags, uint8_t* rx,
                             uint64_t rx_stride, u32 rx_len, u32 nrx, uint8_t* rx_code,
                             u32 rx_flags, hipStream_t s)
{
    const int sh = fixed_shape((tx_len + 15) / 16);
    // one launch when both batches take the same plain kernel shape; else
    // (ICMP extensions, different shapes, frames <= 64 B) the two launches
    // it stands for
    if (ntx == 0 || nrx == 0 || sh == 0 || sh != fixed_shape((rx_len + 15) / 16) ||
        (tx_flags & GCS_CF_ICMP) || (rx_flags & GCS_VF_ICMP)) {
        hipError_t e = ntx ? launch_compute_fixed(tx, tx_stride, tx_len, ntx, tx_code, tx_csum,
                                                  tx_flags, s)
                           : hipSuccess;
        if (e != hipSuccess || nrx == 0)
            return e;
        return launch_verify_fixed(rx, rx_stride, rx_len, nrx, rx_code, rx_flags, s);
    }
#define GCS_STEP(G_, U_, L_)                                                                      \
    return launch_step_gu<G_, U_, L_>(tx, tx_stride, tx_len, ntx, tx_code, tx_csum, tx_flags, rx, \
                                      rx_stride, rx_len, nrx, rx_code, rx_flags, s)
    switch (sh) {
    case 1: GCS_STEP(8, 1, false);
    case 2: GCS_STEP(16, 1, false);
    case 3: GCS_STEP(32, 1, false);
    case 4: GCS_STEP(32, 2, false);
    case 5: GCS_STEP(32, 3, false);
    case 6: GCS_STEP(64, 2, false);
    default: GCS_STEP(64, 4, true);
    }
#undef GCS_STEP
}

hipError_t launch_verify_fixed(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                               uint8_t* verdict, u32 flags, hipStream_t s)
{
    if (flags & GCS_VF_ICMP)
        return dispatch_fixed<false, true>(frames, stride, frame_len, n, verdict, nullptr, flags,
                                           Ext{}, s);
    return dispatch_fixed<false, false>(frames, stride, frame_len, n, verdict, nullptr, flags,
                                        Ext{}, s);
}

hipError_t launch_compute_fixed(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                                uint8_t* status, uint32_t* csums, u32 flags, hipStream_t s)
{
    if (flags & GCS_CF_ICMP)
        return dispatch_fixed<true, true>(frames, stride, frame_len, n, status, csums, flags,
                                          Ext{}, s);
    return dispatch_fixed<true, false>(frames, stride, frame_len, n, status, csums, flags, Ext{},
                                       s);
}

hipError_t launch_classify_fixed(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                                 uint8_t* verdict, u32 flags, const Ext& ext, hipStream_t s)
{
    return dispatch_fixed<false, true>(frames, stride, frame_len, n, verdict, nullptr, flags, ext,
                                       s);
}

// The shipped prefix-sum stream (k_desc_stream; tools/kbench.hip imix, DESIGN.md
// §4): 8 chunks per lane per trip, block regions up to 12,288 chunks (192 KiB per
// 256 frames; C3 blocks span ~91 KiB), NT loads.  TX stashes chunks 0..3 (the
// sector written back, sc1 stores: 340 vs 372 us interleaved against nt,
// kbench_imix_stream_wm*.log), RX chunks 0..2 (ihl = 5 fast frames; HDR3:
// 240.7-245.7 vs 249-255 us interleaved, kbench_imix_stream_h3*.log).  With the
// class passes out of the kernel both run 8 waves per SIMD (round 4).
// Both run 7 waves per SIMD: 72 VGPRs hold the per-frame path in k_desc's
// shape (verify 32 lanes x 3 chunks, fill 32 x 2, no spill), for blocks that do
// not stream (sparse descriptors such as 2 KiB mbuf rooms); at 8 waves only
// 64 x 1 fits.  Sparse 2 KiB rooms: verify 274 vs 402 us, fill 365 vs 448 us;
// packed C3 fill 333.8 vs 331.3 us at 8 waves (r04_kbench_*_tx7.log).
template <bool COMPUTE>
using StreamShip = std::conditional_t<COMPUTE, StreamShape<8, 8192, 7, 4, 32, 2>,
                                      StreamShape<8, 8192, 7, 3, 32, 3>>;
// passes per block region (blockIdx.y): 3 x 8,192 chunks hold 256 packed
// frames of up to 1,536 B; what a block has beyond them goes per frame
constexpr int kStreamPasses = 3;
// Frames one per room (GCS_VF_ROOMS / GCS_CF_ROOMS): k_desc<32, 3>, one group
// per frame, XCD-contiguous blocks, line write-back for fills of lines that fit
// the Infinity Cache.  1M x 1500 B in 2 KiB rooms: verify 240-243 us, fill
// 291-294 us against 278-281 / 363 us on the stream kernel's per-frame path;
// 2 or 4 frames per group (descriptors, or descriptors and loads, together;
// 92-140 VGPRs) and descriptors staged in LDS measured 257-340 / 301-388 us
// (profiles/r05/c2_rooms_k.jsonl).
template <bool COMPUTE>
static hipError_t launch_rooms(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                               const uint16_t* len, u32 n, uint8_t* code, uint32_t* csums,
                               u32 flags, hipStream_t s)
{
    constexpr int G = 32, U = 3, FPB = kBlock / G;
    const dim3 rg((n + FPB - 1) / FPB);
    if constexpr (COMPUTE) {
        if ((uint64_t)n * 128 <= line_wb_bytes() && !(flags & GCS_CF_SECTOR_WB)) {
            hipLaunchKernelGGL((k_desc<G, U, COMPUTE, kNT, WM_LINE_SC1, kXCD>), rg, dim3(kBlock),
                               0, s, frames, frames_bytes, off, len, n, code, csums, flags);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_desc<G, U, COMPUTE, kNT, kWM, kXCD>), rg, dim3(kBlock), 0, s, frames,
                       frames_bytes, off, len, n, code, csums, flags);
    return hipGetLastError();
}

template <bool COMPUTE>
static hipError_t launch_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                              const uint16_t* len, u32 n, uint8_t* code, uint32_t* csums,
                              u32 flags, bool ext_on, const Ext& ext, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    if (!ext_on && (flags & GCS_VF_ROOMS)) {
        static_assert(GCS_VF_ROOMS == GCS_CF_ROOMS, "one rooms bit");
        return launch_rooms<COMPUTE>(frames, frames_bytes, off, len, n, code, csums, flags, s);
    }
    const dim3 grid((n + kDescFrames - 1) / kDescFrames);
    static_assert(kDescFrames == kBlock, "one descriptor per thread");
    if (ext_on) {
        using S = DescShip<COMPUTE>;
        hipLaunchKernelGGL((k_desc_mixed_x<S, COMPUTE, kXCD, kDescOcc>), grid, dim3(kBlock), 0, s,
                           frames, frames_bytes, off, len, n, code, csums, flags, ext);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_desc_stream<StreamShip<COMPUTE>, COMPUTE, WM_SECTOR_SC1, kXCD>),
                       dim3(grid.x, kStreamPasses), dim3(kBlock), 0, s, frames, frames_bytes, off,
                       len, n, code, csums, flags);
    return hipGetLastError();
}

hipError_t launch_verify_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                              const uint16_t* len, u32 n, uint8_t* verdict, u32 flags,
                              hipStream_t s)
{
    return launch_desc<false>(frames, frames_bytes, off, len, n, verdict, nullptr, flags,
                              (flags & GCS_VF_ICMP) != 0, Ext{}, s);
}

hipError_t launch_compute_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                               const uint16_t* len, u32 n, uint8_t* status, uint32_t* csums,
                               u32 flags, hipStream_t s)
{
    return launch_desc<true>(frames, frames_bytes, off, len, n, status, csums, flags,
                             (flags & GCS_CF_ICMP) != 0, Ext{}, s);
}

hipError_t launch_classify_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                                const uint16_t* len, u32 n, uint8_t* verdict, u32 flags,
                                const Ext& ext, hipStream_t s)
{
    return launch_desc<false>(frames, frames_bytes, off, len, n, verdict, nullptr, flags, true,
                              ext, s);
}

hipError_t launch_icmp_fn(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off,
                          const uint16_t* len, u32 n, uint16_t* out, hipStream_t s)
{
    constexpr int G = 16, FPB = kBlock / G;
    hipLaunchKernelGGL((k_tcp_fn<G, false>), dim3((n + FPB - 1) / FPB), dim3(kBlock), 0, s, buf,
                       buf_bytes, off, len, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                       n, out);
    return hipGetLastError();
}

hipError_t launch_rss_fn(const uint32_t* sip, const uint32_t* dip, const uint16_t* sp,
                         const uint16_t* dp, u32 n, const Ext& ext, hipStream_t s)
{
    hipLaunchKernelGGL(k_rss_fn, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, sip, dip,
                       sp, dp, n, ext);
    return hipGetLastError();
}

hipError_t launch_copy_fill(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                            const uint16_t* len, const uint8_t* src, uint64_t src_bytes,
                            const uint64_t* src_off, u32 n, uint8_t* status, uint32_t* csums,
                            u32 flags, hipStream_t s)
{
    // 16 lanes x 6 chunks per frame (124 VGPRs, 4 waves per SIMD, no spills):
    // as fast as <32,3> at 6 waves, which spills (576-624 us per 1M x 1500 B).
    // Payload chunks leave with nt stores: 602 vs 625 us back to back, 627 vs
    // 625 interleaved (sc0 sc1: 621 / 616; tools/kbench copy, kbench_cf_wm*.log)
    constexpr int G = 16, U = 6, FPB = kBlock / G;
    hipLaunchKernelGGL((k_copy_fill<G, U, 1, WM_SECTOR_NT>), dim3((n + FPB - 1) / FPB),
                       dim3(kBlock), 0, s, frames,
                       frames_bytes, off, len, src, src_bytes, src_off, n, status, csums, flags);
    return hipGetLastError();
}

hipError_t launch_gro(const uint8_t* in, uint64_t in_bytes, const uint64_t* off,
                      const uint16_t* len, const uint8_t* verdict, u32 n, u32 window,
                      u32 max_len, uint8_t* out, uint64_t out_bytes, uint64_t* out_off,
                      uint16_t* out_len, uint32_t* head, hipStream_t s)
{
    // windows of <= 64 frames on the small-LDS instantiation: 1M x 1500 B in
    // runs of 8, 928 us (LDS-bound, 4 blocks per CU) -> 809 (89 VGPRs, 5 per
    // SIMD) -> 772 us (<= 80 VGPRs, 6 per SIMD) -> 687 us with phase D as one
    // stream over the window's output (FLAT; 53 VGPRs, 8 waves per SIMD; the
    // run-per-wave form 761 us on the same box) -> 671-674 us with the word-wise
    // continuation test and scanned chains (ACX; phases A-C 121 -> 90 us) ->
    // 646 us back to back with nt stores (678 interleaved behind other kernels,
    // where sc0 sc1 stores measured 655; plain 671-674 both ways) -> 648-650 us
    // both ways with waves 1-3 reading the window's input into the caches while
    // wave 0 parses (PF = 8 loads per lane in flight; tools/kbench lro)
    // (round 4's pipelined persistent form, wave 0 planning the next window
    // while waves 1-3 stream this one, measured 770-805 us against 650:
    // three streaming waves per block at 5 blocks per CU, 15 per CU, against
    // 32 here -- tools/attic/gro_pipe.hip, kbench lro)
    // (round 5, blocked A/B: descriptors synthesized instead of loaded 649 vs
    // 653 us, and wave 3 reading window blockIdx + 1024's descriptors and
    // header lines ahead 652 us: phase A's trips are hidden already.  The
    // interleaved runs' 25 us "gain" was the first variant of each round
    // running behind the D2D copy's write-back -- profiles/r05/kbench_blocked.log)
    // Windows of 65-256 frames (round 5): the FLAT form over the block
    // (WIDE), 1,024 threads so that two blocks per CU (52 KB of LDS each)
    // still stream with 32 waves: 1M x 1500 B in windows of 256, 670-672 us
    // against 860-870 us for round 2's run-per-wave k_gro<2, 256> (695 us at
    // 512 threads, 891 at 256; tools/kbench lro, profiles/r05/kbench_w256*.log).
    if (window <= 64)
        hipLaunchKernelGGL((k_gro<2, 64, 8, true, WM_SECTOR_NT, true, 8>),
                           dim3((n + window - 1) / window), dim3(kBlock), 0, s, in, in_bytes, off,
                           len, verdict, n, window, max_len, out, out_bytes, out_off, out_len,
                           head);
    else
        hipLaunchKernelGGL((k_gro<2, kGroW, 8, true, WM_SECTOR_NT, true, 0, kGroWideThreads>),
                           dim3((n + window - 1) / window), dim3(kGroWideThreads), 0, s, in,
                           in_bytes, off, len, verdict, n, window, max_len, out, out_bytes, out_off,
                           out_len, head);
    return hipGetLastError();
}

hipError_t launch_tcp_fn(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off,
                         const uint16_t* len, const uint32_t* saddr, const uint32_t* daddr,
                         u32 n, uint16_t* out, hipStream_t s)
{
    constexpr int G = 16, FPB = kBlock / G;
    hipLaunchKernelGGL((k_tcp_fn<G>), dim3((n + FPB - 1) / FPB), dim3(kBlock), 0, s, buf,
                       buf_bytes, off, len, saddr, daddr, n, out);
    return hipGetLastError();
}

hipError_t launch_ip_fn(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off,
                        const uint8_t* ihl, u32 n, uint16_t* out, hipStream_t s)
{
    hipLaunchKernelGGL(k_ip_fn, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, buf,
                       buf_bytes, off, ihl, n, out);
    return hipGetLastError();
}

}  // namespace gcs
