// gcs_device.h -- device-side building blocks of the gfx950 checksum kernels.
//
// Reference algorithm (derivation in DESIGN.md §3):
//   TCPCalcChecksum  mtcp/src/tcp_util.c:244-277  -- u32 sum of LE16 words, odd tail
//                    masked to its low byte (:262-263), + saddr/daddr halves,
//                    htons(len), htons(6); two-step fold; ~.
//   ip_fast_csum     io_engine/include/ps.h:66-95 -- x86 ADC chain over ihl dwords;
//                    for ihl<=4 the raw low 16 bits of dword 0 (:72-73).
//
// Both folds are evaluated as EXACT integer sums of 16-bit words split across
// lanes and added back together (no overflow: a 64 KiB segment sums to
// < 2^31), then folded once, so results are bit-identical to the sequential
// reference.  For ip_fast_csum with ihl>=5 the x86 ADC chain equals
// ~fold16(sum of the header's 16-bit words): the end-around-carry sum R of the
// dwords is congruent to that word sum mod 0xFFFF, is 0 only for an all-zero
// header, and the final `adcl $0` can never carry out (state (0xFFFFFFFF, CF=1)
// is unreachable from `addl`), so nothing is dropped.
//
// Layout: frames in HBM, each 16 B-aligned.  A frame is owned by a group of G
// lanes (G | 64); lane `sub` loads the 16 B chunks c = j*G + sub (j < U) with
// one global_load_dwordx4 each, so every load instruction of a group reads
// G*16 contiguous bytes (whole 128 B lines).  Each lane keeps three partial
// sums (IP header words; TCP segment words + pseudo header; one extra field),
// the group all-reduces them on DPP, and the group applies the reference's
// verdict order.  No LDS tiles, no MFMA: an HBM-bound integer reduction.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtcp_gpucsum.h"

namespace gcs {

typedef uint32_t u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

// TX check-field write-back modes (A/B'd in tools/kbench.hip)
enum { WM_HALFWORD = 0,   // two 2-byte stores by the group leader
       WM_CHUNK = 1,      // the 16 B chunk(s) holding a check field, rewritten whole
       WM_SECTOR = 2,     // the 64 B sector(s) holding a check field, rewritten whole
       WM_SECTOR_NT = 3,  // ... with non-temporal stores
       WM_SECTOR_SC1 = 4, // ... with sc1 (write-through past the XCD L2) stores
       WM_LINE_SC1 = 5,   // the 128 B line(s) holding a check field, sc1 stores
       WM_CHUNK_SC1 = 6,  // WM_CHUNK with sc1 stores
       WM_SECTOR_SC01 = 7, // WM_SECTOR with sc0 sc1 (system scope) stores
       WM_LINE_NT = 8,     // WM_LINE_SC1 with non-temporal stores
       WM_LINE = 9         // WM_LINE_SC1 with plain stores
};

__host__ __device__ constexpr bool wm_line(int wm)
{
    return wm == WM_LINE_SC1 || wm == WM_LINE_NT || wm == WM_LINE;
}

__host__ __device__ constexpr bool wm_sc1(int wm)
{
    return wm == WM_SECTOR_SC1 || wm == WM_LINE_SC1 || wm == WM_CHUNK_SC1;
}

// ---------------------------------------------------------------------------
// scalar helpers

// acc + lo16(d) + hi16(d) in ONE VALU op: v_sad_u16(d, 0, acc) =
// |d.lo - 0| + |d.hi - 0| + acc.
__device__ __forceinline__ u32 sad(u32 d, u32 acc) { return __builtin_amdgcn_sad_u16(d, 0u, acc); }

__device__ __forceinline__ u32 hsum(u32 d) { return sad(d, 0u); }

__device__ __forceinline__ u32 sad4(uint4 v, u32 acc)
{
    return sad(v.w, sad(v.z, sad(v.y, sad(v.x, acc))));
}

__device__ __forceinline__ u32 hsum4(uint4 v) { return sad4(v, 0u); }

// byte mask keeping the low r bytes of a dword, r clamped to [0, 4]
__device__ __forceinline__ u32 low_mask(int r)
{
    r = r < 0 ? 0 : (r > 4 ? 4 : r);
    return (u32)((1ull << (8 * r)) - 1ull);
}

// two-step fold of tcp_util.c:271-272 (also what ps.h's addw/adcl produces)
__device__ __forceinline__ u32 fold16(u32 s)
{
    s = (s >> 16) + (s & 0xFFFFu);
    s += s >> 16;
    return s & 0xFFFFu;
}

__device__ __forceinline__ u32 csum16(u32 s) { return (~fold16(s)) & 0xFFFFu; }

__device__ __forceinline__ u32 bswap16(u32 v) { return ((v >> 8) & 0xFFu) | ((v & 0xFFu) << 8); }

// Mask of the 16-bit words of a dword at frame offset p (p % 4 == 0) that lie
// in [a, b), a even.  A word straddling b (b odd) keeps its low byte only: the
// reference's `*w & ntohs(0xFF00)` on a little-endian host.
__device__ __forceinline__ u32 region_mask(int p, int a, int b)
{
    u32 start = p >= a ? 0xFFFFFFFFu : (p + 2 >= a ? 0xFFFF0000u : 0u);
    return start & low_mask(b - p);
}

__device__ __forceinline__ u32 region_sum(u32 d, int p, int a, int b)
{
    return hsum(d & region_mask(p, a, b));
}

__device__ __forceinline__ u32 pick(uint4 v, int k)
{
    return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}

// Replace the high half of dword k of v by `hi16`.
__device__ __forceinline__ uint4 patch_hi(uint4 v, int k, u32 hi16)
{
    const u32 m = 0x0000FFFFu, s = hi16 << 16;
    v.x = k == 0 ? (v.x & m) | s : v.x;
    v.y = k == 1 ? (v.y & m) | s : v.y;
    v.z = k == 2 ? (v.z & m) | s : v.z;
    v.w = k == 3 ? (v.w & m) | s : v.w;
    return v;
}

// All-reduce (sum) inside aligned groups of G lanes.  Within a 16-lane row the
// butterfly runs on DPP (VALU only): quad_perm [1,0,3,2] and [2,3,0,1],
// row_half_mirror, row_mirror -- after the quad steps every lane of a quad
// holds the quad sum, so a mirror adds exactly the partner's sum.  The 16 ->
// 32 step is a ds_swizzle (xor 16, no LDS memory access), 32 -> 64 a bpermute.
template <int G>
__device__ __forceinline__ u32 group_sum(u32 x)
{
    if constexpr (G >= 2)
        x += (u32)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
    if constexpr (G >= 4)
        x += (u32)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
    if constexpr (G >= 8)
        x += (u32)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);
    if constexpr (G >= 16)
        x += (u32)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);
    if constexpr (G >= 32)
        x += (u32)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);
    if constexpr (G >= 64)
        x += __shfl_xor(x, 32, 64);
    return x;
}

// Inclusive prefix sum (u32, wrapping) over the 64 lanes of a wave, on DPP:
// row_shr 1/2/4/8 inside each 16-lane row, then row_bcast:15 (rows 1, 3) and
// row_bcast:31 (rows 2, 3).  A lane whose source lies outside its row, or a
// row the mask leaves out, adds `old` = 0.  Every lane must be active.
__device__ __forceinline__ u32 wave_incl_scan(u32 x)
{
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

// Sum of the LE 16-bit words of chunk v inside its first r bytes (r in
// [0, 16]); a word straddling r (r odd) keeps its low byte, the reference's
// odd-tail rule (tcp_util.c:262-263).
__device__ __forceinline__ u32 chunk_prefix_sum(uint4 v, int r)
{
    u32 s = hsum(v.x & low_mask(r));
    s = sad(v.y & low_mask(r - 4), s);
    s = sad(v.z & low_mask(r - 8), s);
    return sad(v.w & low_mask(r - 12), s);
}

// Value of lane SRC (< G) of this lane's G-group.
template <int G, int SRC>
__device__ __forceinline__ u32 group_bcast(u32 x)
{
    static_assert(SRC < G, "source lane inside the group");
    if constexpr (G == 4) {
        return (u32)__builtin_amdgcn_mov_dpp((int)x, SRC * 0x55, 0xF, 0xF, false);
    } else if constexpr (G <= 32) {
        // ds_swizzle bit mode: src lane = (lane & and_mask) | or_mask in a 32-lane half
        constexpr int and_mask = 0x1F & ~(G - 1);
        return (u32)__builtin_amdgcn_ds_swizzle((int)x, and_mask | (SRC << 5));
    } else {
        return __shfl(x, SRC, 64);
    }
}

// One global_load_dwordx4; NT adds the non-temporal (streaming) cache hint.
// Frames are always global memory (HBM or registered host memory); the cast to
// address space 1 makes that explicit, so a pointer the compiler cannot trace
// (one read from LDS or a request ring) still gets global_load, not flat_load
// (a flat op also waits on lgkmcnt and takes the aperture check).
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
typedef const __attribute__((address_space(1))) uint8_t gu8;

template <bool NT>
__device__ __forceinline__ uint4 ldg16(const uint8_t* p)
{
    gu32x4* q = (gu32x4*)(p);
    u32x4 r = NT ? __builtin_nontemporal_load(q) : *q;
    return make_uint4(r.x, r.y, r.z, r.w);
}

// A 2 B store into a frame (always global memory: global_store_short even
// where the compiler cannot trace the pointer, as in the burst server).
__device__ __forceinline__ void stg_u16(uint8_t* p, uint16_t v)
{
    *(__attribute__((address_space(1))) uint16_t*)(p) = v;
}

// One global_store_dwordx4 with the cache policy of write mode WM.
template <int WM>
__device__ __forceinline__ void stg16(uint8_t* p, uint4 v)
{
    u32x4 d = u32x4{v.x, v.y, v.z, v.w};
    if constexpr (WM == WM_SECTOR_NT || WM == WM_LINE_NT) {
        __builtin_nontemporal_store(d, reinterpret_cast<u32x4*>(p));
    } else if constexpr (wm_sc1(WM)) {
        // No result register, so nothing to wait for before the kernel ends; but
        // the trailing s_nop 1 is required: hipcc does not pad an asm store, and
        // its next instruction could overwrite the data VGPRs before the store
        // has read them (cdna_hip_programming.md §5.7 item 1).
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(d)
                     : "memory");
    } else if constexpr (WM == WM_SECTOR_SC01) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" : : "v"(p), "v"(d)
                     : "memory");
    } else {
        *reinterpret_cast<u32x4*>(p) = d;
    }
}

// 16-byte chunk load; `avail` = readable bytes from p (only checked when SAFE)
template <bool SAFE, bool NT>
__device__ __forceinline__ uint4 load_chunk(const uint8_t* p, int64_t avail)
{
    if (!SAFE || avail >= 16)
        return ldg16<NT>(p);
    uint8_t b[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        b[k] = (k < avail) ? ((gu8*)p)[k] : 0;
    uint4 v;
    v.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((u32)b[3] << 24);
    v.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((u32)b[7] << 24);
    v.z = b[8] | (b[9] << 8) | (b[10] << 16) | ((u32)b[11] << 24);
    v.w = b[12] | (b[13] << 8) | (b[14] << 16) | ((u32)b[15] << 24);
    return v;
}

// One global_load_lds_dwordx4 (LDS-DMA): lane l's 16 B from src land at LDS
// byte lds_dst + 16*l, lds_dst wave-uniform; no VGPR destination.  M0 is
// written and restored inside the statement (cdna_hip_programming.md §5.7,
// the LDS-DMA recipe).  hipcc does not count asm loads: wait with wait_vmcnt.
template <bool NT>
__device__ __forceinline__ void glds16(const uint8_t* src, u32 lds_dst)
{
    u32 keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
}

// s_waitcnt vmcnt(N) alone (gfx9 encoding: vmcnt in [3:0] and [15:14]).
template <int N>
__device__ __forceinline__ void wait_vmcnt()
{
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
    asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------------------
// per-frame work for one group of G lanes

struct Hdr {
    u32 d3, d4, d5;   // frame bytes 12..15, 16..19, 20..23
};

struct Acc {
    u32 ip;    // IP header words [14, 14+4*ihl)          (COMPUTE: minus iph->check)
    u32 tcp;   // TCP words [ts, te) + saddr/daddr halves (COMPUTE: minus tcph->check)
    u32 x;     // VERIFY: the byte holding tcph->doff
};

// Accumulate the chunk at frame offset cb.  ts = 14 + 4*ihl, te = 14 + tot_len.
template <bool COMPUTE>
__device__ __forceinline__ void accum_chunk(uint4 v, int cb, int ts, int te, Acc& a)
{
    if (cb >= ts && cb + 16 <= te) {          // interior of the TCP segment
        a.tcp = sad4(v, a.tcp);
    } else if (cb < ts || cb < te) {          // edge chunk: exact word masks
        int p = cb;
        a.ip = sad(v.x & region_mask(p, 14, ts), a.ip);
        a.ip = sad(v.y & region_mask(p + 4, 14, ts), a.ip);
        a.ip = sad(v.z & region_mask(p + 8, 14, ts), a.ip);
        a.ip = sad(v.w & region_mask(p + 12, 14, ts), a.ip);
        a.tcp = sad(v.x & region_mask(p, ts, te), a.tcp);
        a.tcp = sad(v.y & region_mask(p + 4, ts, te), a.tcp);
        a.tcp = sad(v.z & region_mask(p + 8, ts, te), a.tcp);
        a.tcp = sad(v.w & region_mask(p + 12, ts, te), a.tcp);
        if (cb == 16) {
            // pseudo header: saddr halves at 26, 28; daddr low half at 30
            a.tcp = sad(v.w, sad(v.z & 0xFFFF0000u, a.tcp));
            if (COMPUTE)
                a.ip -= v.z & 0xFFFFu;        // iph->check is 0 when folded (ip_out.c:153)
        } else if (cb == 32) {
            a.tcp += v.x & 0xFFFFu;           // daddr high half at 32
        }
    }
    // Fields at ihl-dependent offsets may sit in an interior chunk.
    if (COMPUTE) {
        int pc = ts + 14;                     // dword whose high half is tcph->check
        if (pc >= cb && pc < cb + 16 && pc + 4 <= te)
            a.tcp -= pick(v, (pc - cb) >> 2) >> 16;
    } else {
        int pd = ts + 10;                     // dword whose byte 2 is doff<<4 | res
        if (pd >= cb && pd < cb + 16)
            a.x += (pick(v, (pd - cb) >> 2) >> 16) & 0xFFu;
    }
}

// ihl == 5 (ts = 34), the header mTCP always emits (ip_out.c:72, :143): the
// word masks of chunks 0..3 are constants of the chunk index, so each lane
// computes them once.  ip = words [14, 34); tcp = words [34, te) plus the
// pseudo-header address halves at 26..33 (tcp_util.c:266-267); COMPUTE
// leaves out iph->check (bytes 24-25) and tcph->check (bytes 50-51).
struct Mask5 {
    u32 ip[4];
    u32 tcp[4];
};

template <bool COMPUTE>
__device__ __forceinline__ Mask5 masks5(int c)
{
    const u32 F = 0xFFFFFFFFu, H = 0xFFFF0000u, Lo = 0x0000FFFFu;
    Mask5 m;
    m.ip[0] = c == 2 ? Lo : (c == 1 ? F : 0u);               // 32-33 | 16-19
    m.ip[1] = c == 1 ? F : 0u;                                // 20-23
    m.ip[2] = c == 1 ? (COMPUTE ? H : F) : 0u;                // 24-27
    m.ip[3] = c == 1 ? F : (c == 0 ? H : 0u);                 // 28-31 | 14-15
    m.tcp[0] = c >= 2 ? ((COMPUTE && c == 3) ? Lo : F) : 0u;  // 32-35 ... 48-51
    m.tcp[1] = c >= 2 ? F : 0u;
    m.tcp[2] = c >= 2 ? F : (c == 1 ? H : 0u);                // 26-27 (saddr lo)
    m.tcp[3] = c >= 1 ? F : 0u;                               // 28-31 (saddr hi, daddr lo)
    return m;
}

// HDR: the chunk may be one of chunks 0..3 (masks m); otherwise it is a
// TCP-segment chunk (c >= 4) and only te limits it.
template <bool COMPUTE, bool HDR>
__device__ __forceinline__ void accum_fast5(uint4 v, int c, int te, const Mask5& m, Acc& a)
{
    const int cb = 16 * c;
    u32 t0 = HDR ? m.tcp[0] : 0xFFFFFFFFu, t1 = HDR ? m.tcp[1] : 0xFFFFFFFFu;
    // COMPUTE leaves out tcph->check only when the whole word lies in the
    // segment (te >= 52), exactly as accum_chunk does; the ICMP fill
    // (epilogue) relies on the two paths agreeing for short messages.
    if (COMPUTE && HDR && c == 3 && te < 52)
        t0 = 0xFFFFFFFFu;
    u32 t2 = HDR ? m.tcp[2] : 0xFFFFFFFFu, t3 = HDR ? m.tcp[3] : 0xFFFFFFFFu;
    if (HDR) {
        a.ip = sad(v.x & m.ip[0], a.ip);
        a.ip = sad(v.y & m.ip[1], a.ip);
        a.ip = sad(v.z & m.ip[2], a.ip);
        a.ip = sad(v.w & m.ip[3], a.ip);
        if (!COMPUTE && c == 2)
            a.x += (v.w >> 16) & 0xFFu;           // byte 46: doff << 4 | res
    }
    if (cb + 16 > te) {                           // the chunk holding the segment's end
        t0 &= low_mask(te - cb);
        t1 &= low_mask(te - cb - 4);
        t2 &= low_mask(te - cb - 8);
        t3 &= low_mask(te - cb - 12);
    }
    a.tcp = sad(v.x & t0, a.tcp);
    a.tcp = sad(v.y & t1, a.tcp);
    a.tcp = sad(v.z & t2, a.tcp);
    a.tcp = sad(v.w & t3, a.tcp);
}

// ---------------------------------------------------------------------------
// Extensions: the ICMP fold and RSS steering.

// Per-frame extension outputs; pointers already offset to this frame.
struct XFrame {
    u32 key[4];                // RSS key bits 0..127, big-endian words (rss.c:19-40)
    uint32_t* hash;            // this frame's RSS outputs (nullable)
    uint16_t* queue;
    u32 nq, nq_magic, endian;  // GetRSSCPUCore mapping; nq_magic = ceil(2^32 / nq)
    const u32* nib;            // one-lane groups: LDS nibble tables (rss_nibble_tables)
};

// The 16-bit word at frame byte b (b even) if this lane loaded it, else 0.
// Every word of the first G*U chunks is held by exactly one lane of the
// group, so a group_sum of the results is that word.
template <int G, int U>
__device__ __forceinline__ u32 held_hw(const uint4 (&v)[U], int sub, int b)
{
    const int c = b >> 4;
    u32 d = 0;
#pragma unroll
    for (int j = 0; j < U; j++)
        d = (c == j * G + sub) ? pick(v[j], (b >> 2) & 3) : d;
    return (b & 2) ? (d >> 16) : (d & 0xFFFFu);
}

template <int G>
__device__ __forceinline__ u32 group_xor(u32 x)
{
    if constexpr (G >= 2)
        x ^= (u32)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
    if constexpr (G >= 4)
        x ^= (u32)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
    if constexpr (G >= 8)
        x ^= (u32)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);
    if constexpr (G >= 16)
        x ^= (u32)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);
    if constexpr (G >= 32)
        x ^= (u32)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);
    if constexpr (G >= 64)
        x ^= __shfl_xor(x, 32, 64);
    return x;
}

// The 32 key bits starting at bit i (BuildKeyCache's cache[i], rss.c:27-40):
// a funnel shift of two key words (v_alignbit).
__device__ __forceinline__ u32 key_window(const u32 (&K)[4], int i)
{
    const int w = i >> 5, s = i & 31;
    const u32 hi = w == 0 ? K[0] : (w == 1 ? K[1] : K[2]);
    const u32 lo = w == 0 ? K[1] : (w == 1 ? K[2] : K[3]);
    return (u32)((((uint64_t)hi << 32) | lo) >> (32 - s));
}

constexpr int kNibEntries = 24 * 16;

// For one-lane groups (k_small, k_rss_fn) every lane hashes its own frame, so
// the 96 bit-steps cannot be spread over idle lanes.  Instead the block
// builds, in LDS, the table of each input nibble's contribution: nib[p*16+v]
// = XOR of key windows 4p+t over the set bits t of v (MSB-first); a hash is
// then 24 LDS lookups.  Built from the key alone (no memory reads); every
// thread of the block must call this before its first lookup.
__device__ __forceinline__ void rss_nibble_tables(const u32 (&K)[4], u32* nib)
{
    for (int e = threadIdx.x; e < kNibEntries; e += blockDim.x) {
        const int p = e >> 4, v = e & 15;
        u32 h = 0;
#pragma unroll
        for (int t = 0; t < 4; t++)
            h ^= ((v >> (3 - t)) & 1) ? key_window(K, 4 * p + t) : 0u;
        nib[e] = h;
    }
    __syncthreads();
}

// GetRSSHash (rss.c:44-86) of the host-order tuple words T0 = sip, T1 = dip,
// T2 = sp << 16 | dp (uniform in the group): input bit i (MSB-first) selects
// key window i.  The 96 bits are split over the group's lanes (lane sub takes
// i = sub, sub + G, ...) and XOR-reduced on DPP: no memory, a few VALU ops
// per lane.
template <int G>
__device__ __forceinline__ u32 rss_hash(const u32 (&K)[4], u32 T0, u32 T1, u32 T2, int sub,
                                        const u32* nib = nullptr)
{
    if constexpr (G == 1) {
        u32 h = 0;
#pragma unroll
        for (int p = 0; p < 24; p++) {
            const u32 word = p < 8 ? T0 : (p < 16 ? T1 : T2);
            h ^= nib[p * 16 + ((word >> (28 - 4 * (p & 7))) & 15u)];
        }
        return h;
    }
    constexpr int M = (96 + G - 1) / G;
    u32 h = 0;
#pragma unroll
    for (int m = 0; m < M; m++) {
        const int i = sub + G * m;
        const u32 word = i < 32 ? T0 : (i < 64 ? T1 : T2);
        const u32 bit = (word >> (31 - (i & 31))) & 1u;
        h ^= (bit && i < 96) ? key_window(K, i) : 0u;
    }
    return group_xor<G>(h);
}

// GetRSSCPUCore's mapping (rss.c:97-115) of hash h: i40e (endian) takes 9
// bits plus {3,1,-1,-3}[m & 3], ixgbe / mlx 7 bits; then % nq, as
// m - nq * umulhi(m, ceil(2^32 / nq)) (exact: m < 2^10, nq < 2^16).
__device__ __forceinline__ u32 rss_queue(const XFrame& x, u32 h)
{
    u32 m;
    if (x.endian) {
        m = h & 0x1FFu;
        const u32 r = m & 3u;
        m += r == 0 ? 3u : (r == 1 ? 1u : (r == 2 ? 0xFFFFFFFFu : 0xFFFFFFFDu));
    } else {
        m = h & 0x7Fu;
    }
    return x.nq == 1 ? 0u : m - x.nq * __umulhi(m, x.nq_magic);
}

// Verdict for one frame, in the reference's order.  EXT with GCS_VF_ICMP:
// IPv4 ICMP frames get the verdict of ICMPChecksum (icmp.c:89), whose sum
// over [ts, te) is `icmp`.
template <bool EXT = false>
__device__ __forceinline__ u32 rx_verdict(const Hdr& h, const Acc& a, u32 len, bool desc_ok,
                                          u32 flags = 0, u32 icmp = 0)
{
    if (!desc_ok) return GCS_V_BAD_DESC;
    if (len < 14) return GCS_V_DROP_TRUNC;
    if ((h.d3 & 0xFFFFu) != 0x0008u) return GCS_V_NOT_IPV4;         // eth_in.c:35
    if (len < 34) return GCS_V_DROP_TRUNC;
    u32 vihl = (h.d3 >> 16) & 0xFFu;
    u32 ihl = vihl & 15u, version = vihl >> 4;
    u32 tot = bswap16(h.d4 & 0xFFFFu);
    u32 proto = h.d5 >> 24;
    if (tot < 20) return GCS_V_DROP_IPLEN;                          // ip_in.c:25
    if (ihl >= 5 && 14 + 4 * ihl > len) return GCS_V_DROP_TRUNC;
    u32 ipc = ihl <= 4 ? (h.d3 >> 16) : csum16(a.ip);               // ps.h:72-73 quirk
    if (ipc != 0) return GCS_V_DROP_IPCSUM;                          // ip_in.c:35
    if (version != 4) return GCS_V_NOT_V4;                           // ip_in.c:47
    if (EXT && proto == 1 && (flags & GCS_VF_ICMP)) {                // ip_in.c:56
        if (tot < 4 * ihl) return GCS_V_ICMP_BADCSUM;                 // folds nothing: 0xFFFF
        if (14 + tot > len) return GCS_V_DROP_TRUNC;
        return csum16(icmp) != 0 ? GCS_V_ICMP_BADCSUM : GCS_V_ICMP_OK; // icmp.c:89-91
    }
    if (proto != 6) return GCS_V_NOT_TCP;                            // ip_in.c:52-59
    u32 ts = 14 + 4 * ihl;
    if (ts + 13 > len) return GCS_V_DROP_TRUNC;
    u32 doff = a.x >> 4;
    if (tot < 4 * (ihl + doff)) return GCS_V_DROP_TCPLEN;            // tcp_in.c:1221
    if (14 + tot > len) return GCS_V_DROP_TRUNC;
    u32 s = a.tcp + bswap16((tot - 4 * ihl) & 0xFFFFu) + 0x0600u;    // tcp_util.c:266-269
    return csum16(s) != 0 ? GCS_V_DROP_TCPCSUM : GCS_V_ACCEPT;        // tcp_in.c:1231-1239
}

// Replace the low half of dword k of v by `lo16`.
__device__ __forceinline__ uint4 patch_lo(uint4 v, int k, u32 lo16)
{
    const u32 m = 0xFFFF0000u;
    v.x = k == 0 ? (v.x & m) | lo16 : v.x;
    v.y = k == 1 ? (v.y & m) | lo16 : v.y;
    v.z = k == 2 ? (v.z & m) | lo16 : v.z;
    v.w = k == 3 ? (v.w & m) | lo16 : v.w;
    return v;
}

// Group reduction, then the verdict (RX) or the check-field fill (TX).
// `v` holds this lane's chunks c = j*G + sub of the frame's FIRST U*G chunks
// (the check fields always lie in chunks 1..5); `active` = false for padding
// groups, which take part in the cross-lane steps but write nothing.
// EXT adds the ICMP fold (GCS_VF_ICMP / GCS_CF_ICMP) and RSS steering: the
// tuple words are gathered from the lanes holding them (held_hw).  `wlim` =
// bytes writable from f: a whole-chunk write-back never goes past it (a frame
// ending at a buffer end that is not 16 B-aligned gets halfword stores).
template <int G, int U, bool COMPUTE, int WM, bool EXT = false>
__device__ __forceinline__ void epilogue(const Hdr& h, Acc a, uint8_t* __restrict__ f, u32 len,
                                         int64_t wlim, bool desc_ok, int sub, u32 flags,
                                         uint8_t* __restrict__ out_code,
                                         uint32_t* __restrict__ out_csum, bool active,
                                         const uint4 (&v)[U], const XFrame& xf = XFrame{},
                                         uint8_t* stage = nullptr)
{
    const u32 ihl = (h.d3 >> 16) & 15u;
    const u32 ts = 14 + 4 * ihl;
    // EXT: g_sip / g_dip / g_l4 = the wire bytes 26..29, 30..33, ts..ts+3 as
    // LE dwords (ICMP: type, code, checksum); g_tc = the word at ts+16.
    a.ip = group_sum<G>(a.ip);
    a.tcp = group_sum<G>(a.tcp);
    if (!COMPUTE)
        a.x = group_sum<G>(a.x);
    u32 g_sip = 0, g_dip = 0, g_l4 = 0, g_tc = 0, rh = 0;
    if constexpr (EXT) {
        static_assert(GCS_VF_ICMP == GCS_CF_ICMP, "one ICMP flag bit for RX and TX");
        // wave-uniform: the tuple is gathered only when RSS is on (kernel-
        // uniform) or an ICMP frame is in this wave
        const bool want_rss = !COMPUTE && (xf.hash || xf.queue);
        const bool want_icmp = (flags & GCS_VF_ICMP) && __any(active && (h.d5 >> 24) == 1u);
        // ihl == 5 in every frame of the wave: the tuple sits at fixed places,
        // chunk 1 dwords 2-3 and chunk 2 dwords 0-1 (bytes 24..39), the TCP
        // check's word at chunk 3 -- held by group lanes 1, 2, 3: four lane
        // reads instead of the held_hw selects and group sums
        bool fast = false;
        if constexpr (G >= 4)
            fast = (want_rss || want_icmp) && __all(!active || ihl == 5u);
        if (fast) {
            if constexpr (G >= 4) {
                const u32 c1z = group_bcast<G, 1>(v[0].z), c1w = group_bcast<G, 1>(v[0].w);
                const u32 c2x = group_bcast<G, 2>(v[0].x), c2y = group_bcast<G, 2>(v[0].y);
                g_sip = (c1z >> 16) | (c1w << 16);          // bytes 26..29
                g_dip = (c1w >> 16) | (c2x << 16);          // bytes 30..33
                g_l4 = (c2x >> 16) | (c2y << 16);           // bytes 34..37
                if (COMPUTE)
                    g_tc = group_bcast<G, 3>(v[0].x) >> 16; // bytes 50..51
            }
        } else if (want_rss || want_icmp) {
            g_sip = held_hw<G, U>(v, sub, 26) | (held_hw<G, U>(v, sub, 28) << 16);
            g_dip = held_hw<G, U>(v, sub, 30) | (held_hw<G, U>(v, sub, 32) << 16);
            g_l4 = held_hw<G, U>(v, sub, (int)ts) | (held_hw<G, U>(v, sub, (int)ts + 2) << 16);
            g_sip = group_sum<G>(g_sip);
            g_dip = group_sum<G>(g_dip);
            g_l4 = group_sum<G>(g_l4);
            if (COMPUTE)
                g_tc = group_sum<G>(held_hw<G, U>(v, sub, (int)ts + 16));
        }
        if (want_rss)
            rh = rss_hash<G>(xf.key, __builtin_bswap32(g_sip), __builtin_bswap32(g_dip),
                             __builtin_bswap32(g_l4), sub, xf.nib);
    }
    if (!active)
        return;
    // a.tcp less the pseudo-header address halves: the plain word sum over
    // [ts, te) that ICMPChecksum folds (no pseudo header, icmp.c:18-42).
    const u32 l4sum = EXT ? a.tcp - hsum(g_sip) - hsum(g_dip) : 0u;

    if (!COMPUTE) {
        if (sub != 0)
            return;
        u32 vd = rx_verdict<EXT>(h, a, len, desc_ok, flags, l4sum);
        if (vd == GCS_V_DROP_TCPCSUM && (flags & GCS_VF_ZERO_BAD_TCP_CHECK) && ts + 18u <= len)
            stg_u16(f + ts + 16, 0);         // tcp_in.c:1237
        out_code[0] = (uint8_t)vd;
        if constexpr (EXT) {
            const bool acc = vd == GCS_V_ACCEPT;
            if (xf.hash)
                *xf.hash = acc ? rh : 0u;
            if (xf.queue)
                *xf.queue = (uint16_t)(acc ? rss_queue(xf, rh) : 0xFFFFu);
        }
        return;
    }
    // TX fill: ip_out.c:143-173, tcp_out.c:244, 323-333; EXT + GCS_CF_ICMP:
    // icmp.c:57-69.  Every lane of the group evaluates the (uniform) status so
    // that WM_CHUNK / WM_SECTOR can rewrite whole chunks from the lanes that
    // hold them.
    u32 st, ipc = 0, l4c = 0;
    if (!desc_ok) {
        st = GCS_TX_BAD_DESC;
    } else if (len < 14 || (h.d3 & 0xFFFFu) != 0x0008u) {
        st = GCS_TX_NOT_IPV4;
    } else if (len < 34 || ihl < 5 || 14u + 4u * ihl > len) {
        st = GCS_TX_BAD_HDR;
    } else {
        u32 tot = bswap16(h.d4 & 0xFFFFu);
        const u32 proto = h.d5 >> 24;
        ipc = csum16(a.ip);
        if (proto == 6) {
            if (tot < 4u * ihl + 20u || 14u + tot > len) {
                st = GCS_TX_BAD_TCPLEN;
            } else {
                l4c = csum16(a.tcp + bswap16((tot - 4 * ihl) & 0xFFFFu) + 0x0600u);
                st = GCS_TX_OK;
            }
        } else if (EXT && proto == 1 && (flags & GCS_CF_ICMP)) {
            if (tot < 4u * ihl + 8u || 14u + tot > len) {
                st = GCS_TX_BAD_ICMPLEN;
            } else {
                // the accumulation left out the word at ts+16 (the TCP check's
                // place) when it lies in the message: add it back; the ICMP
                // check itself (ts+2) counts as zero (icmp.c:60)
                const u32 te = 14u + tot;
                const u32 s = l4sum + (ts + 18u <= te ? g_tc : 0u) - (g_l4 >> 16);
                l4c = csum16(s);
                st = GCS_TX_ICMP_OK;
            }
        } else {
            st = GCS_TX_IP_ONLY;
        }
    }
    const bool wip = st == GCS_TX_OK || st == GCS_TX_IP_ONLY || st == GCS_TX_BAD_TCPLEN ||
                     (EXT && (st == GCS_TX_ICMP_OK || st == GCS_TX_BAD_ICMPLEN));
    const bool wtcp = st == GCS_TX_OK;
    const bool wicmp = EXT && st == GCS_TX_ICMP_OK;
    if (!(flags & GCS_CF_NO_INPLACE) && wip) {
        if constexpr (WM == WM_HALFWORD) {
            if (sub == 0) {
                stg_u16(f + 24, (uint16_t)ipc);
                if (wtcp)
                    stg_u16(f + ts + 16, (uint16_t)l4c);
                if (wicmp)
                    stg_u16(f + ts + 2, (uint16_t)l4c);
            }
        } else {
            const int nchunks = (int)((len + 15) >> 4);
            // the buffer-end test in 32 bits (chunks c < 8 here): no 64-bit
            // invariant for it stays live across k_gro's batch loop (5 -> 3
            // spilled VGPRs there; the same speed)
            const int wl = wlim > 256 ? 256 : (int)wlim;
            const int ctcp = (int)(ts + 16) >> 4;            // chunk holding tcph->check
            const int cicmp = (int)(ts + 2) >> 4;            // chunk holding icmph->checksum
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int c = j * G + sub;
                if (j * G >= 8 || c >= nchunks || c >= 8)
                    continue;
                const bool has_ip = c == 1;
                const bool has_tcp = wtcp && c == ctcp;
                const bool has_icmp = wicmp && c == cicmp;
                const bool take = (WM == WM_CHUNK || WM == WM_CHUNK_SC1)
                                      ? (has_ip || has_tcp || has_icmp)
                                      : wm_line(WM)
                                      ? true                       // c < 8: line 0 holds all
                                      : ((c >> 2) == 0 || (wtcp && (c >> 2) == (ctcp >> 2)) ||
                                         (wicmp && (c >> 2) == (cicmp >> 2)));
                if (!take)
                    continue;
                if (16 * c + 16 > wl) {                      // chunk crosses the buffer end
                    if (has_ip)
                        stg_u16(f + 24, (uint16_t)ipc);
                    if (has_tcp)
                        stg_u16(f + ts + 16, (uint16_t)l4c);
                    if (has_icmp)
                        stg_u16(f + ts + 2, (uint16_t)l4c);
                    continue;
                }
                uint4 w = v[j];
                if (has_ip)
                    w.z = (w.z & 0xFFFF0000u) | ipc;                 // bytes 24..25
                if (has_tcp)
                    w = patch_hi(w, (int)((ts + 14) >> 2) & 3, l4c); // bytes ts+16..17
                if (has_icmp)
                    w = patch_lo(w, (int)((ts + 2) >> 2) & 3, l4c);  // bytes ts+2..3
                if (stage != nullptr && c < 4)                      // sector 0 staged in LDS
                    *reinterpret_cast<uint4*>(stage + 16 * c) = w;
                else
                    stg16<WM>(f + 16 * c, w);
            }
        }
    }
    if (sub == 0) {
        if (out_code)
            out_code[0] = (uint8_t)st;
        if (out_csum)
            out_csum[0] = ipc | (l4c << 16);
    }
}

// One frame per group: load, broadcast the header words, accumulate, epilogue.
// LOOP: frames longer than G*U chunks are walked in further batches (the
// first batch is kept for the TX write-back).  `active` = false: a padding
// group of a block-uniform loop -- it loads nothing and writes nothing but
// still takes part in the wave's cross-lane steps.
template <int G, int U, bool SAFE, bool NT>
__device__ __forceinline__ void load_first(const uint8_t* __restrict__ f, int nchunks,
                                           int64_t avail, int sub, uint4 (&v)[U])
{
#pragma unroll
    for (int j = 0; j < U; j++) {
        int c = j * G + sub;
        v[j] = c < nchunks ? load_chunk<SAFE, NT>(f + 16 * c, avail - 16 * c)
                           : make_uint4(0, 0, 0, 0);
    }
}

// The frame's first U*G chunks are already in v (load_first); `wf` is where
// the TX write-back goes (normally f).
template <int G, int U, bool COMPUTE, bool LOOP, bool SAFE, bool NT, int WM, bool EXT = false>
__device__ __forceinline__ void frame_body(const uint4 (&v)[U], uint8_t* __restrict__ f,
                                           uint8_t* __restrict__ wf, u32 len, int64_t avail,
                                           bool desc_ok, int sub, u32 flags,
                                           uint8_t* __restrict__ out_code,
                                           uint32_t* __restrict__ out_csum, bool active,
                                           const XFrame& xf = XFrame{}, uint8_t* stage = nullptr)
{
    const int nchunks = (desc_ok && active) ? (int)((len + 15) >> 4) : 0;
    // header words: chunk 0 lives in group lane 0, chunk 1 in group lane 1 (j = 0)
    Hdr h;
    h.d3 = group_bcast<G, 0>(v[0].w);
    h.d4 = group_bcast<G, 1>(v[0].x);
    h.d5 = group_bcast<G, 1>(v[0].y);
    const int ts = 14 + 4 * (int)((h.d3 >> 16) & 15u);
    const int te = 14 + (int)bswap16(h.d4 & 0xFFFFu);

    Acc a = {0u, 0u, 0u};
    if (__all(ts == 34 || !active)) {         // wave-uniform: every frame has ihl == 5
        const Mask5 m = masks5<COMPUTE>(sub);
        accum_fast5<COMPUTE, true>(v[0], sub, te, m, a);
#pragma unroll
        for (int j = 1; j < U; j++)
            accum_fast5<COMPUTE, false>(v[j], j * G + sub, te, m, a);
    } else {
#pragma unroll
        for (int j = 0; j < U; j++)
            accum_chunk<COMPUTE>(v[j], 16 * (j * G + sub), ts, te, a);
    }
    if (LOOP && nchunks > G * U) {
        uint4 w[U];
        for (int base = G * U; base < nchunks; base += G * U) {
#pragma unroll
            for (int j = 0; j < U; j++) {
                int c = base + j * G + sub;
                w[j] = c < nchunks ? load_chunk<SAFE, NT>(f + 16 * c, avail - 16 * c)
                                   : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < U; j++)
                accum_chunk<COMPUTE>(w[j], 16 * (base + j * G + sub), ts, te, a);
        }
    }
    epilogue<G, U, COMPUTE, WM, EXT>(h, a, wf, len, avail, desc_ok, sub, flags, out_code, out_csum,
                                     active, v, xf, stage);
}

template <int G, int U, bool COMPUTE, bool LOOP, bool SAFE, bool NT, int WM, bool EXT = false>
__device__ __forceinline__ void do_frame(uint8_t* __restrict__ f, u32 len, int64_t avail,
                                         bool desc_ok, int sub, u32 flags,
                                         uint8_t* __restrict__ out_code,
                                         uint32_t* __restrict__ out_csum, bool active = true,
                                         const XFrame& xf = XFrame{})
{
    const int nchunks = (desc_ok && active) ? (int)((len + 15) >> 4) : 0;
    uint4 v[U];
    load_first<G, U, SAFE, NT>(f, nchunks, avail, sub, v);
    frame_body<G, U, COMPUTE, LOOP, SAFE, NT, WM, EXT>(v, f, f, len, avail, desc_ok, sub, flags,
                                                       out_code, out_csum, active, xf);
}

}  // namespace gcs
