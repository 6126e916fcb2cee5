// gcs_kernels.hip -- gfx950 (CDNA4) kernels for mTCP's software checksum path.
//
// Reference algorithm (see DESIGN.md for the full derivation):
//   TCPCalcChecksum  mtcp/src/tcp_util.c:244-277  -- u32 sum of LE16 words, odd tail
//                    masked to its low byte (:262-263), + saddr/daddr halves,
//                    htons(len), htons(6); two-step fold; ~.
//   ip_fast_csum     io_engine/include/ps.h:66-95 -- x86 ADC chain over ihl dwords;
//                    for ihl<=4 the raw low 16 bits of dword 0 (:72-73).
//
// Both folds are evaluated here as EXACT integer sums of 16-bit words split
// across lanes and added back together (no overflow: a 64 KiB segment sums to
// < 2^31), then folded once, so the result is bit-identical to the sequential
// reference.  For ip_fast_csum with ihl>=5 the x86 ADC chain equals
// ~fold16(sum of the header's 16-bit words): the end-around-carry sum R of the
// dwords is congruent to that word sum mod 0xFFFF, is 0 only for an all-zero
// header, and the final `adcl $0` can never carry out (state (0xFFFFFFFF, CF=1)
// is unreachable from `addl`), so nothing is dropped.
//
// Layout: a batch of frames in HBM, each frame 16 B-aligned.  A frame is owned
// by a group of G lanes (G | 64); lane `sub` of the group loads the 16 B chunks
// c = j*G + sub (j < U) with one global_load_dwordx4 each, so every load
// instruction of a group reads G*16 contiguous bytes (full 128 B lines).  Each
// lane keeps three partial sums (IP header words, TCP segment words + pseudo
// header, one "extra" field), the group reduces them with xor-shuffles, and the
// group's lane 0 applies the reference's verdict order and writes one byte.
// No LDS tiles, no MFMA: this is an HBM-bound integer reduction.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gcs_internal.h"

namespace gcs {

typedef uint32_t u32;

// ---------------------------------------------------------------------------
// scalar helpers

__device__ __forceinline__ u32 hsum(u32 d) { return (d & 0xFFFFu) + (d >> 16); }

__device__ __forceinline__ u32 hsum4(uint4 v)
{
    return hsum(v.x) + hsum(v.y) + hsum(v.z) + hsum(v.w);
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

// keep the low r bytes of d, r clamped to [0, 4]
__device__ __forceinline__ u32 keep_low(u32 d, int r)
{
    r = r < 0 ? 0 : (r > 4 ? 4 : r);
    return d & (u32)((1ull << (8 * r)) - 1ull);
}

// Sum of the 16-bit words of dword d (frame offset p, p % 4 == 0) that lie in
// [a, b), a even.  A word straddling b (b odd) contributes its low byte only:
// the reference's `*w & ntohs(0xFF00)` on a little-endian host.
__device__ __forceinline__ u32 region_sum(u32 d, int p, int a, int b)
{
    u32 t = keep_low(d, b - p);
    u32 lo = (p >= a) ? (t & 0xFFFFu) : 0u;
    u32 hi = (p + 2 >= a) ? (t >> 16) : 0u;
    return lo + hi;
}

__device__ __forceinline__ u32 pick(uint4 v, int k)
{
    return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}

template <int G>
__device__ __forceinline__ u32 group_sum(u32 x)
{
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1)
        x += __shfl_xor(x, m, G);
    return x;
}

// 16-byte chunk load; `avail` = readable bytes from p (only checked when SAFE)
template <bool SAFE>
__device__ __forceinline__ uint4 load_chunk(const uint8_t* p, int64_t avail)
{
    if (!SAFE || avail >= 16)
        return *reinterpret_cast<const uint4*>(p);
    uint8_t b[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        b[k] = (k < avail) ? p[k] : 0;
    uint4 v;
    v.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((u32)b[3] << 24);
    v.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((u32)b[7] << 24);
    v.z = b[8] | (b[9] << 8) | (b[10] << 16) | ((u32)b[11] << 24);
    v.w = b[12] | (b[13] << 8) | (b[14] << 16) | ((u32)b[15] << 24);
    return v;
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

// Accumulate chunk at frame offset cb.  ts = 14 + 4*ihl, te = 14 + tot_len.
template <bool COMPUTE>
__device__ __forceinline__ void accum_chunk(uint4 v, int cb, int ts, int te, Acc& a)
{
    if (cb >= ts && cb + 16 <= te) {          // interior of the TCP segment
        a.tcp += hsum4(v);
    } else if (cb < ts || cb < te) {          // edge chunk: exact word masks
        int p = cb;
        a.ip += region_sum(v.x, p, 14, ts) + region_sum(v.y, p + 4, 14, ts) +
                region_sum(v.z, p + 8, 14, ts) + region_sum(v.w, p + 12, 14, ts);
        a.tcp += region_sum(v.x, p, ts, te) + region_sum(v.y, p + 4, ts, te) +
                 region_sum(v.z, p + 8, ts, te) + region_sum(v.w, p + 12, ts, te);
        if (cb == 16) {
            // pseudo header: saddr halves at 26, 28; daddr low half at 30
            a.tcp += (v.z >> 16) + hsum(v.w);
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

// Verdict for one frame (group lane 0), in the reference's order.
__device__ __forceinline__ u32 rx_verdict(const Hdr& h, const Acc& a, u32 len, bool desc_ok)
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
    if (proto != 6) return GCS_V_NOT_TCP;                            // ip_in.c:52-59
    u32 ts = 14 + 4 * ihl;
    if (ts + 13 > len) return GCS_V_DROP_TRUNC;
    u32 doff = a.x >> 4;
    if (tot < 4 * (ihl + doff)) return GCS_V_DROP_TCPLEN;            // tcp_in.c:1221
    if (14 + tot > len) return GCS_V_DROP_TRUNC;
    u32 s = a.tcp + bswap16((tot - 4 * ihl) & 0xFFFFu) + 0x0600u;    // tcp_util.c:266-269
    return csum16(s) != 0 ? GCS_V_DROP_TCPCSUM : GCS_V_ACCEPT;        // tcp_in.c:1231-1239
}

template <int G, int U, bool COMPUTE, bool LOOP, bool SAFE>
__device__ __forceinline__ void do_frame(uint8_t* __restrict__ f, u32 len, int64_t avail,
                                         bool desc_ok, int sub, u32 flags,
                                         uint8_t* __restrict__ out_code,
                                         uint32_t* __restrict__ out_csum)
{
    const int nchunks = desc_ok ? (int)((len + 15) >> 4) : 0;
    uint4 v[U];
#pragma unroll
    for (int j = 0; j < U; j++) {
        int c = j * G + sub;
        v[j] = c < nchunks ? load_chunk<SAFE>(f + 16 * c, avail - 16 * c) : make_uint4(0, 0, 0, 0);
    }
    // header words: chunk 0 lives in group lane 0, chunk 1 in group lane 1 (j = 0)
    Hdr h;
    h.d3 = __shfl(v[0].w, 0, G);
    h.d4 = __shfl(v[0].x, 1, G);
    h.d5 = __shfl(v[0].y, 1, G);
    const int ihl = (h.d3 >> 16) & 15;
    const int ts = 14 + 4 * ihl;
    const int te = 14 + (int)bswap16(h.d4 & 0xFFFFu);

    Acc a = {0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < U; j++)
        accum_chunk<COMPUTE>(v[j], 16 * (j * G + sub), ts, te, a);
    if (LOOP) {
        for (int base = G * U; base < nchunks; base += G * U) {
#pragma unroll
            for (int j = 0; j < U; j++) {
                int c = base + j * G + sub;
                v[j] = c < nchunks ? load_chunk<SAFE>(f + 16 * c, avail - 16 * c)
                                   : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < U; j++)
                accum_chunk<COMPUTE>(v[j], 16 * (base + j * G + sub), ts, te, a);
        }
    }
    a.ip = group_sum<G>(a.ip);
    a.tcp = group_sum<G>(a.tcp);
    if (!COMPUTE)
        a.x = group_sum<G>(a.x);
    if (sub != 0)
        return;

    if (!COMPUTE) {
        u32 vd = rx_verdict(h, a, len, desc_ok);
        if (vd == GCS_V_DROP_TCPCSUM && (flags & GCS_VF_ZERO_BAD_TCP_CHECK) &&
            (u32)ts + 18u <= len)
            *reinterpret_cast<uint16_t*>(f + ts + 16) = 0;         // tcp_in.c:1237
        out_code[0] = (uint8_t)vd;
        return;
    }
    // TX fill: ip_out.c:143-173, tcp_out.c:244, 323-333
    u32 st, cs = 0;
    const bool inplace = !(flags & GCS_CF_NO_INPLACE);
    if (!desc_ok) {
        st = GCS_TX_BAD_DESC;
    } else if (len < 14 || (h.d3 & 0xFFFFu) != 0x0008u) {
        st = GCS_TX_NOT_IPV4;
    } else if (len < 34 || ihl < 5 || 14u + 4u * ihl > len) {
        st = GCS_TX_BAD_HDR;
    } else {
        u32 tot = (u32)(te - 14);
        u32 ipc = csum16(a.ip);
        if (inplace)
            *reinterpret_cast<uint16_t*>(f + 24) = (uint16_t)ipc;
        cs = ipc;
        if ((h.d5 >> 24) != 6) {
            st = GCS_TX_IP_ONLY;
        } else if (tot < 4u * ihl + 20u || 14u + tot > len) {
            st = GCS_TX_BAD_TCPLEN;
        } else {
            u32 s = a.tcp + bswap16((tot - 4 * ihl) & 0xFFFFu) + 0x0600u;
            u32 tcpc = csum16(s);
            if (inplace)
                *reinterpret_cast<uint16_t*>(f + ts + 16) = (uint16_t)tcpc;
            cs |= tcpc << 16;
            st = GCS_TX_OK;
        }
    }
    if (out_code)
        out_code[0] = (uint8_t)st;
    if (out_csum)
        out_csum[0] = cs;
}

// ---------------------------------------------------------------------------
// kernels

constexpr int kBlock = 256;

// Fixed stride: frame i at frames + i*stride, length frame_len, 16*ceil(len/16) <= stride.
template <int G, int U, bool COMPUTE, bool LOOP>
__global__ void __launch_bounds__(kBlock)
k_fixed(uint8_t* __restrict__ frames, uint64_t stride, u32 frame_len, u32 n,
        uint8_t* __restrict__ out_code, uint32_t* __restrict__ out_csum, u32 flags)
{
    constexpr int FPB = kBlock / G;                    // frames per block
    const int sub = threadIdx.x & (G - 1);
    const uint64_t i = (uint64_t)blockIdx.x * FPB + threadIdx.x / G;
    if (i >= n)
        return;                                        // whole group leaves together
    do_frame<G, U, COMPUTE, LOOP, false>(frames + i * stride, frame_len, (int64_t)stride, true,
                                         sub, flags, out_code ? out_code + i : nullptr,
                                         out_csum ? out_csum + i : nullptr);
}

// Descriptor batch: frame i at frames + off[i], length len[i].
template <int G, int U, bool COMPUTE>
__global__ void __launch_bounds__(kBlock)
k_desc(uint8_t* __restrict__ frames, uint64_t frames_bytes, const uint64_t* __restrict__ off,
       const uint16_t* __restrict__ lens, u32 n, uint8_t* __restrict__ out_code,
       uint32_t* __restrict__ out_csum, u32 flags)
{
    constexpr int FPB = kBlock / G;
    const int sub = threadIdx.x & (G - 1);
    const uint64_t i = (uint64_t)blockIdx.x * FPB + threadIdx.x / G;
    if (i >= n)
        return;
    const uint64_t o = off[i];
    const u32 len = lens[i];
    const bool ok = (o & 15) == 0 && o <= frames_bytes && len <= frames_bytes - o;
    uint8_t* f = frames + (ok ? o : 0);
    do_frame<G, U, COMPUTE, true, true>(f, len, ok ? (int64_t)(frames_bytes - o) : 0, ok, sub,
                                        flags, out_code ? out_code + i : nullptr,
                                        out_csum ? out_csum + i : nullptr);
}

// TCPCalcChecksum(buf + off[i], len[i], saddr[i], daddr[i]), G lanes per item.
template <int G>
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
        uint4 v = load_chunk<true>(buf + base + 16 * c, avail - 16 * c);
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
    const u32 sa = saddr[i], da = daddr[i];
    s += (sa & 0xFFFFu) + (sa >> 16) + (da & 0xFFFFu) + (da >> 16);   // tcp_util.c:266-267
    s += bswap16(len) + 0x0600u;                                       // :268-269
    out[i] = (uint16_t)csum16(s);
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

template <int G, int U, bool COMPUTE, bool LOOP>
static hipError_t launch_fixed(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                               uint8_t* code, uint32_t* csum, u32 flags, hipStream_t s)
{
    constexpr int FPB = kBlock / G;
    dim3 grid((n + FPB - 1) / FPB);
    hipLaunchKernelGGL((k_fixed<G, U, COMPUTE, LOOP>), grid, dim3(kBlock), 0, s, frames, stride,
                       frame_len, n, code, csum, flags);
    return hipGetLastError();
}

template <bool COMPUTE>
static hipError_t dispatch_fixed(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                                 uint8_t* code, uint32_t* csum, u32 flags, hipStream_t s)
{
    const u32 chunks = (frame_len + 15) / 16;
    if (chunks <= 4)   return launch_fixed<4, 1, COMPUTE, false>(frames, stride, frame_len, n, code, csum, flags, s);
    if (chunks <= 8)   return launch_fixed<8, 1, COMPUTE, false>(frames, stride, frame_len, n, code, csum, flags, s);
    if (chunks <= 16)  return launch_fixed<16, 1, COMPUTE, false>(frames, stride, frame_len, n, code, csum, flags, s);
    if (chunks <= 32)  return launch_fixed<32, 1, COMPUTE, false>(frames, stride, frame_len, n, code, csum, flags, s);
    if (chunks <= 64)  return launch_fixed<32, 2, COMPUTE, false>(frames, stride, frame_len, n, code, csum, flags, s);
    if (chunks <= 96)  return launch_fixed<32, 3, COMPUTE, false>(frames, stride, frame_len, n, code, csum, flags, s);
    if (chunks <= 128) return launch_fixed<64, 2, COMPUTE, false>(frames, stride, frame_len, n, code, csum, flags, s);
    return launch_fixed<64, 4, COMPUTE, true>(frames, stride, frame_len, n, code, csum, flags, s);
}

hipError_t launch_verify_fixed(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                               uint8_t* verdict, u32 flags, hipStream_t s)
{
    return dispatch_fixed<false>(frames, stride, frame_len, n, verdict, nullptr, flags, s);
}

hipError_t launch_compute_fixed(uint8_t* frames, uint64_t stride, u32 frame_len, u32 n,
                                uint8_t* status, uint32_t* csums, u32 flags, hipStream_t s)
{
    return dispatch_fixed<true>(frames, stride, frame_len, n, status, csums, flags, s);
}

constexpr int kDescG = 16, kDescU = 2;

hipError_t launch_verify_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                              const uint16_t* len, u32 n, uint8_t* verdict, u32 flags,
                              hipStream_t s)
{
    constexpr int FPB = kBlock / kDescG;
    hipLaunchKernelGGL((k_desc<kDescG, kDescU, false>), dim3((n + FPB - 1) / FPB), dim3(kBlock),
                       0, s, frames, frames_bytes, off, len, n, verdict, (uint32_t*)nullptr,
                       flags);
    return hipGetLastError();
}

hipError_t launch_compute_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                               const uint16_t* len, u32 n, uint8_t* status, uint32_t* csums,
                               u32 flags, hipStream_t s)
{
    constexpr int FPB = kBlock / kDescG;
    hipLaunchKernelGGL((k_desc<kDescG, kDescU, true>), dim3((n + FPB - 1) / FPB), dim3(kBlock),
                       0, s, frames, frames_bytes, off, len, n, status, csums, flags);
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
