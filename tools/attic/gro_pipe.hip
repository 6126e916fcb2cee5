// Measured, not shipped (round 4): LRO as a persistent pipelined kernel.  A
// block takes windows blockIdx.x, + gridDim.x, ...; wave 0 plans the next
// window (k_gro's phases A-D1) while waves 1-3 stream the current one.  It
// measured 770-805 us per 1M x 1500 B against the shipped k_gro FLAT's 650
// (kbench lro): three streaming waves per block at 5 blocks per CU leave 15
// streaming waves per CU against FLAT's 32.  Included by tools/kbench.hip
// after the product kernels (it uses their device helpers).
// LRO, pipelined (round 4; windows of <= 64 frames, as k_gro FLAT): a
// persistent block takes windows blockIdx.x, + gridDim.x, ...  Wave 0 PLANS
// the next window -- phases A-D1 of k_gro (headers into LDS, continuation,
// runs cut at max_len, run offsets, the output's segment table), all
// wave-local -- into the other of two plan buffers, while waves 1-3 STREAM
// the current one (D2: the window's output chunks as one stream, 3 waves)
// and then finish its merged runs (D3).  In k_gro a block's four waves sat
// in A-D1 (one dependent header trip, then LDS work: ~14% of a block's life)
// with nothing streaming but a prefetch; here the planning overlaps the
// stream of the previous window.  Same rules, same bytes (oracle/csum_ref.c
// ref_gro_batch; the NIC merge of dpdk_module.c:855-881).
namespace gcs {

constexpr int kPipeW = 64;                // frames per window (wave 0: one per lane)
constexpr int kPipeRows = 256;            // 64-chunk output rows with a start entry (256 KiB)

struct alignas(16) GroPlan {
    uint8_t hdr[kPipeW][kGroHdr];         // first 96 B of each frame
    int pay[kPipeW];                      // TCP payload bytes of a mergeable frame, else -1
    uint32_t pref[kPipeW];                // payload offset of a member within its run
    uint64_t soff[kPipeW];                // descriptors
    uint64_t run_off[kPipeW];             // runs: output offset, length, head, members
    uint32_t run_len[kPipeW];
    uint16_t run_t[kPipeW], run_n[kPipeW];
    uint16_t rhead[kPipeW], rn_at[kPipeW], ridx[kPipeW];
    uint32_t rl_at[kPipeW];
    uint8_t cont[kPipeW], dok[kPipeW];
    uint32_t sg_st[2 * kPipeW], sg_len[2 * kPipeW];   // the output's segments, in order
    uint64_t sg_src[2 * kPipeW];
    uint8_t sg_kind[2 * kPipeW], sg_run[2 * kPipeW];
    uint8_t sg_row[kPipeRows];            // segment holding each output row's first byte
    int cnt, nruns, nseg;
    uint32_t nout;                        // output bytes (runs at 16 B-aligned offsets)
    uint64_t o0;                          // the window's first input (= output) offset
};

// LDS writes of one lane read by another lane of the SAME wave: order them
// (one wave executes its LDS instructions in order; the fence keeps the
// compiler from moving them).
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Phases A-D1 of k_gro for window wi, by ONE wave (lane t = frame t).
__device__ void gro_plan(GroPlan& P, u32 wi, const uint8_t* __restrict__ in, uint64_t in_bytes,
                         const uint64_t* __restrict__ off, const uint16_t* __restrict__ lens,
                         const uint8_t* __restrict__ verdict, u32 n, u32 window, u32 max_len,
                         uint64_t* __restrict__ out_off, uint16_t* __restrict__ out_len,
                         uint32_t* __restrict__ head)
{
    const int t = threadIdx.x & 63;
    const uint64_t w0 = (uint64_t)wi * window;
    const int cnt = (int)min<uint64_t>(window, n - w0);
    const uint4 z = make_uint4(0, 0, 0, 0);
    // A: parse
    if (t < cnt) {
        const uint64_t o = off[w0 + t];
        const u32 L = lens[w0 + t];
        P.soff[t] = o;
        const bool ok = (o & 15) == 0 && o <= in_bytes && L <= in_bytes - o;
        const bool acc = ok && verdict[w0 + t] == GCS_V_ACCEPT;
        P.dok[t] = ok;
        uint4 v[kGroHdr / 16];
#pragma unroll
        for (int c = 0; c < kGroHdr / 16; c++)
            v[c] = acc ? load_chunk<true, false>(in + o + 16 * c, (int64_t)(in_bytes - o) - 16 * c)
                       : z;
#pragma unroll
        for (int c = 0; c < kGroHdr / 16; c++)
            *reinterpret_cast<uint4*>(&P.hdr[t][16 * c]) = v[c];
        const uint8_t* h = P.hdr[t];
        int p = -1;
        if (acc && (v[0].w & 0x000F0000u) == 0x00050000u)     // ihl == 5 (byte 14)
            p = (int)lds_be16(h + 16) - 20 - 4 * (h[46] >> 4);
        P.pay[t] = p;
    }
    if (t == 0) {
        P.cnt = cnt;
        P.o0 = cnt ? off[w0] : 0;
    }
    wave_sync();
    // B: continuation
    if (t < cnt)
        P.cont[t] = t > 0 && gro_cont32(P.hdr[t - 1], P.hdr[t], P.pay[t - 1], P.pay[t]);
    wave_sync();
    // C: runs.  A chain whose whole payload fits max_len is one run: its
    // members' payload offsets are a segmented scan of the wave; other chains
    // are cut greedily at max_len by their first lane (ref_gro_batch's walk).
    const bool valid = t < cnt, start = !valid || t == 0 || !P.cont[t];
    {
        const uint64_t sm = __ballot(start);
        const uint64_t upto = t == 63 ? ~0ull : ((2ull << t) - 1);
        const int sh = 63 - __clzll(sm & upto);                 // chain head
        const uint64_t above = sm & ~upto;
        const int se = above ? __ffsll((long long)above) - 2 : 63;   // chain's last lane
        const u32 pv = valid && P.pay[t] > 0 ? (u32)P.pay[t] : 0u;
        const u32 incl = wave_incl_scan(pv), excl = incl - pv;
        const u32 hx = (u32)__shfl((int)excl, sh, 64);
        const u32 tot = (u32)__shfl((int)incl, se, 64) - hx;      // the chain's payload
        const int hp = __shfl(valid ? P.pay[t] : -1, sh, 64);
        const u32 hhl = 34 + 4 * (P.hdr[sh][46] >> 4);
        const bool fits = hp > 0 && hhl + tot <= max_len;
        if (valid && fits) {
            P.pref[t] = excl - hx;
            P.rhead[t] = (uint16_t)sh;
            if (t == sh) {
                P.rn_at[t] = (uint16_t)(se - sh + 1);
                P.rl_at[t] = hhl + tot;
            }
        }
        if (!fits && valid && start) {
            int cur = t;
            u32 mlen = P.pay[t] > 0 ? 34 + 4 * (P.hdr[t][46] >> 4) + (u32)P.pay[t]
                                    : (P.dok[t] ? (u32)lens[w0 + t] : 0u);   // bad descriptor: nothing
            P.pref[t] = 0;
            P.rhead[t] = (uint16_t)t;
            P.rn_at[t] = 1;
            for (int k = t + 1; k < cnt && P.cont[k]; k++) {
                if (mlen + (u32)P.pay[k] <= max_len) {
                    P.pref[k] = mlen - (34 + 4 * (P.hdr[cur][46] >> 4));
                    mlen += (u32)P.pay[k];
                    P.rhead[k] = (uint16_t)cur;
                    P.rn_at[cur]++;
                    continue;
                }
                P.rl_at[cur] = mlen;                         // max_len cut: k heads a new run
                cur = k;
                mlen = 34 + 4 * (P.hdr[k][46] >> 4) + (u32)P.pay[k];
                P.pref[k] = 0;
                P.rhead[k] = (uint16_t)k;
                P.rn_at[k] = 1;
            }
            P.rl_at[cur] = mlen;
        }
    }
    wave_sync();
    // run numbers and 16 B-aligned output offsets: one wave scan
    const bool rs = valid && P.rhead[t] == t;
    const u32 rl = rs ? P.rl_at[t] : 0u;
    const u32 xs1 = rs ? 1u : 0u, xl1 = rs ? (rl + 15u) & ~15u : 0u;
    const u32 is = wave_incl_scan(xs1), il = wave_incl_scan(xl1);
    const u32 xs = is - xs1, xl = il - xl1;
    const uint64_t o0 = cnt ? off[w0] : 0;
    if (rs) {
        P.run_t[xs] = (uint16_t)t;
        P.run_n[xs] = P.rn_at[t];
        P.run_len[xs] = rl;
        P.run_off[xs] = o0 + xl;
        P.ridx[t] = (uint16_t)xs;
    }
    if (t == 63) {
        P.nruns = (int)is;
        P.nout = il;
    }
    wave_sync();
    if (valid) {
        const int hk = P.rhead[t];
        const int r = P.ridx[hk];
        head[w0 + t] = (uint32_t)(w0 + hk);
        out_off[w0 + t] = P.run_off[r];
        out_len[w0 + t] = hk == t ? (uint16_t)P.run_len[r] : (uint16_t)0;
    }
    // D1: the output as segments: a merged run's head headers (from LDS),
    // each member's payload, or a single frame as it is
    {
        int ns = 0, k0 = SEG_HDR;
        u32 st0 = 0, ln0 = 0, ln1 = 0;
        uint64_t sr0 = 0, sr1 = 0;
        int rr = 0;
        if (valid) {
            const int hk = P.rhead[t];
            rr = P.ridx[hk];
            const int nm = P.run_n[rr];
            const u32 rel = (u32)(P.run_off[rr] - o0);
            if (nm == 1) {
                if (P.run_len[rr] > 0) {
                    ns = 1;
                    k0 = SEG_WHOLE;
                    st0 = rel;
                    ln0 = P.run_len[rr];
                    sr0 = P.soff[t];
                }
            } else {
                const u32 hl = 34 + 4 * (P.hdr[hk][46] >> 4);
                if (t == hk) {
                    ns = 2;
                    k0 = SEG_HDR;
                    st0 = rel;
                    ln0 = hl;
                    sr0 = (uint64_t)hk;
                    ln1 = (u32)P.pay[t];
                    sr1 = P.soff[t] + hl;
                } else {
                    ns = 1;
                    k0 = SEG_PAY;
                    st0 = rel + hl + P.pref[t];
                    ln0 = (u32)P.pay[t];
                    sr0 = P.soff[t] + hl;
                }
            }
        }
        const u32 incl = wave_incl_scan((u32)ns);
        const int e = (int)(incl - (u32)ns);
        if (ns >= 1) {
            P.sg_st[e] = st0;
            P.sg_len[e] = ln0;
            P.sg_src[e] = sr0;
            P.sg_kind[e] = (uint8_t)k0;
            P.sg_run[e] = (uint8_t)rr;
        }
        if (ns == 2) {
            P.sg_st[e + 1] = st0 + ln0;
            P.sg_len[e + 1] = ln1;
            P.sg_src[e + 1] = sr1;
            P.sg_kind[e + 1] = SEG_PAY;
            P.sg_run[e + 1] = (uint8_t)rr;
        }
        if (t == 63)
            P.nseg = (int)incl;
    }
    wave_sync();
    // per 64-chunk row of the output, the segment holding its first byte
    {
        const int nsg = P.nseg;
        const u32 nrow = ((P.nout >> 4) + 63) >> 6;
        for (u32 rw = t; rw < nrow && rw < (u32)kPipeRows; rw += 64) {
            const u32 p = rw << 10;
            int sgi = 0;
#pragma unroll
            for (int step = 64; step > 0; step >>= 1)
                if (sgi + step < nsg && P.sg_st[sgi + step] <= p)
                    sgi += step;
            P.sg_row[rw] = (uint8_t)sgi;
        }
    }
}

// D2 of k_gro FLAT over NWS streaming waves (sw = this wave's index among
// them): the window's output chunks as one stream, every chunk folded to one
// word sum and scanned, chunks 0..3 of merged runs parked in rstash for D3.
template <int U, int NWS, int FWM>
__device__ void gro_stream(const GroPlan& P, int sw, const uint8_t* __restrict__ in,
                           uint64_t in_bytes, uint8_t* __restrict__ out, uint64_t out_bytes,
                           uint4 (*rstash)[4], u32* rpf, u32* rqe, u32* wtot)
{
    const int lane = threadIdx.x & 63;
    const uint4 z = make_uint4(0, 0, 0, 0);
    const int nseg = P.nseg;
    const uint64_t o0 = P.o0;
    const u32 NOUT = P.nout >> 4;
    const u32 QW = ((NOUT + NWS * 64 - 1) / (NWS * 64)) * 64;
    const u32 lo = sw * QW, hi = lo + QW < NOUT ? lo + QW : NOUT;
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
            int sgi = rw < (u32)kPipeRows ? P.sg_row[rw] : 0;   // past the table: search
#pragma unroll
            for (int k = 0; k < 3; k++)
                if (sgi + 1 < nseg && P.sg_st[sgi + 1] <= p)
                    sgi++;
            if (sgi + 1 < nseg && P.sg_st[sgi + 1] <= p) {   // tiny segments: search on
                int lo2 = sgi + 1, hi2 = nseg - 1;
                while (lo2 < hi2) {
                    const int mid = (lo2 + hi2 + 1) >> 1;
                    if (P.sg_st[mid] <= p) lo2 = mid; else hi2 = mid - 1;
                }
                sgi = lo2;
            }
            sj[j] = sgi;
            x[j] = z;
            y[j] = z;
            int plan = AS_ZERO;
            if (c < hi) {
                const u32 ss = P.sg_st[sgi], sl = P.sg_len[sgi], kd = P.sg_kind[sgi];
                const int r = P.sg_run[sgi];
                const u32 rend = (u32)(P.run_off[r] - o0) + P.run_len[r];
                const u32 offs = p - ss, rem = sl - offs;
                const u32 need = rend - p < 16u ? rend - p : 16u;
                const uint8_t* pa = in + P.sg_src[sgi] + offs;
                if (kd == SEG_HDR && offs + 16 <= (u32)kGroHdr) {
                    x[j] = *reinterpret_cast<const uint4*>(&P.hdr[P.sg_src[sgi]][offs]);
                    plan = AS_ONE;
                } else if (kd != SEG_HDR && pa + 16 <= in_end) {
                    x[j] = ldg16u(pa);
                    plan = AS_ONE;
                } else {
                    plan = AS_BYTES;
                }
                if (plan == AS_ONE && rem < need) {
                    const int s2 = sgi + 1;
                    const uint8_t* pb = in + P.sg_src[s2];
                    if (s2 < nseg && P.sg_run[s2] == r && P.sg_st[s2] == ss + sl &&
                        P.sg_kind[s2] == SEG_PAY && P.sg_len[s2] >= need - rem && pb + 16 <= in_end) {
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
            const int sgi = sj[j], r = P.sg_run[sgi];
            const u32 ss = P.sg_st[sgi], sl = P.sg_len[sgi];
            const u32 rrel = (u32)(P.run_off[r] - o0), rend = rrel + P.run_len[r];
            const bool merged = P.sg_kind[sgi] != SEG_WHOLE;
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
                    while (s2 + 1 < nseg && q >= P.sg_st[s2] + P.sg_len[s2])
                        s2++;
                    if (q < P.sg_st[s2] || q >= P.sg_st[s2] + P.sg_len[s2])
                        continue;
                    const u32 b = P.sg_kind[s2] == SEG_HDR
                                      ? (u32)P.hdr[P.sg_src[s2]][q - P.sg_st[s2]]
                                      : (in + P.sg_src[s2] + (q - P.sg_st[s2]) < in_end
                                             ? (u32)in[P.sg_src[s2] + (q - P.sg_st[s2])] : 0u);
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
        wtot[sw] = run;
}

// D3 of k_gro FLAT: lane r of the streaming waves finishes merged run r --
// tot_len and PSH into the head's headers, both checks from chunks 0..3 and
// the prefix difference -- and writes its chunks 0..3.
template <int NWS, int FWM>
__device__ void gro_finish(const GroPlan& P, int r, uint8_t* __restrict__ out, uint64_t out_bytes,
                           uint4 (*rstash)[4], const u32* rpf, const u32* rqe, const u32* wtot)
{
    if (r >= P.nruns || P.run_n[r] <= 1)
        return;
    const uint64_t o0 = P.o0;
    uint8_t* ob = out + o0;
    const int64_t wl_all = o0 <= out_bytes ? (int64_t)(out_bytes - o0) : 0;
    const u32 NOUT = P.nout >> 4;
    const u32 QW = ((NOUT + NWS * 64 - 1) / (NWS * 64)) * 64;
    const int k0 = P.run_t[r], nm = P.run_n[r];
    const u32 mlen = P.run_len[r], rrel = (u32)(P.run_off[r] - o0);
    uint4 sc[4] = {rstash[r][0], rstash[r][1], rstash[r][2], rstash[r][3]};
    const u32 raw = hsum4(sc[0]) + hsum4(sc[1]) + hsum4(sc[2]) + hsum4(sc[3]);
    uint8_t psh = 0;
    for (int k = k0; k < k0 + nm; k++)
        psh |= P.hdr[k][47] & 0x08;
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
            for (int k = 0; k < NWS - 1; k++)
                b += (u32)k < q ? wtot[k] : 0u;
            return b;
        };
        const u32 p0 = rpf[r] + wbase(rrel >> 4);
        const u32 p1 = rqe[r] + wbase((rrel + mlen - 1) >> 4);
        a.tcp += (p1 - p0) - raw;
    }
    uint8_t st = 0;
    uint32_t cs = 0;
    epilogue<1, 4, true, WM_SECTOR, false>(h, a, ob + rrel, mlen, 0, true, 0, GCS_CF_NO_INPLACE,
                                           &st, &cs, true, sc);
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

constexpr int kGroPipeU = 3;      // chunks per lane per trip (3 streaming waves per block)
constexpr int kGroPipeOcc = 5;    // waves per SIMD (two plans + the stash: 5 blocks per CU)

template <int U, int OCC, int FWM>
__global__ void __launch_bounds__(kBlock, OCC)
k_gro_pipe(const uint8_t* __restrict__ in, uint64_t in_bytes, const uint64_t* __restrict__ off,
           const uint16_t* __restrict__ lens, const uint8_t* __restrict__ verdict, u32 n,
           u32 window, u32 max_len, uint8_t* __restrict__ out, uint64_t out_bytes,
           uint64_t* __restrict__ out_off, uint16_t* __restrict__ out_len,
           uint32_t* __restrict__ head)
{
    constexpr int NWS = kBlock / 64 - 1;          // streaming waves
    __shared__ GroPlan plan[2];
    __shared__ uint4 rstash[kPipeW][4];           // chunks 0..3 of each merged run
    __shared__ u32 rpf[kPipeW], rqe[kPipeW], wtot[NWS];
    const int wave = threadIdx.x >> 6;
    const u32 nwin = (n + window - 1) / window;
    u32 wi = blockIdx.x;
    if (wi >= nwin)
        return;                                   // block-uniform
    if (wave == 0)
        gro_plan(plan[0], wi, in, in_bytes, off, lens, verdict, n, window, max_len, out_off,
                 out_len, head);
    __syncthreads();
    for (int k = 0; wi < nwin; k ^= 1, wi += gridDim.x) {
        if (wave == 0) {
            if (wi + gridDim.x < nwin)
                gro_plan(plan[k ^ 1], wi + gridDim.x, in, in_bytes, off, lens, verdict, n, window,
                         max_len, out_off, out_len, head);
        } else {
            gro_stream<U, NWS, FWM>(plan[k], wave - 1, in, in_bytes, out, out_bytes, rstash, rpf,
                                    rqe, wtot);
        }
        __syncthreads();
        if (wave != 0)
            gro_finish<NWS, FWM>(plan[k], (int)threadIdx.x - 64, out, out_bytes, rstash, rpf, rqe,
                                 wtot);
        __syncthreads();
    }
}

}  // namespace gcs
