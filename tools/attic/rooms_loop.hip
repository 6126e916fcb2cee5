// tools/attic/rooms_loop.hip -- NOT product code.  Round 5's grid-stride form
// of the rooms kernel (frames one per 2 KiB room), kept as a measurement
// record for tools/kbench.hip (included there after the library kernels).
// 1M x 1500 B in 2 KiB rooms, the same box, interleaved: verify 310-338 us and
// fill 350-373 us at 32 / 16 / 8 blocks per CU, against 245-294 / 297 us for
// the shipped k_desc<32, 3> (profiles/r05/kbench_rooms_loop.log).

namespace gcs {

// Frames one per room, a group walking frames gidx, gidx + groups, ... over a
// grid sized to the resident capacity: the descriptor of the group's next frame
// is loaded with the current frame's chunks (3 VGPRs), so each frame costs one
// memory trip instead of k_desc's two (descriptor, then chunks).
template <int G, int U, bool COMPUTE, bool NT, int WM, int OCC = 1>
__global__ void __launch_bounds__(kBlock, OCC)
k_rooms(uint8_t* __restrict__ frames, uint64_t frames_bytes, const uint64_t* __restrict__ off,
        const uint16_t* __restrict__ lens, u32 n, uint8_t* __restrict__ out_code,
        uint32_t* __restrict__ out_csum, u32 flags)
{
    constexpr int FPB = kBlock / G;
    const int sub = threadIdx.x & (G - 1);
    const uint64_t groups = (uint64_t)gridDim.x * FPB;
    uint64_t i = (uint64_t)xcd_block(blockIdx.x, gridDim.x) * FPB + threadIdx.x / G;
    if (i >= n)
        return;
    uint64_t o = off[i];
    u32 len = lens[i];
    for (;;) {                                         // group-uniform
        const uint64_t nx = i + groups;
        uint64_t onx = 0;
        u32 lnx = 0;
        if (nx < n) {
            onx = off[nx];
            lnx = lens[nx];
        }
        const bool ok = (o & 15) == 0 && o <= frames_bytes && len <= frames_bytes - o;
        do_frame<G, U, COMPUTE, true, true, NT, WM>(frames + (ok ? o : 0), len,
                                                    ok ? (int64_t)(frames_bytes - o) : 0, ok, sub,
                                                    flags, out_code ? out_code + i : nullptr,
                                                    out_csum ? out_csum + i : nullptr);
        if (nx >= n)
            break;
        i = nx;
        o = onx;
        len = lnx;
    }
}

// The same walk software-pipelined: frame k+1's chunks (and frame k+2's
// descriptor) are loaded before frame k is folded and written, so the wait for
// the next frame's data never waits for this frame's stores (vmcnt counts both
// on CDNA).
template <int G, int U, bool COMPUTE, bool NT, int WM, int OCC = 1, bool LOOP = true>
__global__ void __launch_bounds__(kBlock, OCC)
k_rooms_pipe(uint8_t* __restrict__ frames, uint64_t frames_bytes, const uint64_t* __restrict__ off,
             const uint16_t* __restrict__ lens, u32 n, uint8_t* __restrict__ out_code,
             uint32_t* __restrict__ out_csum, u32 flags)
{
    constexpr int FPB = kBlock / G;
    const int sub = threadIdx.x & (G - 1);
    const uint64_t groups = (uint64_t)gridDim.x * FPB;
    uint64_t i = (uint64_t)xcd_block(blockIdx.x, gridDim.x) * FPB + threadIdx.x / G;
    if (i >= n)
        return;
    auto valid = [&](uint64_t o, u32 len) {
        return (o & 15) == 0 && o <= frames_bytes && len <= frames_bytes - o;
    };
    uint64_t o = off[i];
    u32 len = lens[i];
    bool ok = valid(o, len);
    uint4 v[U];
    load_first<G, U, true, NT>(frames + (ok ? o : 0), ok ? (int)((len + 15) >> 4) : 0,
                               ok ? (int64_t)(frames_bytes - o) : 0, sub, v);
    uint64_t nx = i + groups, on = 0;
    u32 ln = 0;
    if (nx < n) {
        on = off[nx];
        ln = lens[nx];
    }
    for (;;) {                                         // group-uniform
        uint4 vn[U];
#pragma unroll
        for (int j = 0; j < U; j++)
            vn[j] = make_uint4(0, 0, 0, 0);
        bool okn = false;
        const uint64_t nnx = nx + groups;
        uint64_t onn = 0;
        u32 lnn = 0;
        if (nx < n) {
            okn = valid(on, ln);
            load_first<G, U, true, NT>(frames + (okn ? on : 0), okn ? (int)((ln + 15) >> 4) : 0,
                                       okn ? (int64_t)(frames_bytes - on) : 0, sub, vn);
            if (nnx < n) {
                onn = off[nnx];
                lnn = lens[nnx];
            }
        }
        uint8_t* f = frames + (ok ? o : 0);
        frame_body<G, U, COMPUTE, LOOP, true, NT, WM>(v, f, f, len,
                                                      ok ? (int64_t)(frames_bytes - o) : 0, ok,
                                                      sub, flags, out_code ? out_code + i : nullptr,
                                                      out_csum ? out_csum + i : nullptr, true);
        if (nx >= n)
            break;
#pragma unroll
        for (int j = 0; j < U; j++)
            v[j] = vn[j];
        i = nx;
        o = on;
        len = ln;
        ok = okn;
        nx = nnx;
        on = onn;
        ln = lnn;
    }
}

}  // namespace gcs
