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
template <int G, int U, bool COMPUTE, bool NT, int WM>
__global__ void __launch_bounds__(kBlock)
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

}  // namespace gcs
