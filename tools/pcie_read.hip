// pcie_read.hip -- how fast a burst's frames come over PCIe into the GPU as a
// function of how many CUs pull them (MEASUREMENT TOOL, not product code).
//
// 64 frames x 1536 B (an mTCP RX burst of 1500 B frames) in registered host
// memory (hipHostRegister, uncached as gcs_host_register maps it, or cached),
// read by B blocks of T threads, each lane loading its 16 B chunks and folding
// them into a word written per block.  One launch per timed sample (HIP events
// around it, launch overhead included and the same for every B), median of
// 200.  Prints one JSON object.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// rooms: chunk c of the burst is chunk c % 96 of frame c / 96, frames one per
// 2 KiB room (the server's layout) instead of packed
__global__ void k_pull(const u32x4* __restrict__ src, uint64_t chunks, uint32_t* __restrict__ out,
                       int rooms)
{
    uint32_t s = 0;
#pragma unroll 8
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < chunks;
         c += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = rooms ? (c / 96) * 128 + c % 96 : c;
        const u32x4 v = __builtin_nontemporal_load(&src[a]);
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    s = __reduce_add_sync(0xFFFFFFFFFFFFFFFFull, s);
    if ((threadIdx.x & 63) == 0)
        atomicAdd(&out[blockIdx.x], s);
}

int main(int argc, char** argv)
{
    const bool cached = argc > 1 && std::strcmp(argv[1], "cached") == 0;
    const int rooms = argc > 2 && std::strcmp(argv[2], "rooms") == 0;
    const size_t bytes = 64 * 1536;
    const size_t alloc = 64 * 2048 + 8192;
    uint8_t* host = static_cast<uint8_t*>(std::aligned_alloc(4096, alloc));
    std::memset(host, 0x5A, alloc);
    CHECK(hipHostRegister(host, alloc, cached ? hipHostRegisterMapped
                                              : (hipHostRegisterMapped | hipExtHostRegisterUncached)));
    uint8_t* dev = nullptr;
    CHECK(hipHostGetDevicePointer((void**)&dev, host, 0));
    uint32_t* out = nullptr;
    CHECK(hipMalloc(&out, 4096 * sizeof(uint32_t)));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::printf("{\"region\": \"%s\", \"layout\": \"%s\", \"bytes\": %zu, \"rows\": [",
                cached ? "cached" : "uncached", rooms ? "rooms" : "packed", bytes);
    bool first = true;
    for (int threads : {256, 1024}) {
        for (int blocks : {1, 2, 4, 8, 16, 32, 64, 128}) {
            std::vector<float> ms;
            for (int r = 0; r < 220; r++) {
                std::memset(host, r & 0xFF, 64 * 2048);      // fresh frames, as a NIC writes them
                CHECK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(k_pull, dim3(blocks), dim3(threads), 0, 0,
                                   reinterpret_cast<const u32x4*>(dev), bytes / 16, out, rooms);
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float t = 0;
                CHECK(hipEventElapsedTime(&t, e0, e1));
                if (r >= 20)
                    ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            const float med = ms[ms.size() / 2];
            std::printf("%s{\"threads\": %d, \"blocks\": %d, \"us_median\": %.3f, \"gb_per_s\": %.2f}",
                        first ? "" : ", ", threads, blocks, med * 1e3, bytes / (med * 1e-3) / 1e9);
            first = false;
        }
    }
    // a launch that reads nothing: the launch + event overhead alone
    std::vector<float> ms;
    for (int r = 0; r < 220; r++) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_pull, dim3(8), dim3(256), 0, 0, reinterpret_cast<const u32x4*>(dev),
                           (uint64_t)0, out, 0);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float t = 0;
        CHECK(hipEventElapsedTime(&t, e0, e1));
        if (r >= 20)
            ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("], \"empty_launch_us\": %.3f}\n", ms[ms.size() / 2] * 1e3);
    CHECK(hipHostUnregister(host));
    std::free(host);
    return 0;
}
