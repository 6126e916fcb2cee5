// pingpong.hip -- host<->GPU round-trip latency of a resident polling kernel,
// mailbox in pinned host memory (the burst server's today) vs in fine-grained
// device memory written by the host over PCIe (large BAR).  Not product code.
//   hipcc --offload-arch=gfx950 -O3 tools/pingpong.hip -o tools/pingpong
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,            \
                         hipGetErrorString(e_));                                      \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

// One wave polls `req` until it reads q, answers ack = q (host memory), for
// `rounds` requests; every poll loop is bounded (max_polls) and the clock-based
// bound ends the kernel even if the host stops.
__global__ void k_pong(const volatile uint32_t* req, uint32_t* ack, uint32_t rounds,
                       uint64_t max_ticks)
{
    if (threadIdx.x != 0)
        return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t q = 1; q <= rounds; q++) {
        for (uint32_t polls = 0;; polls++) {
            if (*req == q)
                break;
            if (polls > (1u << 24) || __builtin_amdgcn_s_memrealtime() - t0 > max_ticks)
                return;
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(ack, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static void run(const char* name, volatile uint32_t* req_host, const uint32_t* req_dev,
                hipStream_t s, uint32_t rounds)
{
    uint32_t* ack;
    CK(hipHostMalloc((void**)&ack, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *ack = 0;
    *req_host = 0;
    uint32_t* dack;
    CK(hipHostGetDevicePointer((void**)&dack, ack, 0));
    hipLaunchKernelGGL(k_pong, dim3(1), dim3(64), 0, s, (const volatile uint32_t*)req_dev, dack,
                       rounds, (uint64_t)100 * 1000 * 1000 * 2);   // <= ~2 s at 100 MHz
    std::vector<double> us;
    for (uint32_t q = 1; q <= rounds; q++) {
        const auto t0 = std::chrono::steady_clock::now();
        *req_host = q;
        bool ok = false;
        while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(100)) {
            if (__atomic_load_n(ack, __ATOMIC_ACQUIRE) == q) {
                ok = true;
                break;
            }
        }
        if (!ok) {
            std::printf("%s: no answer to request %u\n", name, q);
            break;
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                         .count());
    }
    CK(hipStreamSynchronize(s));
    if (!us.empty()) {
        std::sort(us.begin(), us.end());
        std::printf("%-44s round trip median %.2f us  p10 %.2f  p90 %.2f  (%zu)\n", name,
                    us[us.size() / 2], us[us.size() / 10], us[us.size() * 9 / 10], us.size());
    }
    CK(hipHostFree(ack));
}

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const uint32_t rounds = 2000;
    // 1: request word in pinned host memory (today's mailbox)
    uint32_t* hreq;
    CK(hipHostMalloc((void**)&hreq, 64, hipHostMallocCoherent | hipHostMallocMapped));
    uint32_t* hreq_dev;
    CK(hipHostGetDevicePointer((void**)&hreq_dev, hreq, 0));
    run("request in pinned host memory", hreq, hreq_dev, s, rounds);
    // 2: request word in fine-grained device memory, written by the host
    uint32_t* dreq = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&dreq, 4096, hipDeviceMallocFinegrained);
    if (e != hipSuccess) {
        std::printf("fine-grained device memory: %s\n", hipGetErrorString(e));
    } else {
        hipPointerAttribute_t at;
        CK(hipPointerGetAttributes(&at, dreq));
        std::printf("fine-grained device alloc: type %d host ptr %p dev ptr %p\n", (int)at.type,
                    at.hostPointer, at.devicePointer);
        run("request in fine-grained device memory", dreq, dreq, s, rounds);
    }
    // 3: uncached device memory
    uint32_t* ureq = nullptr;
    e = hipExtMallocWithFlags((void**)&ureq, 4096, hipDeviceMallocUncached);
    if (e != hipSuccess)
        std::printf("uncached device memory: %s\n", hipGetErrorString(e));
    else
        run("request in uncached device memory", ureq, ureq, s, rounds);
    return 0;
}
