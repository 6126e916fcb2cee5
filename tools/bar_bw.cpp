// bar_bw.cpp -- host stores into fine-grained device memory over the BAR: the
// write rate T threads reach together, copying bursts of B bytes from their own
// pageable buffers (what the library's device staging does per burst,
// gcs_api.cpp), with memcpy and with non-temporal 32 B stores.  Prints one JSON
// object.  Not product code.
//   hipcc -O2 -mavx2 -std=c++17 tools/bar_bw.cpp -o tools/bar_bw -lpthread
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static void copy_nt(uint8_t* dst, const uint8_t* src, size_t n)
{
    size_t i = 0;
    for (; i + 32 <= n; i += 32)
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i),
                            _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)));
    if (i < n)
        std::memcpy(dst + i, src + i, n - i);
}

int main(int argc, char** argv)
{
    const size_t burst = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 38u << 10;
    const double seconds = 0.2;
    const int counts[] = {1, 2, 4, 8, 12, 16};
    uint8_t* dev = nullptr;
    const size_t per = (burst + 4095) / 4096 * 4096;
    if (hipExtMallocWithFlags((void**)&dev, per * 16, hipDeviceMallocFinegrained) != hipSuccess) {
        std::printf("{\"error\": \"fine-grained device allocation failed\"}\n");
        return 1;
    }
    std::printf("{\"burst_bytes\": %zu, \"rates_gb_per_s\": {", burst);
    bool first = true;
    for (int method = 0; method < 2; method++) {
        for (int t : counts) {
            std::atomic<uint64_t> total{0};
            std::atomic<bool> go{false};
            std::vector<std::thread> th;
            for (int k = 0; k < t; k++)
                th.emplace_back([&, k] {
                    std::vector<uint8_t> src(burst, (uint8_t)k);
                    uint8_t* d = dev + per * k;
                    while (!go.load())
                        ;
                    const auto t0 = std::chrono::steady_clock::now();
                    uint64_t n = 0;
                    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0)
                               .count() < seconds) {
                        if (method == 0)
                            std::memcpy(d, src.data(), burst);
                        else
                            copy_nt(d, src.data(), burst);
                        _mm_sfence();
                        n += burst;
                    }
                    total += n;
                });
            go = true;
            for (auto& x : th)
                x.join();
            std::printf("%s\"%s_%dthreads\": %.2f", first ? "" : ", ",
                        method == 0 ? "memcpy" : "nt32", t, total.load() / seconds / 1e9);
            first = false;
        }
    }
    std::printf("}}\n");
    (void)hipFree(dev);
    return 0;
}
