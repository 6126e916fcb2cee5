// gcs_api.cpp -- the extern "C" ABI of libmtcp_gpucsum.so (include/mtcp_gpucsum.h).
//
// Host-side runtime: per-thread contexts bound to one HIP device and one
// non-blocking stream (mTCP's one-context-per-core model, core.c:1153-1245),
// pinned staging for host batches with two slots so that the CPU gather of
// chunk k+1 overlaps the H2D/kernel/D2H of chunk k, and only verdicts (1 B per
// frame) or check fields (4 B per frame) come back over PCIe.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>

#include "gcs_internal.h"

namespace {

thread_local char g_hip_err[256] = "";

int hip_fail(hipError_t e, const char* what)
{
    std::snprintf(g_hip_err, sizeof g_hip_err, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    if (e == hipErrorOutOfMemory)
        return GCS_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice)
        return GCS_ENODEV;
    return GCS_EHIP;
}

#define HIP_TRY(call)                                     \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

constexpr int kSlots = 2;
constexpr uint64_t kSlotAlign = 64;   // pslib packing, io_engine/lib/pslib.c:146

struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint8_t* h_frames = nullptr;   // pinned
    uint8_t* d_frames = nullptr;
    uint64_t* h_off = nullptr;
    uint64_t* d_off = nullptr;
    uint16_t* h_len = nullptr;
    uint16_t* d_len = nullptr;
    uint8_t* h_code = nullptr;
    uint8_t* d_code = nullptr;
    uint32_t* h_csum = nullptr;
    uint32_t* d_csum = nullptr;
    // bookkeeping of the chunk in flight
    bool busy = false;
    uint32_t first = 0, count = 0;
};

}  // namespace

struct gcs_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t max_frames = 0;   // per slot
    uint64_t max_bytes = 0;    // per slot
    Slot slot[kSlots];
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        if (prev != dev)
            (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

hipStream_t pick_stream(gcs_ctx* ctx, void* stream)
{
    return stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
}

void free_slot(Slot& s)
{
    if (s.h_frames) (void)hipHostFree(s.h_frames);
    if (s.h_off) (void)hipHostFree(s.h_off);
    if (s.h_len) (void)hipHostFree(s.h_len);
    if (s.h_code) (void)hipHostFree(s.h_code);
    if (s.h_csum) (void)hipHostFree(s.h_csum);
    if (s.d_frames) (void)hipFree(s.d_frames);
    if (s.d_off) (void)hipFree(s.d_off);
    if (s.d_len) (void)hipFree(s.d_len);
    if (s.d_code) (void)hipFree(s.d_code);
    if (s.d_csum) (void)hipFree(s.d_csum);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = Slot();
}

int alloc_slot(Slot& s, uint32_t frames, uint64_t bytes)
{
    HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    HIP_TRY(hipHostMalloc((void**)&s.h_frames, bytes, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_off, frames * sizeof(uint64_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_len, frames * sizeof(uint16_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_code, frames, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_csum, frames * sizeof(uint32_t), hipHostMallocDefault));
    HIP_TRY(hipMalloc((void**)&s.d_frames, bytes));
    HIP_TRY(hipMalloc((void**)&s.d_off, frames * sizeof(uint64_t)));
    HIP_TRY(hipMalloc((void**)&s.d_len, frames * sizeof(uint16_t)));
    HIP_TRY(hipMalloc((void**)&s.d_code, frames));
    HIP_TRY(hipMalloc((void**)&s.d_csum, frames * sizeof(uint32_t)));
    return GCS_OK;
}

// Write back the check fields the device computed for one TX frame.
void scatter_tx(uint8_t* f, uint32_t len, uint8_t st, uint32_t cs)
{
    if (st != GCS_TX_OK && st != GCS_TX_IP_ONLY && st != GCS_TX_BAD_TCPLEN)
        return;
    uint16_t ipc = (uint16_t)cs;
    std::memcpy(f + 24, &ipc, 2);                     // iph->check (ip_out.c:172)
    if (st == GCS_TX_OK) {
        uint32_t ts = 14 + 4u * (f[14] & 15u);
        uint16_t tcpc = (uint16_t)(cs >> 16);
        if (ts + 18 <= len)
            std::memcpy(f + ts + 16, &tcpc, 2);       // tcph->check (tcp_out.c:330)
    }
}

// Generic staged host batch.  Frames are addressed by base + off[i] or by
// ptrs[i]; `compute` selects TX fill vs RX verify.
int run_host_batch(gcs_ctx* ctx, uint8_t* base, const uint64_t* off, uint8_t* const* ptrs,
                   const uint16_t* len, uint32_t n, uint8_t* code, uint32_t* csums,
                   uint32_t flags, bool compute)
{
    if (!ctx || !len || (!base && !ptrs) || (base && !off))
        return GCS_EINVAL;
    if (!compute && !code)
        return GCS_EINVAL;
    if (ctx->max_frames == 0 || ctx->max_bytes == 0)
        return GCS_ERANGE;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);

    auto frame_ptr = [&](uint32_t i) -> uint8_t* { return ptrs ? ptrs[i] : base + off[i]; };

    // Drain one slot: wait for its stream and hand its results back.
    auto drain = [&](Slot& s) -> int {
        if (!s.busy)
            return GCS_OK;
        HIP_TRY(hipEventSynchronize(s.done));
        s.busy = false;
        if (!compute) {
            std::memcpy(code + s.first, s.h_code, s.count);
            return GCS_OK;
        }
        for (uint32_t k = 0; k < s.count; k++) {
            uint32_t i = s.first + k;
            uint8_t st = s.h_code[k];
            uint32_t cs = s.h_csum[k];
            if (code) code[i] = st;
            if (csums) csums[i] = cs;
            if (!(flags & GCS_CF_NO_INPLACE) && frame_ptr(i))
                scatter_tx(frame_ptr(i), len[i], st, cs);
        }
        return GCS_OK;
    };

    uint32_t next = 0;
    int k = 0;
    while (next < n) {
        Slot& s = ctx->slot[k % kSlots];
        int rc = drain(s);
        if (rc) return rc;
        // gather as many frames as fit this slot
        uint64_t used = 0;
        uint32_t cnt = 0;
        while (next + cnt < n && cnt < ctx->max_frames) {
            uint32_t i = next + cnt;
            uint64_t need = (len[i] + kSlotAlign - 1) / kSlotAlign * kSlotAlign;
            if (used + need > ctx->max_bytes)
                break;
            uint8_t* src = frame_ptr(i);
            if (src)
                std::memcpy(s.h_frames + used, src, len[i]);
            s.h_off[cnt] = used;
            s.h_len[cnt] = src ? len[i] : 0;
            used += need;
            cnt++;
        }
        if (cnt == 0)
            return GCS_ERANGE;   // a single frame larger than the staging
        s.first = next;
        s.count = cnt;
        HIP_TRY(hipMemcpyAsync(s.d_frames, s.h_frames, used, hipMemcpyHostToDevice, s.stream));
        HIP_TRY(hipMemcpyAsync(s.d_off, s.h_off, cnt * sizeof(uint64_t), hipMemcpyHostToDevice,
                               s.stream));
        HIP_TRY(hipMemcpyAsync(s.d_len, s.h_len, cnt * sizeof(uint16_t), hipMemcpyHostToDevice,
                               s.stream));
        if (compute) {
            HIP_TRY(gcs::launch_compute_desc(s.d_frames, used, s.d_off, s.d_len, cnt, s.d_code,
                                             s.d_csum, GCS_CF_NO_INPLACE, s.stream));
            HIP_TRY(hipMemcpyAsync(s.h_csum, s.d_csum, cnt * sizeof(uint32_t),
                                   hipMemcpyDeviceToHost, s.stream));
        } else {
            // the tcp_in.c:1237 side effect is applied on the host copy below
            HIP_TRY(gcs::launch_verify_desc(s.d_frames, used, s.d_off, s.d_len, cnt, s.d_code,
                                            0u, s.stream));
        }
        HIP_TRY(hipMemcpyAsync(s.h_code, s.d_code, cnt, hipMemcpyDeviceToHost, s.stream));
        HIP_TRY(hipEventRecord(s.done, s.stream));
        s.busy = true;
        next += cnt;
        k++;
    }
    for (auto& s : ctx->slot) {
        int rc = drain(s);
        if (rc) return rc;
    }
    if (!compute && (flags & GCS_VF_ZERO_BAD_TCP_CHECK)) {
        for (uint32_t i = 0; i < n; i++) {
            if (code[i] != GCS_V_DROP_TCPCSUM)
                continue;
            uint8_t* f = frame_ptr(i);
            uint32_t ts = 14 + 4u * (f[14] & 15u);
            if (ts + 18 <= len[i])
                f[ts + 16] = f[ts + 17] = 0;          // tcp_in.c:1237
        }
    }
    return GCS_OK;
}

}  // namespace

extern "C" {

int gcs_abi_version(void) { return GCS_ABI_VERSION; }

const char* gcs_strerror(int code)
{
    switch (code) {
    case GCS_OK: return "ok";
    case GCS_EINVAL: return "invalid argument";
    case GCS_ENODEV: return "no such HIP device";
    case GCS_ENOMEM: return "out of memory";
    case GCS_EHIP: return "HIP runtime error";
    case GCS_ERANGE: return "batch exceeds context capacity";
    default: return "unknown error";
    }
}

const char* gcs_last_hip_error(void) { return g_hip_err; }

int gcs_device_count(int* count)
{
    if (!count)
        return GCS_EINVAL;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *count = 0;
        return hip_fail(e, "hipGetDeviceCount");
    }
    *count = c;
    return GCS_OK;
}

int gcs_ctx_create(gcs_ctx** out, int device, uint32_t max_frames, uint64_t max_bytes)
{
    if (!out)
        return GCS_EINVAL;
    *out = nullptr;
    int count = 0;
    int rc = gcs_device_count(&count);
    if (rc)
        return rc;
    if (device < 0 || device >= count)
        return GCS_ENODEV;
    gcs_ctx* ctx = new (std::nothrow) gcs_ctx();
    if (!ctx)
        return GCS_ENOMEM;
    ctx->device = device;
    DeviceGuard g(device);
    hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return hip_fail(e, "hipStreamCreateWithFlags");
    }
    if (max_frames && max_bytes) {
        // split the requested staging between the two slots
        ctx->max_frames = std::max<uint32_t>(1, max_frames / kSlots + 1);
        ctx->max_bytes = (max_bytes / kSlots + kSlotAlign + 2047) / kSlotAlign * kSlotAlign;
        for (auto& s : ctx->slot) {
            rc = alloc_slot(s, ctx->max_frames, ctx->max_bytes);
            if (rc) {
                gcs_ctx_destroy(ctx);
                return rc;
            }
        }
    }
    *out = ctx;
    return GCS_OK;
}

int gcs_ctx_destroy(gcs_ctx* ctx)
{
    if (!ctx)
        return GCS_EINVAL;
    {
        DeviceGuard g(ctx->device);
        for (auto& s : ctx->slot) {
            if (s.stream)
                (void)hipStreamSynchronize(s.stream);
            free_slot(s);
        }
        if (ctx->stream) {
            (void)hipStreamSynchronize(ctx->stream);
            (void)hipStreamDestroy(ctx->stream);
        }
    }
    delete ctx;
    return GCS_OK;
}

int gcs_ctx_device(const gcs_ctx* ctx, int* device)
{
    if (!ctx || !device)
        return GCS_EINVAL;
    *device = ctx->device;
    return GCS_OK;
}

int gcs_ctx_stream(const gcs_ctx* ctx, void** stream)
{
    if (!ctx || !stream)
        return GCS_EINVAL;
    *stream = ctx->stream;
    return GCS_OK;
}

int gcs_sync(gcs_ctx* ctx)
{
    if (!ctx)
        return GCS_EINVAL;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return GCS_OK;
}

int gcs_host_alloc(void** p, uint64_t bytes)
{
    if (!p)
        return GCS_EINVAL;
    HIP_TRY(hipHostMalloc(p, bytes, hipHostMallocDefault));
    return GCS_OK;
}

int gcs_host_free(void* p)
{
    HIP_TRY(hipHostFree(p));
    return GCS_OK;
}

int gcs_dev_alloc(gcs_ctx* ctx, void** p, uint64_t bytes)
{
    if (!ctx || !p)
        return GCS_EINVAL;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipMalloc(p, bytes));
    return GCS_OK;
}

int gcs_dev_free(gcs_ctx* ctx, void* p)
{
    if (!ctx)
        return GCS_EINVAL;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipFree(p));
    return GCS_OK;
}

int gcs_verify_fixed_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t stride, uint32_t frame_len,
                         uint32_t n, uint8_t* d_verdict, uint32_t flags, void* stream)
{
    if (!ctx || (n && (!d_frames || !d_verdict)) || stride % 16 || stride == 0 ||
        (frame_len + 15u) / 16u * 16u > stride)
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_verify_fixed(d_frames, stride, frame_len, n, d_verdict, flags,
                                     pick_stream(ctx, stream)));
    return GCS_OK;
}

int gcs_compute_fixed_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t stride, uint32_t frame_len,
                          uint32_t n, uint8_t* d_status, uint32_t* d_csums, uint32_t flags,
                          void* stream)
{
    if (!ctx || (n && !d_frames) || stride % 16 || stride == 0 ||
        (frame_len + 15u) / 16u * 16u > stride)
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_compute_fixed(d_frames, stride, frame_len, n, d_status, d_csums, flags,
                                      pick_stream(ctx, stream)));
    return GCS_OK;
}

int gcs_verify_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_off,
                   const uint16_t* d_len, uint32_t n, uint8_t* d_verdict, uint32_t flags,
                   void* stream)
{
    if (!ctx || (n && (!d_frames || !d_off || !d_len || !d_verdict)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_verify_desc(d_frames, frames_bytes, d_off, d_len, n, d_verdict, flags,
                                    pick_stream(ctx, stream)));
    return GCS_OK;
}

int gcs_compute_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_off,
                    const uint16_t* d_len, uint32_t n, uint8_t* d_status, uint32_t* d_csums,
                    uint32_t flags, void* stream)
{
    if (!ctx || (n && (!d_frames || !d_off || !d_len)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_compute_desc(d_frames, frames_bytes, d_off, d_len, n, d_status, d_csums,
                                     flags, pick_stream(ctx, stream)));
    return GCS_OK;
}

int gcs_tcp_checksum_dev(gcs_ctx* ctx, const uint8_t* d_buf, uint64_t buf_bytes,
                         const uint64_t* d_off, const uint16_t* d_len, const uint32_t* d_saddr,
                         const uint32_t* d_daddr, uint32_t n, uint16_t* d_out, void* stream)
{
    if (!ctx || (n && (!d_buf || !d_off || !d_len || !d_saddr || !d_daddr || !d_out)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_tcp_fn(d_buf, buf_bytes, d_off, d_len, d_saddr, d_daddr, n, d_out,
                               pick_stream(ctx, stream)));
    return GCS_OK;
}

int gcs_ip_checksum_dev(gcs_ctx* ctx, const uint8_t* d_buf, uint64_t buf_bytes,
                        const uint64_t* d_off, const uint8_t* d_ihl, uint32_t n, uint16_t* d_out,
                        void* stream)
{
    if (!ctx || (n && (!d_buf || !d_off || !d_ihl || !d_out)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_ip_fn(d_buf, buf_bytes, d_off, d_ihl, n, d_out, pick_stream(ctx, stream)));
    return GCS_OK;
}

int gcs_verify(gcs_ctx* ctx, uint8_t* frames, const uint64_t* off, const uint16_t* len,
               uint32_t n, uint8_t* verdict, uint32_t flags)
{
    return run_host_batch(ctx, frames, off, nullptr, len, n, verdict, nullptr, flags, false);
}

int gcs_compute(gcs_ctx* ctx, uint8_t* frames, const uint64_t* off, const uint16_t* len,
                uint32_t n, uint8_t* status, uint32_t* csums)
{
    return run_host_batch(ctx, frames, off, nullptr, len, n, status, csums, 0u, true);
}

int gcs_verify_ptrs(gcs_ctx* ctx, uint8_t* const* pkts, const uint16_t* len, uint32_t n,
                    uint8_t* verdict, uint32_t flags)
{
    return run_host_batch(ctx, nullptr, nullptr, pkts, len, n, verdict, nullptr, flags, false);
}

int gcs_compute_ptrs(gcs_ctx* ctx, uint8_t* const* pkts, const uint16_t* len, uint32_t n,
                     uint8_t* status, uint32_t* csums)
{
    return run_host_batch(ctx, nullptr, nullptr, pkts, len, n, status, csums, 0u, true);
}

}  // extern "C"
