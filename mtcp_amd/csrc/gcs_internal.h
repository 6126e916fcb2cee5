// gcs_internal.h -- launchers shared between gcs_kernels.hip and gcs_api.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtcp_gpucsum.h"

namespace gcs {

// Kernel-level extension arguments (GCS_VF_ICMP / GCS_CF_ICMP / RSS
// steering); the per-frame view is gcs_device.h's XFrame.
struct Ext {
    uint32_t key[4];           // RSS key bits 0..127 as big-endian words
    uint32_t* hash;            // per-frame outputs (nullable)
    uint16_t* queue;
    uint32_t nq, nq_magic, endian;   // nq_magic = ceil(2^32 / nq) (0 for nq == 1)
};

hipError_t launch_verify_fixed(uint8_t* frames, uint64_t stride, uint32_t frame_len, uint32_t n,
                               uint8_t* verdict, uint32_t flags, hipStream_t s);
hipError_t launch_compute_fixed(uint8_t* frames, uint64_t stride, uint32_t frame_len, uint32_t n,
                                uint8_t* status, uint32_t* csums, uint32_t flags, hipStream_t s);
hipError_t launch_verify_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                              const uint16_t* len, uint32_t n, uint8_t* verdict, uint32_t flags,
                              hipStream_t s);
hipError_t launch_compute_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                               const uint16_t* len, uint32_t n, uint8_t* status, uint32_t* csums,
                               uint32_t flags, hipStream_t s);
hipError_t launch_verify_desc_spread(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                                     const uint16_t* len, uint32_t n, uint8_t* verdict,
                                     uint32_t flags, hipStream_t s);
hipError_t launch_compute_desc_spread(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                                      const uint16_t* len, uint32_t n, uint8_t* status,
                                      uint32_t* csums, uint32_t flags, hipStream_t s);
hipError_t launch_classify_fixed(uint8_t* frames, uint64_t stride, uint32_t frame_len,
                                 uint32_t n, uint8_t* verdict, uint32_t flags, const Ext& ext,
                                 hipStream_t s);
hipError_t launch_classify_desc(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                                const uint16_t* len, uint32_t n, uint8_t* verdict,
                                uint32_t flags, const Ext& ext, hipStream_t s);
hipError_t launch_copy_fill(uint8_t* frames, uint64_t frames_bytes, const uint64_t* off,
                            const uint16_t* len, const uint8_t* src, uint64_t src_bytes,
                            const uint64_t* src_off, uint32_t n, uint8_t* status,
                            uint32_t* csums, uint32_t flags, hipStream_t s);
hipError_t launch_gro(const uint8_t* in, uint64_t in_bytes, const uint64_t* off,
                      const uint16_t* len, const uint8_t* verdict, uint32_t n, uint32_t window,
                      uint32_t max_len, uint8_t* out, uint64_t out_bytes, uint64_t* out_off,
                      uint16_t* out_len, uint32_t* head, hipStream_t s);
hipError_t launch_icmp_fn(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off,
                          const uint16_t* len, uint32_t n, uint16_t* out, hipStream_t s);
hipError_t launch_rss_fn(const uint32_t* sip, const uint32_t* dip, const uint16_t* sp,
                         const uint16_t* dp, uint32_t n, const Ext& ext, hipStream_t s);
hipError_t launch_tcp_fn(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off,
                         const uint16_t* len, const uint32_t* saddr, const uint32_t* daddr,
                         uint32_t n, uint16_t* out, hipStream_t s);
hipError_t launch_ip_fn(const uint8_t* buf, uint64_t buf_bytes, const uint64_t* off,
                        const uint8_t* ihl, uint32_t n, uint16_t* out, hipStream_t s);

}  // namespace gcs
