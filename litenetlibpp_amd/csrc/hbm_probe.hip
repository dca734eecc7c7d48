// hbm_probe.hip -- measurement tool, not part of the CRC path: a read-only
// streaming kernel (global_load_dwordx4, XOR-reduced, no stores in the steady
// state) used by bench.py to report the MEASURED HBM read peak next to the
// 8 TB/s nameplate the roofline fraction is quoted against.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_read(const u32x4* __restrict__ p, size_t n16,
                                                   uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const u32x4 a = __builtin_nontemporal_load(p + i);
        const u32x4 b = __builtin_nontemporal_load(p + i + stride);
        const u32x4 c = __builtin_nontemporal_load(p + i + 2 * stride);
        const u32x4 d = __builtin_nontemporal_load(p + i + 3 * stride);
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    }
    for (; i < n16; i += stride) {
        const u32x4 a = p[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the loads alive
}

extern "C" int lnl_probe_stream_read(const void* d, size_t bytes, uint32_t* d_sink, void* stream) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = cus * 8;
    hipLaunchKernelGGL(stream_read, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)d, bytes / 16, d_sink);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
