// hbm_probe.hip -- measurement tool, not part of the CRC path: read-only
// streaming kernels used by bench.py to report the MEASURED HBM read peak next
// to the 8 TB/s nameplate the roofline fraction is quoted against.
//
//   form 0: global_load_dwordx4 nt into registers, XOR-reduced, 4 loads in
//           flight per lane, 8 waves per CU
//   form 1: global_load_lds_dwordx4 nt (LDS-DMA, the CRC kernels' load form),
//           8 KiB contiguous chunks per wave-step, up to 32 wave-instructions
//           (32 KiB) in flight per wave, 8 waves per CU, nothing read back
//           (every load lands in the same 1 KiB LDS slot of the wave)
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

// chunks: bytes / 8192 (the host passes a multiple of 8 KiB)
__global__ __launch_bounds__(256) void stream_read_lds(const uint8_t* __restrict__ p, uint32_t chunks) {
    __shared__ __attribute__((aligned(16))) uint4 slot[4 * 64];  // 1 KiB per wave
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    uint4* const dst = slot + 64 * wave;
    const uint32_t nw = gridDim.x * 4u;
    for (uint32_t c = blockIdx.x * 4u + wave; c < chunks; c += nw) {
        const uint8_t* src = p + (size_t)c * 8192u + 16u * lane;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(src + 1024 * i), (void*)dst, 16, 0, 2);
        asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

extern "C" int lnl_probe_stream_read(const void* d, size_t bytes, uint32_t* d_sink, void* stream, int form) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = cus * 2;
    if (form == 1) {
        const size_t chunks = bytes / 8192u;
        if (chunks == 0 || chunks > 0xFFFFFFFFull) return -22;
        hipLaunchKernelGGL(stream_read_lds, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)d,
                           (uint32_t)chunks);
    } else {
        hipLaunchKernelGGL(stream_read, dim3(cus * 8), dim3(256), 0, (hipStream_t)stream, (const u32x4*)d,
                           bytes / 16, d_sink);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
