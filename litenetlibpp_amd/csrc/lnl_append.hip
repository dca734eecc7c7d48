// lnl_append.hip -- the outbound CRC-32C layer for a device-resident burst
// (lnl_crc32c_append_csr_dev, include/lnl_crc32c.h): datagram i of a CSR burst
// is written to dst + (off[i] - off[0]) + 4 i as payload || LE32(crc_i), the
// wire form net_manager::send_raw puts on the socket with the layer on
// (/root/reference/src/lnl/net_manager.cpp:515-521).
//
// Two passes: the CSR CRC pass (crc32c_span.hip) into crc[], then the copy
// kernel below.  A team of 32 lanes per datagram writes its whole 16-byte
// destination chunks from a dwordx4 + dword source load (v_alignbyte to any
// byte shift); the head chunk and the tail (payload remainder + CRC), which
// share chunks with the neighbouring datagrams, go one byte per lane.  Each
// lane issues the loads of up to kCopyU chunks before it stores any (round 3
// issued one, then stored it: one memory round trip per 512 bytes of a
// datagram).  ~50 VGPRs, 8 waves per SIMD; one datagram per team (below).
//
// The one-pass form (the team computes each datagram's CRC from the registers
// it copies) and the other round-4 copy shapes were built, parity-green and
// slower; they are tools/experiments/round4_experiments.patch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"
#include "crc32c_kernels.h"

namespace lnl {

namespace {

using dev::u32x4;

#define LNL_G LNL_GLOBAL  // crc32c_device.h

struct __attribute__((packed, aligned(4))) U4a {  // 16 bytes at a 4-byte aligned address
    uint32_t x, y, z, w;
};

// 16-byte chunk store (asm: the compiler then keeps the loop rolled and the
// wave reaches its next loads sooner)
__device__ LNL_INLINE void store16(uint64_t a, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(a), "v"(u32x4{x, y, z, w}) : "memory");
}

#ifndef LNL_APPEND_TEAM
#define LNL_APPEND_TEAM 32u  // lanes per datagram (16: 559, 32: 512, 64: 613 us in round 2)
#endif
constexpr uint32_t kAppTeam = LNL_APPEND_TEAM;
#ifndef LNL_APPEND_COPY_U
#define LNL_APPEND_COPY_U 3  // chunk loads in flight per lane (1: round 3's kernel)
#endif
constexpr uint32_t kCopyU = LNL_APPEND_COPY_U;
#ifndef LNL_APPEND_THREADS
#define LNL_APPEND_THREADS 256
#endif
constexpr int kCopyThreads = LNL_APPEND_THREADS;
__device__ inline uint8_t out_byte(uint64_t x, uint64_t P1, uint64_t delta, uint32_t crc) {
    return x < P1 ? *LNL_G(const uint8_t, x - delta) : (uint8_t)(crc >> (8u * (uint32_t)(x - P1)));
}
__global__ __launch_bounds__(kCopyThreads) void append_copy_kernel(AppendArgs a) {
    const uint32_t t = (blockIdx.x * kCopyThreads + threadIdx.x) / kAppTeam;
    const uint32_t nt = gridDim.x * (kCopyThreads / kAppTeam);
    const uint32_t q = threadIdx.x % kAppTeam;
    const uint64_t o0 = a.off[0];
    const uint64_t dstb = (uint64_t)(uintptr_t)a.dst, srcb = (uint64_t)(uintptr_t)a.base - a.off0;
    // the next datagram's offsets and CRC are fetched one datagram ahead
    uint64_t ns = 0, ne = 0;
    uint32_t ncrc = 0;
    if (t < a.n) {
        ns = a.off[t];
        ne = a.off[t + 1];
        ncrc = a.crc[t];
    }
    for (uint32_t i = t; i < a.n; i += nt) {
        const uint64_t s = ns, e = ne;
        const uint32_t crc = ncrc;
        if (i + nt < a.n) {
            ns = a.off[i + nt];
            ne = a.off[i + nt + 1];
            ncrc = a.crc[i + nt];
        }
        const uint64_t P0 = dstb + (s - o0) + 4ull * i, P1 = P0 + (e - s), P2 = P1 + 4u;
        const uint64_t delta = P0 - (srcb + s);
        const uint64_t c0 = (P0 + 15u) & ~(uint64_t)15, c1 = P1 & ~(uint64_t)15;
        if (c0 >= c1) {
            for (uint64_t x = P0 + q; x < P2; x += kAppTeam) *LNL_G(uint8_t, x) = out_byte(x, P1, delta, crc);
            continue;
        }
        // the head chunk [P0, c0) and the tail [c1, P2), one byte per lane,
        // loaded before the chunks so that their latency overlaps them
        const uint64_t x0 = P0 + q, x1 = c1 + q;
        const bool b0 = x0 < c0, b1 = x1 < P2;
        const uint8_t v0 = b0 ? out_byte(x0, P1, delta, crc) : 0;
        const uint8_t v1 = b1 ? out_byte(x1, P1, delta, crc) : 0;
        const uint32_t c = (uint32_t)((c0 - delta) & 3u);  // (the same for every chunk)
        for (uint64_t wb = c0 + 16ull * q; wb < c1; wb += 16ull * kAppTeam * kCopyU) {
            U4a v[kCopyU];
            uint32_t v4[kCopyU];
#pragma unroll
            for (uint32_t u = 0; u < kCopyU; ++u) {
                const uint64_t w = wb + 16ull * kAppTeam * u;
                if (w < c1) {
                    const uint64_t sw = (w - delta) & ~(uint64_t)3;
#if defined(LNL_APPEND_DIAG) && (LNL_APPEND_DIAG & 2)  // (diagnostic build: chunk loads aligned, no 5th dword)
                    v[u] = *LNL_G(const U4a, sw & ~(uint64_t)15);
                    v4[u] = 0u;
#else
                    v[u] = *LNL_G(const U4a, sw);
                    v4[u] = c ? *LNL_G(const uint32_t, sw + 16) : 0u;  // (byte w - delta + 15: inside the payload)
#endif
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < kCopyU; ++u) {
                const uint64_t w = wb + 16ull * kAppTeam * u;
                if (w < c1)
                    store16(w, __builtin_amdgcn_alignbyte(v[u].y, v[u].x, c), __builtin_amdgcn_alignbyte(v[u].z, v[u].y, c),
                            __builtin_amdgcn_alignbyte(v[u].w, v[u].z, c), __builtin_amdgcn_alignbyte(v4[u], v[u].w, c));
            }
        }
#if !(defined(LNL_APPEND_DIAG) && (LNL_APPEND_DIAG & 1))  // (diagnostic build: no head / tail byte stores)
        if (b0) *LNL_G(uint8_t, x0) = v0;
        if (b1) *LNL_G(uint8_t, x1) = v1;
#endif
    }
}

}  // namespace

// Grid: one datagram per team, so the dispatcher hands out the burst in order
// and the whole chip reads and writes inside one moving window of it.  A grid
// capped at 16 workgroups per CU, teams striding over the datagrams, took
// 462 us per config-3 call against 432 (round 5): strided teams
// drift apart and spread the reads and writes over more DRAM pages.
#ifndef LNL_APPEND_WGS
#define LNL_APPEND_WGS 0u  // workgroups per CU (0: no cap; experiments: a strided, persistent grid)
#endif
hipError_t launch_append(const AppendArgs& a, int cus, hipStream_t stream) {
    const uint32_t per = kCopyThreads / kAppTeam;
    const uint32_t want = (a.n + per - 1) / per, cap = LNL_APPEND_WGS ? (uint32_t)cus * LNL_APPEND_WGS : 0xFFFFFFFFu;
    hipLaunchKernelGGL(append_copy_kernel, dim3(want < cap ? (want ? want : 1) : cap), dim3(kCopyThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
