// lnl_append.hip -- the outbound CRC-32C layer for a device-resident burst
// (lnl_crc32c_append_csr_dev, include/lnl_crc32c.h): datagram i of a CSR burst
// is written to dst + (off[i] - off[0]) + 4 i as payload || LE32(crc_i), the
// wire form net_manager::send_raw puts on the socket with the layer on
// (/root/reference/src/lnl/net_manager.cpp:515-521).  The CRCs
// come from the CSR batch path first (crc32c_span.hip); this kernel is the
// append: a shifted copy plus four bytes per datagram.
//
// A team of 32 lanes takes one datagram and walks its destination in 16-byte
// chunks (one per lane, 512 bytes per team step): a chunk that lies wholly
// inside the payload is one dwordx4 store assembled from a dwordx4 and a dword
// load with v_alignbyte (the source is offset from the destination by 4 i and
// the burst's alignment: any byte shift).  The partial chunk at the head and
// the tail (payload remainder + CRC), which share 16-byte chunks with the
// neighbouring datagrams, go one byte per lane, so no team ever writes a byte
// that is not its own.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"
#include "crc32c_kernels.h"

namespace lnl {

namespace {

constexpr int kThreads = 256;
#ifndef LNL_APPEND_TEAM
#define LNL_APPEND_TEAM 32  // measured: 16 lanes 559 us, 32 lanes 512 us, 64 lanes 613 us per config-3 call
#endif
constexpr uint32_t kTeam = LNL_APPEND_TEAM;  // lanes per datagram
#ifndef LNL_APPEND_STORE_SFX
#define LNL_APPEND_STORE_SFX ""  // chunk stores' cache-policy suffix.  The asm store itself is the gain
                                // (489-493 us against 502 us for the C store: the loop is not unrolled
                                // and the wave reaches its next loads sooner); sc0 is no faster than the
                                // default, sc1 / sc0 sc1 / nt are 15-17 % slower
#endif
#ifndef LNL_APPEND_WGS
#define LNL_APPEND_WGS 16u  // workgroups per CU (teams stride over the datagrams)
#endif
#ifndef LNL_APPEND_NT
#define LNL_APPEND_NT 0  // nontemporal chunk stores (1), loads (2), both (3)
#endif
static_assert(kTeam >= 20 && kTeam <= 64, "one byte per lane covers the head (< 16) and tail (< 20) bytes");

struct __attribute__((packed, aligned(4))) U4a {  // 16 bytes at a 4-byte aligned address
    uint32_t x, y, z, w;
};

#define LNL_G LNL_GLOBAL  // crc32c_device.h

__device__ inline uint8_t out_byte(uint64_t x, uint64_t P1, uint64_t delta, uint32_t crc) {
    return x < P1 ? *LNL_G(const uint8_t, x - delta) : (uint8_t)(crc >> (8u * (uint32_t)(x - P1)));
}

__global__ __launch_bounds__(kThreads) void append_kernel(AppendArgs a) {
    const uint32_t t = (blockIdx.x * kThreads + threadIdx.x) / kTeam;  // global team
    const uint32_t nt = gridDim.x * (kThreads / kTeam);
    const uint32_t q = threadIdx.x % kTeam;  // lane within the team
    const uint64_t o0 = a.off[0];
    const uint64_t dstb = (uint64_t)(uintptr_t)a.dst, srcb = (uint64_t)(uintptr_t)a.base - a.off0;
    // the next datagram's offsets and CRC are fetched one datagram ahead
#if defined(LNL_APPEND_BLOCKED) && LNL_APPEND_BLOCKED  // experiments: team t owns a run of consecutive datagrams
    const uint32_t per = (a.n + nt - 1) / nt;
    const uint64_t i0 = (uint64_t)t * per, iend = i0 + per < a.n ? i0 + per : a.n;
    const uint32_t step = 1;
#else  // the product: teams stride over the datagrams, so the burst is written as one front
    const uint64_t i0 = t, iend = a.n;
    const uint32_t step = nt;
#endif
    uint64_t ns = 0, ne = 0;
    uint32_t ncrc = 0;
    if (i0 < iend) {
        ns = a.off[i0];
        ne = a.off[i0 + 1];
        ncrc = a.crc[i0];
    }
    for (uint32_t i = (uint32_t)i0; i < iend; i += step) {
        const uint64_t s = ns, e = ne;
        const uint32_t crc = ncrc;
        if (i + step < iend) {
            ns = a.off[i + step];
            ne = a.off[i + step + 1];
            ncrc = a.crc[i + step];
        }
        const uint64_t P0 = dstb + (s - o0) + 4ull * i;  // first payload byte in dst
        const uint64_t P1 = P0 + (e - s);                // first CRC byte
        const uint64_t P2 = P1 + 4u;                     // end
        const uint64_t delta = P0 - (srcb + s);          // dst - src, every payload byte
        // whole 16-byte chunks inside the payload: [c0, c1)
        const uint64_t c0 = (P0 + 15u) & ~(uint64_t)15, c1 = P1 & ~(uint64_t)15;
        if (c0 >= c1) {  // shorter than that (< 31 payload bytes): every byte on the byte path
            for (uint64_t x = P0 + q; x < P2; x += kTeam) *LNL_G(uint8_t, x) = out_byte(x, P1, delta, crc);
            continue;
        }
        // the bytes outside them -- the partial head chunk [P0, c0) (< 16) and the
        // tail [c1, P2) (payload remainder + CRC, < 20) -- one per lane, loaded
        // before the chunk loop so that their latency overlaps it
        const uint64_t x0 = P0 + q, x1 = c1 + q;
        const bool b0 = x0 < c0, b1 = x1 < P2;
        const uint8_t v0 = b0 ? out_byte(x0, P1, delta, crc) : 0;
        const uint8_t v1 = b1 ? out_byte(x1, P1, delta, crc) : 0;
        const uint32_t c = (uint32_t)((c0 - delta) & 3u);  // (the same for every chunk)
#if defined(LNL_APPEND_UNROLL) && LNL_APPEND_UNROLL == 2  // experiments
#pragma unroll 2
#endif
        for (uint64_t w = c0 + 16ull * q; w < c1; w += 16ull * kTeam) {
            const uint64_t sw = (w - delta) & ~(uint64_t)3;
#if LNL_APPEND_NT & 2
            const dev::u32x4 vv = __builtin_nontemporal_load(LNL_G(const dev::u32x4, sw));  // (4-byte aligned: unaligned dwordx4)
            const U4a v = {vv[0], vv[1], vv[2], vv[3]};
#else
            const U4a v = *LNL_G(const U4a, sw);
#endif
            uint4 o = make_uint4(v.x, v.y, v.z, v.w);
            if (c) {  // (the fifth dword holds byte w - delta + 15, inside the payload)
                const uint32_t v4 = *LNL_G(const uint32_t, sw + 16);
                o.x = __builtin_amdgcn_alignbyte(v.y, v.x, c);
                o.y = __builtin_amdgcn_alignbyte(v.z, v.y, c);
                o.z = __builtin_amdgcn_alignbyte(v.w, v.z, c);
                o.w = __builtin_amdgcn_alignbyte(v4, v.w, c);
            }
#if defined(LNL_APPEND_DIAG) && (LNL_APPEND_DIAG & 2)
            if (w == 7u) *LNL_G(uint4, w) = o;  // diagnostic build only: no chunk stores (wrong burst)
#elif LNL_APPEND_NT & 1
            __builtin_nontemporal_store(dev::u32x4{o.x, o.y, o.z, o.w}, LNL_G(dev::u32x4, w));
#else  // cache-policy suffix (LNL_APPEND_STORE_SFX; "" for the default policy)
            asm volatile("global_store_dwordx4 %0, %1, off " LNL_APPEND_STORE_SFX ::"v"(w),
                         "v"(dev::u32x4{o.x, o.y, o.z, o.w})
                         : "memory");
#endif
        }
#if defined(LNL_APPEND_DIAG) && (LNL_APPEND_DIAG & 1)
        if (x0 == 7u && x1 == 9u) *LNL_G(uint8_t, x0) = v0 ^ v1;  // diagnostic build only: no head / tail stores (wrong burst)
#else
        if (b0) *LNL_G(uint8_t, x0) = v0;
        if (b1) *LNL_G(uint8_t, x1) = v1;
#endif
    }
}

}  // namespace

hipError_t launch_append(const AppendArgs& a, int cus, hipStream_t stream) {
    // 32 teams in flight per CU's worth of blocks; teams stride over datagrams
    const uint32_t want = (a.n + (kThreads / kTeam) - 1) / (kThreads / kTeam);
    const uint32_t cap = (uint32_t)cus * LNL_APPEND_WGS;
    const uint32_t grid = want < cap ? want : cap;
    hipLaunchKernelGGL(append_kernel, dim3(grid ? grid : 1), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
