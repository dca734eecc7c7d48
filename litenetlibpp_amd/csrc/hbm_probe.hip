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
//   forms 11-13: the same loads on one-shot grids handed out in buffer order
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

// forms 11 / 12 (round 5): one-shot grids, sized to the buffer, so the
// dispatcher hands the buffer out in order -- workgroup b reads the U x 4 KiB
// from b x U x 4 KiB on (U = 1: form 11; U = 4: form 12), global_load_dwordx4 nt
template <int U>
__global__ __launch_bounds__(256) void tile_read(const u32x4* __restrict__ p, size_t n16, uint32_t* __restrict__ sink) {
    const size_t base = (size_t)blockIdx.x * 256u * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        v[u] = base + 256u * u < n16 ? __builtin_nontemporal_load(p + base + 256u * u) : u32x4{0u, 0u, 0u, 0u};
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// form 13: one-shot LDS-DMA, one 8 KiB chunk per wave (form 1 without the striding)
__global__ __launch_bounds__(256) void tile_read_lds(const uint8_t* __restrict__ p, uint32_t chunks) {
    __shared__ __attribute__((aligned(16))) uint4 slot[4 * 64];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t c = blockIdx.x * 4u + wave;
    if (c >= chunks) return;
    const uint8_t* src = p + (size_t)c * 8192u + 16u * lane;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(src + 1024 * i), (void*)(slot + 64 * wave), 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

// forms 2-4: the access shape of a segment-per-lane CSR kernel.  Lane l of
// wave-batch w owns the R = kSegR consecutive 128-byte lines starting at
// line (64 w + l) R and reads one line per step:
//   form 2 / 3: each lane loads its own line into VGPRs (8 x dwordx4, 64
//               different lines per wave-instruction), two lines in flight,
//               default / nt cache policy
//   form 4:     LDS-DMA, glds i fetches piece (lane & 7) of the line of lane
//               8 i + lane / 8 (8 lines per wave-instruction), two rows of
//               the wave in flight, then each lane reads its row back with
//               8 x ds_read_b128 (the CRC kernels' load path)
constexpr uint32_t kSegR = 48;

template <bool kNT>
__device__ inline void load_line(const u32x4* q, u32x4* v) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = kNT ? __builtin_nontemporal_load(q + k) : q[k];
}

template <bool kNT>
__global__ __launch_bounds__(256) void seg_read_vgpr(const uint8_t* __restrict__ p, uint32_t nseg,
                                                     uint32_t* __restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gw = blockIdx.x * 4u + (threadIdx.x >> 6), nw = gridDim.x * 4u;
    uint32_t acc = 0;
    for (uint32_t wb = gw; wb * 64u < nseg; wb += nw) {
        const uint32_t g = wb * 64u + lane;
        const u32x4* q = (const u32x4*)(p + (size_t)(g < nseg ? g : nseg - 1u) * kSegR * 128u);
        u32x4 a[8], b[8];
        load_line<kNT>(q, a);
        load_line<kNT>(q + 8, b);
        for (uint32_t t = 0; t < kSegR; t += 2) {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc ^= a[k].x ^ a[k].y ^ a[k].z ^ a[k].w;
            if (t + 2 < kSegR) load_line<kNT>(q + 8 * (t + 2), a);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc ^= b[k].x ^ b[k].y ^ b[k].z ^ b[k].w;
            if (t + 3 < kSegR) load_line<kNT>(q + 8 * (t + 3), b);
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <int kW>
__global__ __launch_bounds__(64 * kW) void seg_read_lds(const uint8_t* __restrict__ p, uint32_t nseg,
                                                       uint32_t* __restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint4 lds[kW * 2 * 512];  // 2 x 8 KiB per wave
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gw = blockIdx.x * kW + wave, nw = gridDim.x * kW;
    uint4* const buf = lds + wave * 1024;
    const uint32_t sub = lane >> 3, piece = lane & 7u;
    uint32_t acc = 0;
    for (uint32_t wb = gw; wb * 64u < nseg; wb += nw) {
        const uint8_t* base = p + (size_t)wb * 64u * kSegR * 128u;
        const uint32_t last = nseg - 1u - wb * 64u;  // lanes past the batch end re-read its last segment
#define ISSUE(T, B)                                                                                   \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                                   \
        const uint32_t q = 8u * i + sub;                                                              \
        const uint32_t qq = q < last ? q : last;                                                      \
        __builtin_amdgcn_global_load_lds((const void*)(base + ((size_t)qq * kSegR + (T)) * 128u + 16u * piece), \
                                         (void*)((B) + 64 * i), 16, 0, 2);                            \
    }
        ISSUE(0u, buf);
        ISSUE(1u, buf + 512);
        for (uint32_t t = 0; t < kSegR; ++t) {
            uint4* const b = buf + (t & 1u) * 512;
            if (t + 1 < kSegR)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t ra = (uint32_t)(uintptr_t)(b + lane * 8);
            uint4 v0, v1, v2, v3, v4, v5, v6, v7;
            asm volatile(
                "ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:16\n\tds_read_b128 %2, %8 offset:32\n\t"
                "ds_read_b128 %3, %8 offset:48\n\tds_read_b128 %4, %8 offset:64\n\tds_read_b128 %5, %8 offset:80\n\t"
                "ds_read_b128 %6, %8 offset:96\n\tds_read_b128 %7, %8 offset:112\n\ts_waitcnt lgkmcnt(0)"
                : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(v4), "=&v"(v5), "=&v"(v6), "=&v"(v7)
                : "v"(ra) : "memory");
            acc ^= v0.x ^ v1.y ^ v2.z ^ v3.w ^ v4.x ^ v5.y ^ v6.z ^ v7.w;
            if (t + 2 < kSegR) { ISSUE(t + 2u, b); }
        }
#undef ISSUE
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// form 7: the same pieces as form 4 (8 lines per wave-instruction), loaded
// into VGPRs (global_load_dwordx4 nt), two rows in flight in registers, then
// written to an 8 KiB LDS scratch (ds_write_b128 x 8) and read back as the
// lane's own row: half the LDS of form 4 per wave
__global__ __launch_bounds__(256) void seg_read_staged(const uint8_t* __restrict__ p, uint32_t nseg,
                                                       uint32_t* __restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint4 lds[4 * 512];  // 8 KiB per wave
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gw = blockIdx.x * 4u + wave, nw = gridDim.x * 4u;
    uint4* const buf = lds + wave * 512;
    const uint32_t sub = lane >> 3, piece = lane & 7u;
    uint32_t acc = 0;
    for (uint32_t wb = gw; wb * 64u < nseg; wb += nw) {
        const uint8_t* base = p + (size_t)wb * 64u * kSegR * 128u;
        const uint32_t last = nseg - 1u - wb * 64u;
        u32x4 a[8], b[8];
        auto load = [&](uint32_t t, u32x4* v) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t q = 8u * i + sub;
                const uint32_t qq = q < last ? q : last;
                v[i] = __builtin_nontemporal_load((const u32x4*)(base + ((size_t)qq * kSegR + t) * 128u + 16u * piece));
            }
        };
        auto consume = [&](const u32x4* v) {
#pragma unroll
            for (int i = 0; i < 8; ++i) buf[64 * i + lane] = *(const uint4*)&v[i];
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
            const uint4* r = buf + lane * 8;
#pragma unroll
            for (int k = 0; k < 8; ++k) acc ^= r[k].x ^ r[k].y ^ r[k].z ^ r[k].w;
        };
        load(0, a);
        load(1, b);
        for (uint32_t t = 0; t < kSegR; t += 2) {
            consume(a);
            if (t + 2 < kSegR) load(t + 2, a);
            consume(b);
            if (t + 3 < kSegR) load(t + 3, b);
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// forms 8-10: the config-2 lane-run kernel's access shape (crc32c_run.hip):
// lane l of wave-batch w streams the kRunRS = 8 x 1400 bytes of its run, one
// 128-byte line per step, lanes kRunRS apart, 8 lanes' lines per
// wave-instruction; D = kLds + kVgpr rows in flight per wave, kLds of them by
// LDS-DMA (read back as the lane's row), kVgpr into registers (XORed as
// loaded: the probe does not transpose them).  Nothing is computed.
//   form 8: 2 LDS-DMA rows (the run kernel today)
//   form 9: 2 LDS-DMA + 2 VGPR rows
//   form 10: 0 LDS-DMA + 4 VGPR rows
constexpr uint32_t kRunRS = 8u * 1400u;
constexpr uint32_t kRunRows = (kRunRS + 127u) / 128u;

template <int kLds, int kVgpr>
__global__ __launch_bounds__(256) void run_read(const uint8_t* __restrict__ p, uint32_t nruns,
                                                uint32_t* __restrict__ sink) {
    constexpr int D = kLds + kVgpr;
    __shared__ __attribute__((aligned(16))) uint4 lds[4 * (kLds > 0 ? kLds : 1) * 512];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gw = blockIdx.x * 4u + wave, nw = gridDim.x * 4u;
    uint4* const bufs = lds + wave * (kLds > 0 ? kLds : 1) * 512;
    const uint32_t sub = lane >> 3, piece = lane & 7u;
    uint32_t acc = 0;
    for (uint32_t wb = gw; wb * 64u < nruns; wb += nw) {
        const uint8_t* base = p + (size_t)wb * 64u * kRunRS;
        const uint32_t last = nruns - 1u - wb * 64u;
        u32x4 v[kVgpr > 0 ? kVgpr : 1][8];
        auto issue = [&](uint32_t t, int slot) {
            if (t >= kRunRows) return;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t q = 8u * i + sub;
                const uint32_t qq = q < last ? q : last;
                // (the run's last row is a half line: stay inside the run, and
                // so inside the buffer for the last one)
                const uint32_t o = t * 128u + 16u * piece;
                const uint8_t* src = base + (size_t)qq * kRunRS + (o < kRunRS - 16u ? o : kRunRS - 16u);
                if (slot < kLds)
                    __builtin_amdgcn_global_load_lds((const void*)src, (void*)(bufs + slot * 512 + 64 * i), 16, 0, 2);
                else
                    v[slot - kLds][i] = __builtin_nontemporal_load((const u32x4*)src);
            }
        };
#pragma unroll
        for (int j = 0; j < D; ++j) issue(j, j);
        for (uint32_t t = 0; t < kRunRows; t += D) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                if (t + j >= kRunRows) break;
                if (t + j + D <= kRunRows) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(8 * (D - 1)) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (j < kLds) {
                    const uint4* r = bufs + j * 512 + lane * 8;
                    uint4 x[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) x[k] = r[k];
#pragma unroll
                    for (int k = 0; k < 8; ++k) acc ^= x[k].x ^ x[k].w;
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) acc ^= v[j - kLds][k].x ^ v[j - kLds][k].w;
                }
                issue(t + j + D, j);
            }
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// FETCH_SIZE calibration for dword-granular random reads (the dispatch walk's
// access shape, lnl_dispatch.hip): thread t reads
// `words` adjacent dwords (1 or 2: load3's aligned pair) at dword offset
// (t & 7) * 2 of 64-byte sector perm(t) = (t * P) mod S, P odd and S a power
// of two, so that `n` threads touch n distinct sectors exactly once: the
// bytes that must cross the memory bus are n x 64 (one sector each) and the
// kernel wants 4 words x n of them.
__global__ __launch_bounds__(256) void sector_read(const uint32_t* __restrict__ p, uint64_t sectors_mask,
                                                   uint32_t n, uint32_t words, uint32_t* sink) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= n) return;
    const uint64_t sec = ((uint64_t)t * 0x9E3779B97F4A7C15ull) & sectors_mask;  // odd multiplier: a permutation
    const uint32_t* q = p + sec * 16u + (t & 7u) * 2u;
    uint32_t v = q[0];
    if (words > 1u) v ^= q[1];
    if (v == 0x9E3779B9u) sink[0] = v;
}

// the same bytes read as one dword per lane, consecutive lanes on consecutive
// dwords (256 B per wave-instruction: the dispatch emit pass's record reads)
__global__ __launch_bounds__(256) void dword_stream(const uint32_t* __restrict__ p, uint64_t n4, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256u) acc ^= p[i];
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

extern "C" int lnl_probe_dword_stream(const void* d, size_t bytes, uint32_t* d_sink, void* stream) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipLaunchKernelGGL(dword_stream, dim3(cus * 8), dim3(256), 0, (hipStream_t)stream, (const uint32_t*)d,
                       (uint64_t)(bytes / 4), d_sink);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// n distinct random 64-byte sectors of the first `bytes` (a power of two of
// sectors is used: the largest that fits), `words` dwords each; returns the
// sector count used, or a negative code.
extern "C" int64_t lnl_probe_sector_read(const void* d, size_t bytes, uint32_t n, uint32_t words, uint32_t* d_sink,
                                         void* stream) {
    uint64_t sectors = 1;
    while (sectors * 2u * 64u <= bytes) sectors *= 2u;
    if (n == 0 || n > sectors || words < 1 || words > 2) return -22;
    hipLaunchKernelGGL(sector_read, dim3((n + 255u) / 256u), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t*)d, sectors - 1u, n, words, d_sink);
    return hipGetLastError() == hipSuccess ? (int64_t)sectors : -5;
}

extern "C" int lnl_probe_stream_read(const void* d, size_t bytes, uint32_t* d_sink, void* stream, int form) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = cus * 2;
    if (form == 11 || form == 12) {
        const size_t n16 = bytes / 16u, per = 256u * (form == 11 ? 1u : 4u);
        const size_t wgs = (n16 + per - 1u) / per;
        if (wgs == 0 || wgs > 0x7FFFFFFFull) return -22;
        if (form == 11)
            hipLaunchKernelGGL(tile_read<1>, dim3((uint32_t)wgs), dim3(256), 0, (hipStream_t)stream, (const u32x4*)d, n16, d_sink);
        else
            hipLaunchKernelGGL(tile_read<4>, dim3((uint32_t)wgs), dim3(256), 0, (hipStream_t)stream, (const u32x4*)d, n16, d_sink);
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (form == 13) {
        const size_t chunks = bytes / 8192u;
        if (chunks == 0 || chunks > 0xFFFFFFFFull) return -22;
        hipLaunchKernelGGL(tile_read_lds, dim3((uint32_t)((chunks + 3u) / 4u)), dim3(256), 0, (hipStream_t)stream,
                           (const uint8_t*)d, (uint32_t)chunks);
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (form >= 8 && form <= 10) {
        const size_t nruns = bytes / kRunRS;
        if (nruns == 0 || nruns > 0xFFFFFFFFull) return -22;
        const uint32_t nr = (uint32_t)nruns;
        if (form == 8)
            hipLaunchKernelGGL((run_read<2, 0>), dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)d, nr, d_sink);
        else if (form == 9)
            hipLaunchKernelGGL((run_read<2, 2>), dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)d, nr, d_sink);
        else
            hipLaunchKernelGGL((run_read<0, 4>), dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)d, nr, d_sink);
        return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (form >= 2 && form <= 7) {
        const size_t nseg = bytes / (kSegR * 128u);
        if (nseg == 0 || nseg > 0xFFFFFFFFull) return -22;
        const uint32_t ns = (uint32_t)nseg;
        if (form == 4)
            hipLaunchKernelGGL(seg_read_lds<4>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)d, ns,
                               d_sink);
        else if (form == 5)  // one 5-wave workgroup per CU
            hipLaunchKernelGGL(seg_read_lds<5>, dim3(cus), dim3(320), 0, (hipStream_t)stream, (const uint8_t*)d, ns,
                               d_sink);
        else if (form == 6)  // one 6-wave workgroup per CU
            hipLaunchKernelGGL(seg_read_lds<6>, dim3(cus), dim3(384), 0, (hipStream_t)stream, (const uint8_t*)d, ns,
                               d_sink);
        else if (form == 7)
            hipLaunchKernelGGL(seg_read_staged, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)d, ns,
                               d_sink);
        else if (form == 3)
            hipLaunchKernelGGL(seg_read_vgpr<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                               (const uint8_t*)d, ns, d_sink);
        else
            hipLaunchKernelGGL(seg_read_vgpr<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                               (const uint8_t*)d, ns, d_sink);
    } else if (form == 1) {
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
