// What does a plain device-to-device copy reach on this box?  (development
// probe, round 5: the outbound append's copy kernel moves 0.78 GB read + 0.78 GB
// written per config-3 call in ~316 us; is that the HBM's read+write ceiling?)
//
//   hipcc --offload-arch=gfx950 -O3 tools/copy_ceiling.hip -o tools/copy_ceiling
//   ./tools/copy_ceiling [MB]
//
// Each form copies MB megabytes (default 768, the config-3 payload) between two
// 16-byte aligned buffers; the result is checked once per form.  Rates count
// read + written bytes (2 x MB / time), the convention of the guide's 6.29 TB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// grid-stride, U chunks of 16 B per lane per iteration (loads first, then stores)
template <int U, int NT>
__global__ void __launch_bounds__(256) copy_gs(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT & 1 ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT & 2)
                __builtin_nontemporal_store(v[u], dst + i + u * stride);
            else
                dst[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

// blocked: workgroup b copies one contiguous tile of T x 16 B x 256 lanes
template <int T>
__global__ void __launch_bounds__(256) copy_tile(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
    const size_t base = (size_t)blockIdx.x * 256 * T + threadIdx.x;
    u32x4 v[T];
#pragma unroll
    for (int u = 0; u < T; ++u)
        if (base + u * 256 < n) v[u] = src[base + u * 256];
#pragma unroll
    for (int u = 0; u < T; ++u)
        if (base + u * 256 < n) dst[base + u * 256] = v[u];
}

template <typename F>
double time_us(F&& f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) f();
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1e3 / reps;
}

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 768;
    const size_t bytes = mb << 20, n = bytes / 16;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    u32x4 *s = nullptr, *d = nullptr;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    std::vector<unsigned> h(bytes / 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned)(i * 2654435761u);
    CK(hipMemcpy(s, h.data(), bytes, hipMemcpyHostToDevice));
    const int reps = 20;
    auto check = [&](const char* name) {
        std::vector<unsigned> o(bytes / 4);
        CK(hipMemcpy(o.data(), d, bytes, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < o.size(); i += 4093)
            if (o[i] != h[i]) {
                std::printf("%s: MISMATCH at %zu\n", name, i);
                std::exit(2);
            }
        CK(hipMemset(d, 0, bytes));
    };
    auto report = [&](const char* name, double us) {
        std::printf("%-34s %9.2f us  %7.1f GB/s (r+w)\n", name, us, 2.0 * bytes / us / 1e3);
        std::fflush(stdout);
    };
    report("hipMemcpyAsync D2D", time_us([&] { CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); }, reps));
    check("memcpy");
#define GS(U, NT, WPC)                                                                                  \
    do {                                                                                                \
        const unsigned g = (unsigned)cus * WPC;                                                         \
        report("grid-stride U=" #U " nt=" #NT " wg/CU=" #WPC,                                           \
               time_us([&] { copy_gs<U, NT><<<g, 256>>>(s, d, n); }, reps));                             \
        CK(hipGetLastError());                                                                          \
        check("gs");                                                                                    \
    } while (0)
    GS(1, 0, 8);
    GS(1, 0, 32);
    GS(2, 0, 16);
    GS(4, 0, 8);
    GS(4, 0, 16);
    GS(4, 2, 16);
    GS(4, 1, 16);
    GS(4, 3, 16);
    GS(8, 0, 8);
#define TILE(T)                                                                                          \
    do {                                                                                                 \
        const unsigned g = (unsigned)((n + 256 * T - 1) / (256 * T));                                    \
        report("tile T=" #T, time_us([&] { copy_tile<T><<<g, 256>>>(s, d, n); }, reps));                  \
        CK(hipGetLastError());                                                                           \
        check("tile");                                                                                   \
    } while (0)
    TILE(1);
    TILE(4);
    TILE(8);
    TILE(16);
    CK(hipFree(s));
    CK(hipFree(d));
    return 0;
}
