// crc32c_bucket.hip -- CSR pre-pass: group datagrams by the number of
// 128-byte lines they touch (config 3, batched inbound verify).
//
// The batch kernel gives one lane one datagram and a wave as many rows as its
// longest datagram touches lines.  With lengths uniform in 64..1400 B the
// longest of 64 random datagrams almost always spans 12 lines while the mean
// is ~6.7, so nearly half of all row slots would fetch the zero line.  This
// pre-pass writes a permutation `perm` that lists the datagrams bucket by
// bucket (bucket = line count, 0 for empty datagrams, kBuckets-1 for very
// long ones); the batch kernel then takes its 64 lanes from consecutive perm
// entries, so a wave's lanes need the same number of rows.
//
// Two passes over the offsets (8 bytes per datagram each), both cheap next to
// the payload: count per bucket (workgroup histogram in LDS, one global
// atomic per workgroup and bucket), then scatter (the workgroup reserves a
// range per bucket with one global atomic and places its datagrams with their
// LDS ranks).  Order within a bucket depends on atomic order; CRCs are written
// by datagram index, so results do not.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_kernels.h"

namespace lnl {

namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = 16;
constexpr uint32_t kPerBlock = kThreads * kPerThread;

__device__ inline uint32_t bucket_of(const BucketArgs& a, uint32_t i) {
    const uint64_t s = a.off[i], e = a.off[i + 1];
    const uint32_t total = (uint32_t)(e - s);
    const uint32_t len = a.verify ? (total >= 5u ? total - 4u : 0u) : total;
    if (len == 0) return 0;
    const uint64_t abs0 = (uint64_t)(uintptr_t)a.base + (s - a.off0);
    const uint64_t abs1 = abs0 + len - 1u;
    const uint64_t t = (abs1 >> 7) - (abs0 >> 7) + 1u;
    return t < (uint64_t)kBuckets ? (uint32_t)t : (uint32_t)kBuckets - 1u;
}

__global__ __launch_bounds__(kThreads) void bucket_count_kernel(BucketArgs a) {
    __shared__ uint32_t hist[kBuckets];
    if (threadIdx.x < kBuckets) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * kPerBlock + threadIdx.x;
    for (int j = 0; j < kPerThread; ++j) {
        const uint32_t i = i0 + j * kThreads;
        if (i < a.n) atomicAdd(&hist[bucket_of(a, i)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kBuckets && hist[threadIdx.x]) atomicAdd(&a.counts[threadIdx.x], hist[threadIdx.x]);
}

__global__ __launch_bounds__(kThreads) void bucket_scatter_kernel(BucketArgs a) {
    __shared__ uint32_t hist[kBuckets], base[kBuckets];
    if (threadIdx.x < kBuckets) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * kPerBlock + threadIdx.x;
    uint32_t key[kPerThread], rank[kPerThread];
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) {
        const uint32_t i = i0 + j * kThreads;
        key[j] = i < a.n ? bucket_of(a, i) : 0u;
        rank[j] = i < a.n ? atomicAdd(&hist[key[j]], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < kBuckets) {
        // exclusive prefix of the global counts (64 values) + this block's range
        uint32_t before = 0;
        for (uint32_t k = 0; k < threadIdx.x; ++k) before += a.counts[k];
        const uint32_t h = hist[threadIdx.x];
        base[threadIdx.x] = before + (h ? atomicAdd(&a.fill[threadIdx.x], h) : 0u);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) {
        const uint32_t i = i0 + j * kThreads;
        if (i < a.n) a.perm[base[key[j]] + rank[j]] = i;
    }
}

}  // namespace

hipError_t launch_csr_buckets(const BucketArgs& a, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(a.counts, 0, 2 * kBuckets * sizeof(uint32_t), stream);  // counts + fill
    if (e != hipSuccess) return e;
    const uint32_t grid = (a.n + kPerBlock - 1) / kPerBlock;
    hipLaunchKernelGGL(bucket_count_kernel, dim3(grid), dim3(kThreads), 0, stream, a);
    hipLaunchKernelGGL(bucket_scatter_kernel, dim3(grid), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
