// crc32c_bucket.hip -- CSR pre-pass: group datagrams by the number of
// 128-byte lines they touch (config 3, batched inbound verify).
//
// The batch kernel gives one lane one datagram and a wave as many rows as its
// longest datagram touches lines.  With lengths uniform in 64..1400 B the
// longest of 64 random datagrams almost always spans 12 lines while the mean
// is ~6.7, so nearly half of all row slots would fetch the zero line.  This
// pre-pass writes one 16-byte descriptor per datagram (index, CRC length,
// start), listed bucket by bucket (bucket = line count, 0 for empty
// datagrams, kBuckets-1 for very long ones); the batch kernel then takes its
// 64 lanes from consecutive descriptors -- one coalesced 16-byte load per lane
// instead of an index plus two random offset reads -- so a wave's lanes need
// the same number of rows.
//
// Three small launches over the offsets (8 bytes per datagram, read twice),
// cheap next to the payload: a histogram per workgroup of 1024 datagrams, a
// per-bucket exclusive scan over the workgroups, then the placement (scanned
// base + LDS rank).  Buckets stay in datagram order and the layout is
// deterministic; see LNL_BUCKET_LAYOUT below for the two measured
// alternatives.  CRCs are written by datagram index, so results never depend
// on the layout.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>

#include "crc32c_kernels.h"

#ifndef LNL_EXPERIMENTS
#define LNL_EXPERIMENTS 0
#endif

namespace lnl {

namespace {

// Descriptor layout (LNL_BUCKET_LAYOUT):
//   0 atomic    bucket after bucket, ranks from global atomics (16 counter
//               copies, so a bucket is 16 interleaved runs), counters memset
//   1 interleave position-ordered buckets, batches interleaved by progress so
//               that neighbouring datagrams are processed together -- parity
//               clean but slower: 0.230 ms per config-3 batch (the batch kernel
//               itself 155 -> 190 us), placing the descriptors 25 us
//   2 ordered   (default) position-ordered buckets, bucket after bucket: ranks
//               from per-workgroup histograms and a per-bucket scan, no global
//               atomics, no memset, deterministic; as fast as 0 (0.174-0.177 ms)
#ifndef LNL_BUCKET_LAYOUT
#define LNL_BUCKET_LAYOUT 2
#endif

constexpr int kThreads = 256;
constexpr int kBucketPerThread = 4;               // bucket count and scatter passes
constexpr uint32_t kBucketPerBlock = kThreads * kBucketPerThread;

// bucket, CRC length and start (relative to base) of datagram i
__device__ inline uint32_t bucket_of(const BucketArgs& a, uint32_t i, uint32_t& len, uint64_t& start) {
    const uint64_t s = a.off[i], e = a.off[i + 1];
    const uint32_t total = (uint32_t)(e - s);
    len = a.verify ? (total >= 5u ? total - 4u : 0u) : total;
    start = s - a.off0;
    if (len == 0) return 0;
    const uint64_t abs0 = (uint64_t)(uintptr_t)a.base + start;
    const uint64_t abs1 = abs0 + len - 1u;
    const uint64_t t = (abs1 >> 7) - (abs0 >> 7) + 1u;
    return t < (uint64_t)kBuckets ? (uint32_t)t : (uint32_t)kBuckets - 1u;
}

__global__ __launch_bounds__(kThreads) void bucket_count_kernel(BucketArgs a) {
    // one histogram per wave (less LDS-atomic contention), summed at the end
    constexpr int kW = kThreads / 64;
    __shared__ uint32_t hist[kW][kBuckets];
    for (int k = threadIdx.x; k < kW * kBuckets; k += kThreads) (&hist[0][0])[k] = 0;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * kBucketPerBlock + threadIdx.x;
    uint32_t key[kBucketPerThread];
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j) {  // all loads first
        const uint32_t i = i0 + j * kThreads;
        uint32_t len;
        uint64_t start;
        key[j] = i < a.n ? bucket_of(a, i, len, start) : kBuckets;
    }
    uint32_t* h = hist[threadIdx.x >> 6];
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j)
        if (key[j] < kBuckets) atomicAdd(&h[key[j]], 1u);
    __syncthreads();
    if (threadIdx.x < kBuckets) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kW; ++w) c += hist[w][threadIdx.x];
        if (c) atomicAdd(&a.counts[(blockIdx.x % kCounterCopies) * kBuckets + threadIdx.x], c);
    }
}

__global__ __launch_bounds__(kThreads) void bucket_scatter_kernel(BucketArgs a) {
    __shared__ uint32_t hist[kBuckets], base[kBuckets], tot[kBuckets], part[kBuckets];
    const uint32_t copy = blockIdx.x % kCounterCopies;
    if (threadIdx.x < kBuckets) {
        // bucket b's range is split into kCounterCopies sub-ranges, one per
        // counter copy: total over copies, and the copies before this one
        uint32_t t = 0, p = 0;
#pragma unroll
        for (uint32_t c = 0; c < kCounterCopies; ++c) {
            const uint32_t v = a.counts[c * kBuckets + threadIdx.x];
            t += v;
            p += c < copy ? v : 0u;
        }
        hist[threadIdx.x] = 0;
        tot[threadIdx.x] = t;
        part[threadIdx.x] = p;
    }
    __syncthreads();
    const uint32_t i0 = blockIdx.x * kBucketPerBlock + threadIdx.x;
    uint32_t key[kBucketPerThread], rank[kBucketPerThread], len[kBucketPerThread];
    uint64_t start[kBucketPerThread];
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j) {  // all loads first
        const uint32_t i = i0 + j * kThreads;
        key[j] = i < a.n ? bucket_of(a, i, len[j], start[j]) : 0u;
    }
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j) {
        const uint32_t i = i0 + j * kThreads;
        rank[j] = i < a.n ? atomicAdd(&hist[key[j]], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < kBuckets) {
        // exclusive prefix of the global counts + this block's range
        uint32_t before = 0;
        for (uint32_t k = 0; k < threadIdx.x; ++k) before += tot[k];
        const uint32_t h = hist[threadIdx.x];
        base[threadIdx.x] = before + part[threadIdx.x] +
                            (h ? atomicAdd(&a.fill[copy * kBuckets + threadIdx.x], h) : 0u);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j) {
        const uint32_t i = i0 + j * kThreads;
        if (i < a.n)
            a.desc[base[key[j]] + rank[j]] =
                make_uint4(i, len[j], (uint32_t)start[j], (uint32_t)(start[j] >> 32));
    }
}

// ---- position-ordered layouts (LNL_BUCKET_LAYOUT 1 and 2) ---------------------
//
// Every bucket is kept in datagram order: ranks from per-workgroup histograms
// and a per-bucket scan (no global atomics, no counter memset).  Layout 2 lists
// bucket after bucket.  Layout 1 also interleaves the buckets' batches by
// progress -- batch j of bucket k (nb_k batches) sits at "time" (j + 1/2) / nb_k,
// ties by bucket -- so that the chip works on a narrow window of the buffer in
// every bucket at once and the second fetch of a line two neighbouring
// datagrams share could hit in L2 / the Infinity Cache; measured slower.
// Each bucket's last batch is padded with idle entries (index n), so batches
// never mix buckets.

// batches of bucket k before time (2j+1) / (2 nb) in the interleaved order,
// counting bucket k2 (nb2 batches); ties go to the lower bucket
__device__ inline uint32_t batches_before(uint32_t j, uint32_t nb, uint32_t k, uint32_t nb2, uint32_t k2) {
    if (nb2 == 0u) return 0u;
    if (k2 == k) return j;
    const uint32_t X = (2u * j + 1u) * nb2;  // compare odd o = 2 j2 + 1: o * nb < X
    const uint32_t t = (X - 1u) / nb;
    uint32_t c = (t + 1u) / 2u;
    if (k2 < k && X % nb == 0u && ((X / nb) & 1u)) ++c;  // o * nb == X: the lower bucket first
    return c < nb2 ? c : nb2;
}

__device__ inline uint32_t merged_batch(uint32_t k, uint32_t j, const uint32_t* nbs) {
    uint32_t b = 0;
#if LNL_BUCKET_LAYOUT == 2  // ordered: bucket after bucket
    for (uint32_t k2 = 0; k2 < k; ++k2) b += nbs[k2];
    return b + j;
#endif
    for (uint32_t k2 = 0; k2 < (uint32_t)kBuckets; ++k2) b += batches_before(j, nbs[k], k, nbs[k2], k2);
    return b;
}

__global__ __launch_bounds__(kThreads) void bucket_hist_kernel(BucketArgs a) {
    constexpr int kW = kThreads / 64;
    __shared__ uint32_t hist[kW][kBuckets];
    for (int k = threadIdx.x; k < kW * kBuckets; k += kThreads) (&hist[0][0])[k] = 0;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * kBucketPerBlock + threadIdx.x;
    uint32_t key[kBucketPerThread];
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j) {  // all loads first
        const uint32_t i = i0 + j * kThreads;
        uint32_t len;
        uint64_t start;
        key[j] = i < a.n ? bucket_of(a, i, len, start) : kBuckets;
    }
    uint32_t* h = hist[threadIdx.x >> 6];
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j)
        if (key[j] < kBuckets) atomicAdd(&h[key[j]], 1u);
    __syncthreads();
    if (threadIdx.x < kBuckets) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kW; ++w) c += hist[w][threadIdx.x];
        a.hist[blockIdx.x * kBuckets + threadIdx.x] = c;
    }
}

// one workgroup per bucket: exclusive scan of its count over the groups
__global__ __launch_bounds__(kThreads) void bucket_scan_kernel(BucketArgs a, uint32_t groups) {
    __shared__ uint32_t part[kThreads];
    const uint32_t k = blockIdx.x;
    const uint32_t per = (groups + kThreads - 1) / kThreads;
    const uint32_t g0 = threadIdx.x * per, g1 = g0 + per < groups ? g0 + per : groups;
    uint32_t sum = 0;
    for (uint32_t g = g0; g < g1; ++g) sum += a.hist[g * kBuckets + k];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < (uint32_t)kThreads; d <<= 1) {  // inclusive Hillis-Steele scan
        const uint32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - sum;
    for (uint32_t g = g0; g < g1; ++g) {
        a.pbase[g * kBuckets + k] = run;
        run += a.hist[g * kBuckets + k];
    }
    if (threadIdx.x == kThreads - 1) a.tot[k] = part[kThreads - 1];
}

__global__ __launch_bounds__(kThreads) void bucket_place_kernel(BucketArgs a) {
    constexpr uint32_t kSpan = kBucketPerBlock / 64u + 1u;  // batches one group can touch per bucket
    __shared__ uint32_t nbs[kBuckets], pb[kBuckets], hist[kBuckets], tbl[kBuckets][kSpan];
    if (threadIdx.x < kBuckets) {
        nbs[threadIdx.x] = (a.tot[threadIdx.x] + 63u) >> 6;
        pb[threadIdx.x] = a.pbase[blockIdx.x * kBuckets + threadIdx.x];
        hist[threadIdx.x] = 0;
    }
    __syncthreads();
    if (threadIdx.x < kBuckets) {
        // interleaved position of every batch this group's datagrams of bucket k land in
        const uint32_t k = threadIdx.x;
        const uint32_t h = a.hist[blockIdx.x * kBuckets + k];
        if (h) {
            const uint32_t j0 = pb[k] >> 6, j1 = (pb[k] + h - 1u) >> 6;
            for (uint32_t j = j0; j <= j1; ++j) tbl[k][j - j0] = merged_batch(k, j, nbs);
        }
        if (blockIdx.x == 0) {
            // idle entries padding bucket k's last batch, and the descriptor count
            const uint32_t t = a.tot[k];
            if (t & 63u) {
                const uint32_t b = merged_batch(k, nbs[k] - 1u, nbs);
                for (uint32_t r = t & 63u; r < 64u; ++r) a.desc[64u * b + r] = make_uint4(a.n, 0u, 0u, 0u);
            }
            if (k == 0) {
                uint32_t nb = 0;
                for (int k2 = 0; k2 < kBuckets; ++k2) nb += nbs[k2];
                a.ctl[0] = 64u * nb;
            }
        }
    }
    const uint32_t i0 = blockIdx.x * kBucketPerBlock + threadIdx.x;
    uint32_t key[kBucketPerThread], rank[kBucketPerThread], len[kBucketPerThread];
    uint64_t start[kBucketPerThread];
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j) {
        const uint32_t i = i0 + j * kThreads;
        key[j] = i < a.n ? bucket_of(a, i, len[j], start[j]) : 0u;
    }
    __syncthreads();  // tbl ready
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j) {
        const uint32_t i = i0 + j * kThreads;
        rank[j] = i < a.n ? atomicAdd(&hist[key[j]], 1u) : 0u;
    }
#pragma unroll
    for (int j = 0; j < kBucketPerThread; ++j) {
        const uint32_t i = i0 + j * kThreads;
        if (i < a.n) {
            const uint32_t k = key[j], r = pb[k] + rank[j];
            const uint32_t b = tbl[k][(r >> 6) - (pb[k] >> 6)];
            a.desc[64u * b + (r & 63u)] = make_uint4(i, len[j], (uint32_t)start[j], (uint32_t)(start[j] >> 32));
        }
    }
}

// ---- window layout (LNL_BUCKET_WINDOW=1 at run time) ---------------------------
//
// One pass instead of three: every workgroup sorts its own window of
// kBucketPerBlock consecutive datagrams by line count (an LDS counting sort)
// and writes their descriptors into the window's own n-slot range.  Batches
// are 64 consecutive descriptors, so a batch spans at most a few line counts
// (the kernel's per-lane framing pads the shorter lanes), there is no global
// histogram or scan, and neighbouring datagrams -- which share a boundary line
// -- are processed at about the same time.  Descriptor order within a line
// count follows LDS atomics (the CRCs do not depend on it).
template <int kPT, int kWinThreads = 512>
__global__ __launch_bounds__(kWinThreads) void bucket_window_kernel(BucketArgs a) {
    __shared__ uint32_t cnt[kBuckets], basek[kBuckets];
    if (threadIdx.x < kBuckets) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t w0 = blockIdx.x * (kWinThreads * kPT);
    uint32_t key[kPT], rank[kPT], len[kPT];
    uint64_t start[kPT];
#pragma unroll
    for (int j = 0; j < kPT; ++j) {
        const uint32_t i = w0 + threadIdx.x + j * kWinThreads;
        key[j] = i < a.n ? bucket_of(a, i, len[j], start[j]) : 0u;
    }
    // odd windows sort by descending line count, so a window and the next one
    // meet on the same count
    if (blockIdx.x & 1u) {
#pragma unroll
        for (int j = 0; j < kPT; ++j) key[j] = kBuckets - 1u - key[j];
    }
#pragma unroll
    for (int j = 0; j < kPT; ++j) {
        const uint32_t i = w0 + threadIdx.x + j * kWinThreads;
        rank[j] = i < a.n ? atomicAdd(&cnt[key[j]], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < 64u) {  // kBuckets == 64: one wave scans the counts
        const uint32_t c = cnt[threadIdx.x];
        uint32_t v = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)v, d, 64);
            if (threadIdx.x >= (uint32_t)d) v += o;
        }
        basek[threadIdx.x] = v - c;
    }
    __syncthreads();
    // spread placement (a.spread = M): the full windows are visited in M sweeps
    // over the buffer, every M-th window per sweep, so the windows the chip
    // works on at once lie M windows apart across the whole buffer instead of
    // side by side (side by side measured 0.215 ms per config-3 call against
    // 0.177-0.179 at M = 4, W = 2048, and 0.187-0.189 for the global layout)
    uint32_t d0 = w0;
    {
        const uint32_t W = kWinThreads * kPT, gf = a.n / W, M = a.spread, K = M ? gf / M : 0u;
        const uint32_t w = blockIdx.x;
        if (K > 1u && w < K * M) d0 = ((w % M) * K + w / M) * W;
    }
    // XCD placement (a.xcd): the window's batches go to batch indices that the
    // persistent grid's first round gives to one XCD (workgroups round-robin
    // over 8 XCDs, 4 waves each), so the boundary lines two neighbouring
    // datagrams share meet in one L2.  Slot s = 8 g + x of a full group of 8:
    // batch q of the window -> 256 g + 32 (q / 4) + 4 x + q % 4.
    constexpr uint32_t kWB = kWinThreads * kPT / 64u;  // batches per window
    const uint32_t slot = d0 / (kWinThreads * kPT);
    const bool xmap = a.xcd && kWB == 32u && slot < (a.n / (kWinThreads * kPT)) / 8u * 8u;
#pragma unroll
    for (int j = 0; j < kPT; ++j) {
        const uint32_t i = w0 + threadIdx.x + j * kWinThreads;
        const uint32_t r = basek[key[j]] + rank[j];
        const uint32_t q = r >> 6;
        const uint32_t pos = xmap ? 64u * (256u * (slot >> 3) + 32u * (q >> 2) + 4u * (slot & 7u) + (q & 3u)) + (r & 63u)
                                  : d0 + r;
        if (i < a.n)
            a.desc[pos] =
                make_uint4(i, len[j], (uint32_t)start[j], (uint32_t)(start[j] >> 32));
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl[0] = a.n;
}
static_assert(kBuckets == 64, "bucket_window_kernel scans the counts with one wave");

}  // namespace


// Descriptor layout of the product build: windows of 2048 datagrams sorted by
// line count, 256-thread workgroups, placed in 4 sweeps.  The
// experiments build (tools/kvariants.py, -DLNL_EXPERIMENTS=1) reads
// LNL_BUCKET_WINDOW=0..6 / LNL_BUCKET_SPREAD / LNL_BUCKET_XCD to select the
// measured alternatives; the product library never reads the environment.
int bucket_window() {
#if LNL_EXPERIMENTS
    static const int w = [] {
        const char* e = getenv("LNL_BUCKET_WINDOW");
        if (!e) return 1;  // default: windows of 2048
        return e[0] >= '1' && e[0] <= '6' ? e[0] - '0' : 0;
    }();
    return w;
#else
    return 1;
#endif
}

size_t bucket_scratch_words(uint32_t n) {
    const size_t groups = ((size_t)n + kBucketPerBlock - 1) / kBucketPerBlock;
    // hist + pbase + tot + ctl (rounded to 16 B), then n descriptors + padding of every bucket
    const size_t head = LNL_BUCKET_LAYOUT ? 2 * groups * kBuckets + kBuckets + 4 : kBucketCounterWords;
    return (head + 3) / 4 * 4 + 4 * ((size_t)n + 64u * kBuckets);
}

void bucket_layout(BucketArgs& a, uint32_t* w) {
    const size_t groups = ((size_t)a.n + kBucketPerBlock - 1) / kBucketPerBlock;
    size_t head;
    if (LNL_BUCKET_LAYOUT) {
        a.hist = w;
        a.pbase = a.hist + groups * kBuckets;
        a.tot = a.pbase + groups * kBuckets;
        a.ctl = a.tot + kBuckets;
        a.counts = a.fill = nullptr;
        head = 2 * groups * kBuckets + kBuckets + 4;
    } else {
        a.counts = w;
        a.fill = w + kCounterCopies * kBuckets;
        a.hist = a.pbase = a.tot = a.ctl = nullptr;
        head = kBucketCounterWords;
    }
    a.desc = (uint4*)(w + (head + 3) / 4 * 4);
}

hipError_t launch_csr_buckets(const BucketArgs& a, hipStream_t stream) {
    const uint32_t groups = (a.n + kBucketPerBlock - 1) / kBucketPerBlock;
    if (LNL_BUCKET_LAYOUT && bucket_window()) {
        // 1: W = 2048 with 256 threads (default; 0.174-0.176 ms per config-3 call
        // against 0.177-0.179 with 512 and 0.175-0.177 with 1024 threads);
        // 2, 3, 4: W = 4096, 8192, 1024 with 512 threads; 5, 6: W = 2048 with
        // 1024 / 512 threads
        const int wv = bucket_window();
        const uint32_t W = wv == 2 ? 4096u : wv == 3 ? 8192u : wv == 4 ? 1024u : 2048u;
        const dim3 g((a.n + W - 1) / W);
        BucketArgs b = a;
        b.spread = 4u;
#if LNL_EXPERIMENTS
        if (const char* e = getenv("LNL_BUCKET_SPREAD")) b.spread = (uint32_t)atoi(e);
        if (const char* e = getenv("LNL_BUCKET_XCD")) b.xcd = (uint32_t)atoi(e);
#endif
        switch (wv) {
            case 2: hipLaunchKernelGGL((bucket_window_kernel<8>), g, dim3(512), 0, stream, b); break;
            case 3: hipLaunchKernelGGL((bucket_window_kernel<16>), g, dim3(512), 0, stream, b); break;
            case 4: hipLaunchKernelGGL((bucket_window_kernel<2>), g, dim3(512), 0, stream, b); break;
            case 5: hipLaunchKernelGGL((bucket_window_kernel<2, 1024>), g, dim3(1024), 0, stream, b); break;
            case 6: hipLaunchKernelGGL((bucket_window_kernel<4>), g, dim3(512), 0, stream, b); break;
            default: hipLaunchKernelGGL((bucket_window_kernel<8, 256>), g, dim3(256), 0, stream, b); break;
        }
        return hipGetLastError();
    }
    if (LNL_BUCKET_LAYOUT) {
        hipLaunchKernelGGL(bucket_hist_kernel, dim3(groups), dim3(kThreads), 0, stream, a);
        hipLaunchKernelGGL(bucket_scan_kernel, dim3(kBuckets), dim3(kThreads), 0, stream, a, groups);
        hipLaunchKernelGGL(bucket_place_kernel, dim3(groups), dim3(kThreads), 0, stream, a);
        return hipGetLastError();
    }
    hipError_t e = hipMemsetAsync(a.counts, 0, kBucketCounterWords * sizeof(uint32_t), stream);  // counts + fill
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(bucket_count_kernel, dim3(groups), dim3(kThreads), 0, stream, a);
    hipLaunchKernelGGL(bucket_scatter_kernel, dim3(groups), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
