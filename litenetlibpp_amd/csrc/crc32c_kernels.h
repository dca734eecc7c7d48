// crc32c_kernels.h -- launch interface between the C ABI (crc32c_api.cpp) and
// the gfx950 kernels (crc32c_kernels.hip).  Internal; not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lnl {

constexpr int kBlockThreads = 256;  // 4 waves; 64 KiB LDS -> 2 workgroups per CU
constexpr int kWavesPerCU = 8;
// the lane-run kernel's workgroup (crc32c_run.hip): 256 threads, two per CU,
// or 512 (one per CU, its 8 waves sharing LDS progress words for issue fairness)
#ifndef LNL_RUN_THREADS
#define LNL_RUN_THREADS 256
#endif
constexpr int kRunThreads = LNL_RUN_THREADS;

enum : int { kModeFixed = 0, kModeCsr = 1, kModeVerify = 2 };

struct BatchArgs {
    const uint8_t* base;   // d_base
    const uint64_t* off;   // CSR offsets (n + 1), modes Csr / Verify
    uint64_t off0;         // subtracted from every offset (host chunking: chunk-relative)
    uint64_t stride;       // mode Fixed
    uint32_t len;          // mode Fixed
    uint32_t n;            // datagrams
    uint32_t* out;         // CRC per datagram (may be null in Verify mode)
    uint8_t* ok;           // Verify mode: 1 = trailing CRC matches
    uint32_t filter;       // Verify mode: ok = 2 when the CRC matches but net_packet::verify fails (lnl_packet.h)
    const uint8_t* dummy;  // 16 readable bytes (library scratch) for idle glds lanes
    const uint32_t* fold;  // LNL_TABLE_WORDS words from lnl_build_tables (device)
    const uint32_t* perm;  // optional: lane datagrams perm[64 b + lane] (pair / segment leftovers)
    const uint4* desc;     // optional, instead of perm + off: lane descriptors desc[64 b + lane]
                           // {datagram, CRC length, start (lo, hi) relative to base} (CSR buckets)
    const uint32_t* perm_n;  // optional (device): number of perm entries, else n
    const uint32_t* tail_xor;  // optional: out[i] ^= tail_xor[i] for all i < n first (CSR uniform path)
    uint32_t xor_n;            // entries of tail_xor
    // optional (CSR span path): the span kernel's control block ([1] the
    // overflow count, the list in perm; [2] == 0: it did not take the batch,
    // so this kernel takes all of it; crc32c_span.h)
    const uint32_t* span_ctl;
};

// Enqueue one batch kernel on `stream` with `grid` workgroups.
hipError_t launch_crc32c_batch(const BatchArgs& a, int mode, int grid, hipStream_t stream);

// Fixed-stride lane-run kernel (crc32c_run.hip).  Covers datagrams
// [0, nb * 64 * k) of the batch: wave-batch wb = g * slices + j, lane l owns
// datagrams g*64q + l*q + j*k + [0, k).
struct RunArgs {
    const uint8_t* base;
    uint64_t stride;       // S >= len
    uint32_t len;          // >= 129
    uint32_t k;            // datagrams per lane run (even)
    uint32_t q;            // lane spacing in datagrams: q * S % 128 == 0, q % k == 0
    uint32_t slices;       // q / k
    uint32_t nb;           // wave-batches
    uint32_t* out;
    const uint32_t* fold;  // LNL_TABLE_WORDS words from lnl_build_tables (device)
};

hipError_t launch_crc32c_run(const RunArgs& a, int grid, hipStream_t stream);

// CSR pre-pass (crc32c_bucket.hip): desc[] = descriptors of the datagrams
// grouped by the number of 128-byte lines they touch.  counts and fill:
// kBucketCounterWords words of device scratch (zeroed by the launch).
constexpr int kBuckets = 64;
constexpr uint32_t kCounterCopies = 16;  // copies of the global bucket counters (atomic contention)
constexpr uint32_t kBucketCounterWords = 2 * kCounterCopies * kBuckets;  // counts + fill
struct BucketArgs {
    const uint8_t* base;
    const uint64_t* off;
    uint64_t off0;
    uint32_t n;
    uint32_t verify;  // verify mode: the CRC covers all but the last 4 bytes
    // position-ordered layouts (LNL_BUCKET_LAYOUT 1, 2 -- 2 is the default):
    // per-workgroup histograms, their per-bucket prefix, bucket totals, and
    // the descriptor count the batch kernel reads as perm_n
    uint32_t* hist;   // groups x kBuckets
    uint32_t* pbase;  // groups x kBuckets
    uint32_t* tot;    // kBuckets
    uint32_t* ctl;    // [0]: descriptors incl. idle padding (64 x batches)
    // atomic layout (LNL_BUCKET_LAYOUT 0)
    uint32_t* counts;
    uint32_t* fill;   // counts + kCounterCopies * kBuckets
    uint4* desc;      // BatchArgs::desc layout, 16-byte aligned
    uint32_t spread;  // window layout: M, windows visited in M sweeps (0: in order)
    uint32_t xcd;     // window layout: a window's batches on one XCD (W = 2048 only)
};

// scratch words (u32) for a bucketed batch of n datagrams, and its layout
size_t bucket_scratch_words(uint32_t n);
void bucket_layout(BucketArgs& a, uint32_t* scratch);
hipError_t launch_csr_buckets(const BucketArgs& a, hipStream_t stream);

// CSR span path (crc32c_span.hip): every line of the stream read once, lane
// g owns segment g; datagram folds batched wave-uniformly through an LDS
// stash.  launch_span enqueues the pre-pass and the kernel;
// the caller then runs the batch kernel over ovf (perm_n = ctl + 1) with
// span_rec / span_ctl set, which completes the cross-segment heads first.
constexpr int kSpanThreads = 512;  // one workgroup (8 waves) per CU
struct SpanArgs {
    const uint8_t* base;
    const uint64_t* off;
    uint64_t off0;
    uint32_t n;
    uint32_t waves;          // resident waves of the kernel's grid (CUs x 8)
    uint32_t* out;
    const uint32_t* tab;     // kSpanTabWords words (lnl_build_span_tables)
    uint32_t* ctl;           // this call's control block: [1] overflow datagrams (0 on entry),
                             // [2] segments (0: the batch kernel takes the whole batch), [3] R
    uint32_t* ctl_next;      // the other block: the next call's, its count zeroed by this call's span kernel
    uint32_t* xch;           // per wave-batch boundary: exchange block (crc32c_span.h kSpanXch*)
    uint64_t epoch;          // this call's exchange epoch (>= 1, one per call on the scratch)
    uint32_t* ovf;           // n: datagrams left to the batch kernel
    // verify modes (kSpanVerify, kSpanFilter): ok[i] instead of out[i]
    uint32_t mode;
    uint8_t* ok;
    // filter + dispatch (kSpanFilter only; null otherwise): the MERGED walk of
    // every datagram, done by the lane its first byte streams through, into
    // one 8-word block per datagram: [count, record 0 .. 6] (kWalkPlain: not a
    // container); dispatch_fix_kernel turns the blocks into counts + records
    uint32_t* wblk;
};
size_t span_scratch_words(uint32_t n, uint32_t waves);
size_t span_scratch_zero_words(uint32_t waves);  // the leading words that must be 0 at allocation
void span_scratch_layout(SpanArgs& a, uint32_t* scratch, uint32_t parity);
hipError_t launch_span(const SpanArgs& a, int grid, hipStream_t stream);

// Outbound layer over a device burst (lnl_append.hip): datagram i of the CSR
// burst to dst + (off[i] - off[0]) + 4 i as payload || LE32(CRC), the CRCs
// from the CSR CRC pass that runs first (crc in).
struct AppendArgs {
    const uint8_t* base;
    const uint64_t* off;
    uint32_t n;
    uint8_t* dst;
    const uint32_t* crc;  // the CSR pass's CRCs
    uint64_t off0;        // datagram i's bytes are base[off[i] - off0 ..) (host-path chunks: off0 = off[0])
};
hipError_t launch_append(const AppendArgs& a, int cus, hipStream_t stream);

// XOR-encryption layer over a batch (lnl_xor.hip), in place.
constexpr uint32_t kXorMaxKey = 256;
#ifndef LNL_XOR_GROUP
#define LNL_XOR_GROUP 32  // lanes per datagram (lnl_xor.hip)
#endif
constexpr uint32_t kXorPerWg = 256u / LNL_XOR_GROUP;  // datagrams a 256-thread workgroup works on at once
struct XorArgs {
    uint8_t* base;
    const uint64_t* off;  // CSR offsets, or null: fixed stride
    uint64_t off0;
    uint64_t stride;
    uint32_t len;
    uint32_t n;
    uint32_t key_len;     // 1 .. kXorMaxKey
    uint8_t key[kXorMaxKey];
};
hipError_t launch_xor_layer(const XorArgs& a, int grid, hipStream_t stream);
// flat fixed-stride XOR (lnl_xor.hip): host-precomputed stepping constants
struct FlatArgs {
    uint64_t span;    // (n - 1) * stride + len bytes
    uint32_t pieces;  // ceil(span / 16)
    uint32_t whole;   // floor(span / 16): pieces entirely inside the span
    uint32_t S, L, K, n;
    uint32_t SK;              // S % K
    uint32_t sd, sr, srk;     // one grid-stride step of 16 T bytes: / S, % S, (% S) % K
};
hipError_t launch_xor_flat(const XorArgs& a, const FlatArgs& f, int grid, int variant, hipStream_t stream);
// flat CSR XOR (lnl_xor.hip): consecutive lanes own whole 16-byte pieces of the
// batch's byte range; `grid` workgroups of 256 threads, each wave a run of chunks
hipError_t launch_xor_csr_flat(const XorArgs& a, int grid, hipStream_t stream);
// streaming CSR XOR (lnl_xor.hip, the product's CSR path): each wave a run of
// 4 KiB chunks, the next 64 datagram starts in registers
hipError_t launch_xor_csr_stream(const XorArgs& a, int grid, hipStream_t stream);
// grid-interleaved CSR XOR (lnl_xor.hip, the product's CSR path): chunk c to
// wave c mod W; `first` = cap >= 1 words of device scratch for the chunk map
// (cap = n + 1 suffices: the map coarsens itself to fit)
hipError_t launch_xor_csr_grid(const XorArgs& a, uint32_t* first, uint32_t cap, int grid, hipStream_t stream);

// Delivered packets of a filtered burst (lnl_dispatch.hip): accepted
// datagrams, MERGED containers cut into their packets.
struct DispatchArgs {
    const uint8_t* base;
    const uint64_t* off;
    uint64_t off0;
    uint32_t n;
    const uint8_t* status;  // lnl_inbound_filter output
    uint32_t* counts;       // n (scratch)
    uint32_t* first;        // n (scratch): exclusive scan of counts
    uint32_t* rec;          // kDispatchRec * n (scratch): (pos << 16 | len), slot-major
    uint64_t* look;         // one-pass: per-workgroup look-back flags, zeroed (null: two passes)
    uint32_t nt;            // nontemporal stores for the cooperative packet writes
    uint64_t* pkt_start;    // cap: packet start relative to base
    uint32_t* pkt_len;      // cap
    uint32_t* pkt_parent;   // cap: datagram index
    uint32_t cap;
    uint32_t* total;        // device: packets delivered (may exceed cap)
    // fused path (dispatch_fix_kernel): the span kernel's walk blocks, and its
    // control block ([2] != 0: the span kernel took the batch and walked it)
    const uint32_t* blk;
    const uint32_t* span_ctl;
    // two-launch form (batches of at most kDispatchPrefixWgs workgroups): the
    // count / fix-up pass leaves each 256-datagram workgroup's packet total
    // here and the emit pass sums its predecessors' (no scan launch; first is
    // unused).  Null: the hipCUB scan of counts into first.
    uint32_t* wgsum;
    // the walk's bound past the datagram (lnl_dispatch_opts.tail, lnl_dispatch.hip):
    // kDispatchTailDatagram stops at it; the other two walk the reference's
    // zero-filled buffer, and pkt_avail (cap, optional) receives the bytes of
    // each packet that lie inside the datagram
    uint32_t tail;
    uint32_t* pkt_avail;
};
constexpr uint32_t kDispatchTailDatagram = 0, kDispatchTailZero = 1, kDispatchTailLayer = 2;
// buffer_size() of the reference's received packet for a wire datagram of
// `wire` bytes: net_packet() allocates 2048 (ensure(1432), net_packet.h:46-49,
// 194-208) and resize() doubles it while it is short
__host__ __device__ inline uint32_t dispatch_ref_capacity(uint32_t wire) {
    uint32_t cap = 2048u;
    while (cap < wire) cap *= 2u;
    return cap;
}
constexpr uint32_t kDispatchPrefixWgs = 8192;
constexpr uint32_t kDispatchRec = 8;  // packets per datagram kept from the counting walk
constexpr uint32_t kWalkBlock = 8;             // fused path: words per datagram block [count, 7 records]
constexpr uint32_t kWalkPlain = 0x80000000u;    // block count: not a container, one packet
size_t dispatch_scan_bytes(uint32_t n);
hipError_t launch_dispatch(const DispatchArgs& a, void* scan_tmp, size_t scan_bytes, hipStream_t stream);
// Fused path (lnl_inbound_filter_dispatch_csr_dev): the fix-up turns the span
// kernel's walk blocks into counts + records (zero for datagrams not
// accepted; walking again only what the blocks cannot hold), then scan + emit
// as above.
hipError_t launch_dispatch_walked(const DispatchArgs& a, void* scan_tmp, size_t scan_bytes, hipStream_t stream);

}  // namespace lnl
