// crc32c_api.cpp -- the batched (GPU) side of the C ABI, include/lnl_crc32c.h.
//
// Thin: argument checks, per-device lazy state (a 16-byte dummy line the
// kernels point idle LDS-DMA lanes at, the 12 KiB fold tables, the CU count
// for the persistent grid, host-path staging buffers), and kernel launches on
// the caller's stream.
// No batch entry point computes on the CPU: without a usable gfx950 device
// every one of them fails with -ENODEV.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lnl_crc32c.h"
#include "crc32c_bitslice.h"
#include "crc32c_kernels.h"
#include "crc32c_span.h"

#ifndef LNL_EXPERIMENTS
#define LNL_EXPERIMENTS 0  // 1: the experiments build (tools/kvariants.py), never the product
#endif

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(-EIO, "%s: %s", what, hipGetErrorString(e));
}

constexpr int kMaxDevices = 64;

// Host paths (lnl_crc32c_batch_host, lnl_inbound_filter_host,
// lnl_crc32c_append_host and their _ex forms): chunks go round-robin over
// `streams` streams (lnl_host_opts; LNL_HOST_DEFAULT_STREAMS by default), each
// with its own staging slot.  With two, a stream's next H2D waits behind its
// own D2H, so the send side (a D2H as large as its H2D) overlapped the two
// directions only half the time; from three on, the H2D of chunk k + 1 .. k + 3
// runs while chunk k's wire burst comes back.
constexpr int kHostSlots = LNL_HOST_MAX_STREAMS;

// One staging slot: its stream and device buffers, grown on demand.
struct HostSlot {
    hipStream_t stream = nullptr;
    uint8_t* d_bytes = nullptr;
    uint64_t* d_off = nullptr;
    uint32_t* d_out = nullptr;
    uint8_t* d_wire = nullptr;  // append: the chunk's wire burst
    size_t cap_bytes = 0, cap_n = 0, cap_wire = 0;
    // pinned staging for a chunk's small results (CRCs / statuses) when the
    // caller's output array is pageable, and where they go once the chunk is done
    uint8_t* h_stage = nullptr;
    size_t cap_stage = 0;
    void* pend_dst = nullptr;
    size_t pend_bytes = 0;
};

struct DeviceState {
    std::once_flag once;
    int init_rc = 0;
    std::string init_err;
    uint8_t* dummy = nullptr;  // 256 zero bytes of device memory
    uint32_t* fold = nullptr;  // kernel tables (lnl_build_tables), 12.5 KiB
    uint32_t* span_tab = nullptr;  // span kernel's tables (lnl_build_span_tables), 145 KiB
    int cus = 0;
    bool gfx950 = false;
    // host-path staging (guarded by host_mu)
    std::mutex host_mu;
    HostSlot slot[kHostSlots];
};

DeviceState g_dev[kMaxDevices];

int device_state(int dev, DeviceState** out) {
    if (dev < 0 || dev >= kMaxDevices) return fail(-ENODEV, "device index %d out of range", dev);
    DeviceState& S = g_dev[dev];
    std::call_once(S.once, [&] {
        hipDeviceProp_t prop;
        hipError_t e = hipGetDeviceProperties(&prop, dev);
        if (e != hipSuccess) {
            S.init_rc = -ENODEV;
            S.init_err = std::string("hipGetDeviceProperties: ") + hipGetErrorString(e);
            return;
        }
        S.gfx950 = strncmp(prop.gcnArchName, "gfx950", 6) == 0;
        if (!S.gfx950) {
            S.init_rc = -ENODEV;
            S.init_err = std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950";
            return;
        }
        S.cus = prop.multiProcessorCount;
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(dev);
        static uint32_t host_fold[LNL_TABLE_WORDS];
        static uint32_t host_span[lnl::kSpanTabWords];
        static std::once_flag fold_once;
        std::call_once(fold_once, [] {
            lnl_build_tables(host_fold);
            lnl::lnl_build_span_tables(host_span);
        });
        e = hipMalloc(&S.dummy, 256);
        if (e == hipSuccess) e = hipMemset(S.dummy, 0, 256);
        if (e == hipSuccess) e = hipMalloc(&S.fold, sizeof host_fold);
        if (e == hipSuccess) e = hipMemcpy(S.fold, host_fold, sizeof host_fold, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMalloc(&S.span_tab, sizeof host_span);
        if (e == hipSuccess) e = hipMemcpy(S.span_tab, host_span, sizeof host_span, hipMemcpyHostToDevice);
        // CSR / verify calls take their scratch from the stream-ordered pool
        // (hipMallocAsync / hipFreeAsync on the caller's stream).  Keep freed
        // blocks in the pool across synchronisations: with the default
        // threshold (0) the pool trims at every sync and the next call's
        // hipMallocAsync goes back to the driver.
        if (e == hipSuccess) {
            hipMemPool_t pool = nullptr;
            if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess && pool) {
                uint64_t keep = UINT64_MAX;
                (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
            }
        }
        (void)hipSetDevice(cur);
        if (e != hipSuccess) {
            S.init_rc = -ENOMEM;
            S.init_err = std::string("device scratch allocation: ") + hipGetErrorString(e);
        }
    });
    if (S.init_rc) return fail(S.init_rc, "%s", S.init_err.c_str());
    *out = &S;
    return 0;
}

int current_device(DeviceState** S) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail(-ENODEV, "no HIP device: %s", hipGetErrorString(e));
    return device_state(dev, S);
}

// persistent grid of `threads`-thread workgroups for `waves` waves of work
// (at most kWavesPerCU resident waves per CU)
int grid_for_waves(const DeviceState& S, uint32_t waves, int threads = lnl::kBlockThreads) {
    const uint32_t per_wg = (uint32_t)threads / 64;
    const uint32_t wgs = (waves + per_wg - 1) / per_wg;
    const uint32_t cap = (uint32_t)S.cus * (uint32_t)(lnl::kWavesPerCU / per_wg);
    return (int)std::max(1u, std::min(wgs, cap));
}

#ifndef LNL_BATCH_UNCAPPED
#define LNL_BATCH_UNCAPPED 0  // experiments: batch kernel grid not capped at the resident waves
#endif
int launch(const DeviceState& S, lnl::BatchArgs a, int mode, hipStream_t st, uint32_t max_wgs = 0xFFFFFFFFu) {
    a.dummy = S.dummy;
    a.fold = S.fold;
    const uint32_t bw = (a.n + 63u) / 64u, per = (uint32_t)lnl::kBlockThreads / 64u;
    const int want = LNL_BATCH_UNCAPPED ? (int)std::max(1u, (bw + per - 1u) / per) : grid_for_waves(S, bw);
    const int grid = std::min(want, (int)std::min(max_wgs, 0x7FFFFFFFu));
    hipError_t e = lnl::launch_crc32c_batch(a, mode, std::max(grid, 1), st);
    if (e != hipSuccess) return hip_fail(e, "kernel launch");
    return 0;
}

// CSR / verify batches: bucket the datagrams by line count first (crc32c_bucket.hip)
// so that every wave's lanes need the same number of rows.  The descriptors
// live in stream-ordered scratch (hipMallocAsync / hipFreeAsync on `st`), so
// concurrent calls on different streams never share it.  Small batches skip
// the pre-pass (its fixed cost would dominate).
#ifndef LNL_BUCKET_MIN_N
#define LNL_BUCKET_MIN_N 16384
#endif
// CSR kernel selection.  The product library has one path per mode: the span
// kernel for large CSR and status-only verify / filter batches, the bucketed
// batch kernel for verify batches that also want body CRCs.  The experiments
// build (-DLNL_EXPERIMENTS=1, tools/kvariants.py, build/variants/*.so -- never
// loaded by the product path) can send large CSR batches through the bucketed
// batch kernel instead (lnl_crc32c_set_csr_path(4) or LNL_CSR_PATH=bucketed).
// The round-1 experiment kernels (uniform, segment and pair paths, and the
// verify-from-wire epilogue) are kept as tools/experiments/csr_experiment_kernels.patch
// (DESIGN 4.6).
enum CsrPath : int { kPathBucketed = 0, kPathBucketCsr = 4 };
#if !LNL_EXPERIMENTS
constexpr int csr_path() { return kPathBucketed; }
#else
std::atomic<int> g_csr_path{-1};
int csr_path() {
    int p = g_csr_path.load(std::memory_order_relaxed);
    if (p >= 0) return p;
    p = kPathBucketed;
    if (const char* e = getenv("LNL_CSR_PATH")) {
        if (!strcmp(e, "bucketed")) p = kPathBucketCsr;
    }
    int expect = -1;
    g_csr_path.compare_exchange_strong(expect, p);
    return g_csr_path.load();
}

#endif  // LNL_EXPERIMENTS

#ifndef LNL_DISPATCH_SCAN
#define LNL_DISPATCH_SCAN 0  // 1: the hipCUB scan between the dispatch passes at every size (round 4; experiments)
#endif
#ifndef LNL_SPAN_ROUNDS
#define LNL_SPAN_ROUNDS 1u  // wave-batches per resident wave the segment length is chosen for (experiments)
#endif
#ifndef LNL_SPAN_FIX_WGS
#define LNL_SPAN_FIX_WGS 0xFFFFFFFFu  // cap on the batch kernel's grid after the span kernel (experiments)
#endif
// The span path's scratch is kept per (device, stream) across calls: its two
// control blocks (crc32c_span.h kSpanCtlWords) are used by alternate calls and
// each call's span kernel zeroes the other one's overflow count, and its
// wave-batch boundary exchange blocks pair by the call's epoch (nothing is
// reset), so no call needs a memset or a pre-pass launch.  It grows
// stream-ordered (hipFreeAsync / hipMallocAsync on the stream), and the blocks
// are zeroed once when it does.  The cache's mutex is held from the parity's
// choice through the launches, so a stream's calls take the blocks and epochs
// in launch order even from several threads.
//
// Keys.  A stream handle names one stream for every thread, except
// hipStreamPerThread: each thread's launches on it go to that thread's own
// stream, so its scratch is keyed by the thread as well (two threads sharing
// one control block while their kernels run on different streams would race
// on the exchange flags and the overflow count).  nullptr is the legacy null
// stream in this library's launches (it is not built with per-thread default
// streams), one stream for all threads.
// Bound.  At most LNL_STREAM_CACHE streams' scratch is kept per device and map;
// beyond that the least recently used entry is freed.  Its stream may have
// been destroyed, so the free goes on a library-owned stream of the device,
// behind the entry's last use: once more than half the bound is in use on the
// device, every call records an event on its stream when it has enqueued
// everything that reads the entry, and the eviction makes the library stream
// wait for that event (no host or device-wide synchronise, and a caller in
// stream capture is not disturbed by another stream's eviction).  Below half
// the bound no event is recorded: an event record costs 3-5 us a call (round
// 5 A/B, DESIGN round-5 table), and a victim whose last call recorded none -- its stream
// went idle while the cache was small -- is freed after a device synchronise.
// lnl_stream_release frees a stream's entries explicitly, stream-ordered.
// A call holds the cache's mutex from its choice of the entry until that event
// is recorded, so an entry is never evicted or released between a call's
// launches (with_span_scratch, with_xor_map).
struct StreamKey {
    int dev;
    hipStream_t st;
    std::thread::id th;  // hipStreamPerThread only; default otherwise
    bool operator<(const StreamKey& o) const {
        if (dev != o.dev) return dev < o.dev;
        if (st != o.st) return std::less<hipStream_t>()(st, o.st);
        return th < o.th;
    }
};

StreamKey stream_key(hipStream_t st) {
    StreamKey k{0, st, std::thread::id()};
    (void)hipGetDevice(&k.dev);
    if (st == hipStreamPerThread) k.th = std::this_thread::get_id();
    return k;
}

#ifndef LNL_SCRATCH_EVENTS
#define LNL_SCRATCH_EVENTS 1  // 0 (experiments): never record the last-use event
#endif
// The last-use event only orders a free on the library stream of the same device
#ifndef LNL_SCRATCH_EVENT_FLAGS
#define LNL_SCRATCH_EVENT_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif
#ifndef LNL_SCRATCH_EVENT_FROM
#define LNL_SCRATCH_EVENT_FROM (LNL_STREAM_CACHE / 2)  // entries on the device before calls record events
#endif

struct SpanScratch {
    uint32_t* buf = nullptr;
    size_t words = 0;
    uint64_t calls = 0;          // span path: calls made on it (the control block parity and the exchange epoch)
    uint64_t used = 0;           // LRU tick
    hipEvent_t done = nullptr;   // recorded after the last call's launches that read buf, when `fence`
    bool fence = false;          // this call records `done` (the cache is past LNL_SCRATCH_EVENT_FROM)
    bool fenced = false;         // the last call did record it
};

// the library's own stream on the current device (evictions free on it)
hipStream_t library_stream(int dev) {
    static std::mutex mu;
    static hipStream_t st[kMaxDevices] = {};
    std::lock_guard<std::mutex> lk(mu);
    if (dev < 0 || dev >= kMaxDevices) return nullptr;
    if (!st[dev] && hipStreamCreateWithFlags(&st[dev], hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        st[dev] = nullptr;
    }
    return st[dev];
}

struct ScratchCache {
    std::mutex mu;
    std::map<StreamKey, SpanScratch> m;
    uint64_t tick = 0;

    // the entry for st, at least `words` long (the first zero_words zeroed
    // whenever it is (re)allocated, and its call count restarted); evicts
    // beyond the bound.  Caller holds mu.
    int get(hipStream_t st, size_t words, size_t zero_words, SpanScratch** out) {
        const StreamKey key = stream_key(st);
        SpanScratch& s = m[key];
        s.used = ++tick;
        size_t on_dev = 0;
        for (auto& kv : m) on_dev += kv.first.dev == key.dev;
        s.fence = LNL_SCRATCH_EVENTS && on_dev > (size_t)LNL_SCRATCH_EVENT_FROM;
        if (s.fence && !s.done) {
            hipError_t e = hipEventCreateWithFlags(&s.done, LNL_SCRATCH_EVENT_FLAGS);
            if (e != hipSuccess) {
                s.done = nullptr;
                return hip_fail(e, "hipEventCreate");
            }
        }
        if (s.words < words) {
            const size_t grow = words + words / 4;  // headroom: batches of similar sizes reuse it
            if (s.buf) (void)hipFreeAsync(s.buf, st);
            s.buf = nullptr;
            s.words = 0;
            hipError_t e = hipMallocAsync((void**)&s.buf, grow * sizeof(uint32_t), st);
            if (e != hipSuccess) return fail(-ENOMEM, "hipMallocAsync(%zu): %s", grow * 4, hipGetErrorString(e));
            if (zero_words && (e = hipMemsetAsync(s.buf, 0, zero_words * sizeof(uint32_t), st)) != hipSuccess)
                return hip_fail(e, "hipMemsetAsync");
            s.words = grow;
            s.calls = 0;
        }
        *out = &s;
        evict(key);
        return 0;
    }

    // a call's launches that read the entry are enqueued on st.  Caller holds mu.
    static void used_by(SpanScratch* s, hipStream_t st) {
        if (!s) return;
        s->fenced = s->fence && s->done && hipEventRecord(s->done, st) == hipSuccess;
    }

    void evict(const StreamKey& keep) {
        size_t on_dev = 0;
        for (auto& kv : m) on_dev += kv.first.dev == keep.dev;
        if (on_dev <= (size_t)LNL_STREAM_CACHE) return;
        auto victim = m.end();
        for (auto it = m.begin(); it != m.end(); ++it) {
            const bool same = !(it->first < keep) && !(keep < it->first);
            if (it->first.dev == keep.dev && !same && (victim == m.end() || it->second.used < victim->second.used))
                victim = it;
        }
        if (victim == m.end()) return;
        // its stream may be gone: free on the library stream, behind its last
        // use (its event, or a device synchronise when its last call recorded none)
        hipStream_t ls = library_stream(keep.dev);
        SpanScratch& v = victim->second;
        if (!v.fenced || !ls) (void)hipDeviceSynchronize();
        else (void)hipStreamWaitEvent(ls, v.done, 0);
        if (v.buf) {
            if (ls)
                (void)hipFreeAsync(v.buf, ls);
            else
                (void)hipFree(v.buf);
        }
        if (v.done) (void)hipEventDestroy(v.done);
        m.erase(victim);
    }

    void release(hipStream_t st) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = m.find(stream_key(st));
        if (it == m.end()) return;
        if (it->second.buf) (void)hipFreeAsync(it->second.buf, st);
        if (it->second.done) (void)hipEventDestroy(it->second.done);
        m.erase(it);
    }
};

ScratchCache g_span_cache;  // span path: mu held from the parity's choice through the launches

int span_scratch(hipStream_t st, size_t words, size_t zero_words, SpanScratch** s) {
    return g_span_cache.get(st, words, zero_words, s);
}

// The CSR XOR kernel's chunk map (lnl_xor.hip), kept per (device, stream) like
// the span scratch: each call's map kernel rewrites the words its XOR kernel
// reads, in stream order, so calls on one stream share it.  fn(map) enqueues
// the launches that use it, under the cache's mutex.
ScratchCache g_xor_cache;

template <typename F>
int with_xor_map(hipStream_t st, size_t words, F&& fn) {
    std::lock_guard<std::mutex> lk(g_xor_cache.mu);
    SpanScratch* s = nullptr;
    if (int rc = g_xor_cache.get(st, words, 0, &s)) return rc;
    const int rc = fn(s->buf);
    ScratchCache::used_by(s, st);
    return rc;
}

// CSR batches (product path): the span kernel (crc32c_span.hip: every line read
// once, one 512-thread workgroup per CU; no pre-pass), then the batch kernel,
// which completes the cross-wave-batch heads and takes the datagrams the span
// kernel leaves (three or more segments; device-side count), or the whole batch
// when the span kernel does not take it.
// (span_mode: kSpanCrc -> out[i]; kSpanVerify / kSpanFilter -> ok[i], the
// overflow datagrams through the batch kernel in verify mode)
int no_after(const uint32_t*) { return 0; }

// (after(ctl): launches that read this call's span control block, enqueued
// before the cache's mutex is released -- the fused dispatch's fix-up)
template <typename F = decltype(&no_after)>
int launch_csr_span(const DeviceState& S, const lnl::BatchArgs& a, hipStream_t st, uint32_t span_mode = lnl::kSpanCrc,
                    uint32_t* walk_blocks = nullptr, F&& after = &no_after) {
    lnl::SpanArgs g{};
    g.mode = span_mode;
    g.wblk = walk_blocks;  // filter + dispatch: the MERGED walk in the same pass
    g.ok = a.ok;
    g.base = a.base;
    g.off = a.off;
    g.off0 = a.off0;
    g.n = a.n;
    g.waves = (uint32_t)S.cus * (uint32_t)(lnl::kSpanThreads / 64) * LNL_SPAN_ROUNDS;
    g.out = a.out;
    g.tab = S.span_tab;
    std::lock_guard<std::mutex> lk(g_span_cache.mu);
    SpanScratch* sc = nullptr;
    if (int rc = span_scratch(st, lnl::span_scratch_words(a.n, g.waves), lnl::span_scratch_zero_words(g.waves), &sc))
        return rc;
    // control block: alternate calls; exchange epoch: one per call (>= 1: the
    // zeroed arrival words hold epoch 0).  Both advance once the span kernel
    // is launched -- it zeroes the next block's count itself, so a failed
    // batch-kernel launch below leaves nothing stale for the next call.
    lnl::span_scratch_layout(g, sc->buf, (uint32_t)(sc->calls & 1u));
    g.epoch = sc->calls + 1u;
    hipError_t e = lnl::launch_span(g, S.cus, st);
    if (e != hipSuccess) return hip_fail(e, "span kernel launch");
    ++sc->calls;
    int rc = 0;
#if !(defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 32))  // (diagnostic build only: no batch kernel)
    lnl::BatchArgs o = a;
    o.perm = g.ovf;
    o.perm_n = g.ctl + 1;
    o.span_ctl = g.ctl;
    rc = launch(S, o, span_mode == lnl::kSpanCrc ? lnl::kModeCsr : lnl::kModeVerify, st, LNL_SPAN_FIX_WGS);
#endif
    if (rc == 0) rc = after(g.ctl);
    ScratchCache::used_by(sc, st);
    return rc;
}

int launch_csr(const DeviceState& S, lnl::BatchArgs a, int mode, hipStream_t st) {
    if (a.n < LNL_BUCKET_MIN_N) return launch(S, a, mode, st);
    if (mode == lnl::kModeCsr && csr_path() == kPathBucketed) return launch_csr_span(S, a, st);
    void* scratch = nullptr;
    const size_t bytes = lnl::bucket_scratch_words(a.n) * sizeof(uint32_t);
    hipError_t e = hipMallocAsync(&scratch, bytes, st);
    if (e != hipSuccess) return fail(-ENOMEM, "hipMallocAsync(%zu): %s", bytes, hipGetErrorString(e));
    lnl::BucketArgs b{};
    b.base = a.base;
    b.off = a.off;
    b.off0 = a.off0;
    b.n = a.n;
    b.verify = mode == lnl::kModeVerify;
    lnl::bucket_layout(b, (uint32_t*)scratch);
    e = lnl::launch_csr_buckets(b, st);
    int rc = 0;
    if (e != hipSuccess) {
        rc = hip_fail(e, "bucket pre-pass launch");
    } else {
        a.desc = b.desc;
        a.perm_n = b.ctl;  // null for the atomic layout (n descriptors)
        rc = launch(S, a, mode, st);
    }
    e = hipFreeAsync(scratch, st);
    if (rc == 0 && e != hipSuccess) rc = hip_fail(e, "hipFreeAsync");
    return rc;
}

// Lane-run plan for a fixed-stride batch (crc32c_run.hip): how many leading
// datagrams the run kernel covers.  0 = use the batch kernel for all.
// Runs of 4 datagrams per lane, one batch (64 runs) per wave and a grid that
// is not capped at the resident waves: the dispatcher then hands out the
// batches in memory order and the chip reads inside a narrower window of the
// batch.  Round 5: config 2 227.4 against 230.5 us for runs of 8
// on a capped grid, 4000-byte strides 159.7 against 202.5, 512-byte 179.8
// against 222.2, 256-byte 189.3 against 200.5 (1404-byte strides 236.5
// against 235.2).
#ifndef LNL_RUN_K
#define LNL_RUN_K 4
#endif
uint32_t run_plan(size_t stride, uint32_t len, uint32_t n, lnl::RunArgs& r) {
#if defined(LNL_NO_RUN)  // experiment builds only (tools/kvariants.py): batch kernel for everything
    return 0;
#endif
    if (len < 129u || stride < len || stride > (1u << 20)) return 0;
    const uint32_t S = (uint32_t)stride;
    const uint32_t low = S & (0u - S);  // largest power of two dividing S
    const uint32_t p = low >= 128u ? 1u : 128u / low;
    const uint32_t k = LNL_RUN_K;
    uint32_t q = p > k ? p : k;
#ifdef LNL_RUN_QMIN  // experiments: lanes at least QMIN datagrams apart (a multiple of q)
    while (q < (uint32_t)LNL_RUN_QMIN) q *= 2u;
#endif
    if ((uint64_t)64u * q * S >= (1ull << 31)) return 0;  // per-lane 32-bit offsets
    const uint32_t super = 64u * q;
    const uint32_t n_main = n - n % super;
    if (n_main == 0) return 0;
    r.stride = S;
    r.len = len;
    r.k = k;
    r.q = q;
    r.slices = q / k;
    r.nb = n_main / (64u * k);
    return n_main;
}


}  // namespace

extern "C" const char* lnl_crc32c_last_error(void) { return g_err.c_str(); }

extern "C" int lnl_stream_release(void* hip_stream) {
    g_span_cache.release((hipStream_t)hip_stream);
    g_xor_cache.release((hipStream_t)hip_stream);
    return 0;
}

extern "C" int lnl_diag_fill_span_arrivals(void* hip_stream, uint64_t value) {
    const hipStream_t st = (hipStream_t)hip_stream;
    DeviceState* S;
    if (int rc = current_device(&S)) return rc;
    std::lock_guard<std::mutex> lk(g_span_cache.mu);
    auto it = g_span_cache.m.find(stream_key(st));
    if (it == g_span_cache.m.end() || !it->second.buf) return fail(-ENOENT, "no span scratch kept for this stream");
    // only what an earlier call could have left: an epoch up to the calls
    // made (a later one could pair with a future call's arrival)
    if ((value >> 2) > it->second.calls)
        return fail(-EINVAL, "arrival epoch %llu is past the %llu calls made on this stream",
                    (unsigned long long)(value >> 2), (unsigned long long)it->second.calls);
    const uint32_t waves = (uint32_t)S->cus * (uint32_t)(lnl::kSpanThreads / 64) * LNL_SPAN_ROUNDS;
    const size_t blocks = lnl::span_max_segments(waves) / 64u;
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    std::vector<uint64_t> v(blocks, value);
    uint32_t* xch = it->second.buf + 2 * lnl::kSpanCtlWords + lnl::kSpanXchFlag;  // (span_scratch_layout)
    e = hipMemcpy2D(xch, lnl::kSpanXchWords * 4u, v.data(), 8, 8, blocks, hipMemcpyHostToDevice);
    return e == hipSuccess ? 0 : hip_fail(e, "hipMemcpy2D");
}

extern "C" int lnl_crc32c_abi_version(void) { return LNL_CRC32C_ABI_VERSION; }

#if LNL_EXPERIMENTS
// Experiments build only (not in include/lnl_crc32c.h, not in the product
// library): selects the kernel of large CSR / verify batches (0 bucketed batch
// kernel, 1 uniform, 2 segment, 3 pair; see csr_path above).  Returns the
// previous path, or -EINVAL.
extern "C" int lnl_crc32c_set_csr_path(int path) {
    if (path != kPathBucketed && path != kPathBucketCsr) return fail(-EINVAL, "CSR path %d not built", path);
    const int prev = csr_path();
    g_csr_path.store(path);
    return prev;
}
#endif

extern "C" int lnl_crc32c_batch_fixed_dev(const uint8_t* d_base, size_t stride, uint32_t len,
                                          uint32_t n, uint32_t* d_out, void* hip_stream) {
    if (n == 0) return 0;
    if (!d_out) return fail(-EINVAL, "d_out is NULL");
    if (!d_base && len) return fail(-EINVAL, "d_base is NULL");
    DeviceState* S;
    if (int rc = current_device(&S)) return rc;
    hipStream_t st = (hipStream_t)hip_stream;
    if (len == 0) {  // CRC-32C of zero bytes is 0
        hipError_t e = hipMemsetAsync(d_out, 0, (size_t)n * 4u, st);
        return e == hipSuccess ? 0 : hip_fail(e, "hipMemsetAsync");
    }
    lnl::RunArgs r{};
    const uint32_t n_main = run_plan(stride, len, n, r);
    if (n_main) {
        r.base = d_base;
        r.out = d_out;
        r.fold = S->fold;
#ifndef LNL_RUN_UNCAPPED
#define LNL_RUN_UNCAPPED 1  // one batch per wave, grid in batch order (0: capped at the resident waves)
#endif
        const int grid = LNL_RUN_UNCAPPED ? (int)((r.nb + lnl::kRunThreads / 64 - 1) / (lnl::kRunThreads / 64))
                                          : grid_for_waves(*S, r.nb, lnl::kRunThreads);
        hipError_t e = lnl::launch_crc32c_run(r, grid, st);
        if (e != hipSuccess) return hip_fail(e, "kernel launch");
        if (n_main == n) return 0;
    }
    lnl::BatchArgs a{};
    a.base = d_base + (size_t)n_main * stride;
    a.stride = stride;
    a.len = len;
    a.n = n - n_main;
    a.out = d_out + n_main;
    return launch(*S, a, lnl::kModeFixed, st);
}

extern "C" int lnl_crc32c_batch_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                                        uint32_t* d_out, void* hip_stream) {
    if (n == 0) return 0;
    if (!d_out || !d_off) return fail(-EINVAL, "d_out / d_off is NULL");
    if (!d_base) return fail(-EINVAL, "d_base is NULL");
    DeviceState* S;
    if (int rc = current_device(&S)) return rc;
    lnl::BatchArgs a{};
    a.base = d_base;
    a.off = d_off;
    a.n = n;
    a.out = d_out;
    return launch_csr(*S, a, lnl::kModeCsr, (hipStream_t)hip_stream);
}

namespace {
int verify_csr(const uint8_t* d_base, const uint64_t* d_off, uint32_t n, uint8_t* d_ok, uint32_t* d_crc,
               uint32_t filter, void* hip_stream);
}  // namespace

namespace {
// The outbound layer over a device burst: the CSR CRC pass into crc, then the
// copy kernel (lnl_append.hip) writes the wire burst.
int append_csr(const DeviceState& S, const lnl::BatchArgs& src, uint8_t* d_dst, uint32_t* crc, hipStream_t st) {
    if (!crc) return fail(-EINVAL, "the append needs a CRC buffer");
    lnl::BatchArgs a = src;
    a.out = crc;
    if (int rc = launch_csr(S, a, lnl::kModeCsr, st)) return rc;
    lnl::AppendArgs p{src.base, src.off, src.n, d_dst, crc, src.off0};
    hipError_t e = lnl::launch_append(p, S.cus, st);
    return e == hipSuccess ? 0 : hip_fail(e, "append kernel launch");
}
}  // namespace

// The outbound layer over a device burst: the CSR CRC pass, then the copy
// kernel (lnl_append.hip); the CRCs into d_crc when it is not null (else into
// stream-ordered scratch).
extern "C" int lnl_crc32c_append_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n, uint8_t* d_dst,
                                         uint32_t* d_crc, void* hip_stream) {
    if (n == 0) return 0;
    if (!d_off || !d_dst) return fail(-EINVAL, "d_off / d_dst is NULL");
    if (!d_base) return fail(-EINVAL, "d_base is NULL");
    DeviceState* S;
    if (int rc = current_device(&S)) return rc;
    const hipStream_t st = (hipStream_t)hip_stream;
    uint32_t* crc = d_crc;
    const bool scratch = !crc;
    if (scratch) {
        hipError_t e = hipMallocAsync((void**)&crc, (size_t)n * sizeof(uint32_t), st);
        if (e != hipSuccess) return fail(-ENOMEM, "hipMallocAsync(%zu): %s", (size_t)n * 4, hipGetErrorString(e));
    }
    lnl::BatchArgs a{};
    a.base = d_base;
    a.off = d_off;
    a.n = n;
    int rc = append_csr(*S, a, d_dst, crc, st);
    if (scratch) {
        hipError_t e = hipFreeAsync(crc, st);
        if (rc == 0 && e != hipSuccess) rc = hip_fail(e, "hipFreeAsync");
    }
    return rc;
}

extern "C" int lnl_crc32c_verify_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                                         uint8_t* d_ok, uint32_t* d_crc, void* hip_stream) {
    return verify_csr(d_base, d_off, n, d_ok, d_crc, 0u, hip_stream);
}

extern "C" int lnl_inbound_filter_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                                          uint8_t* d_status, void* hip_stream) {
    return verify_csr(d_base, d_off, n, d_status, nullptr, 1u, hip_stream);
}

namespace {
int verify_csr(const uint8_t* d_base, const uint64_t* d_off, uint32_t n, uint8_t* d_ok, uint32_t* d_crc,
               uint32_t filter, void* hip_stream) {
    if (n == 0) return 0;
    if (!d_ok || !d_off) return fail(-EINVAL, "d_ok / d_off is NULL");
    if (!d_base) return fail(-EINVAL, "d_base is NULL");
    DeviceState* S;
    if (int rc = current_device(&S)) return rc;
    lnl::BatchArgs a{};
    a.base = d_base;
    a.off = d_off;
    a.n = n;
    a.out = d_crc;
    a.ok = d_ok;
    a.filter = filter;
    hipStream_t st = (hipStream_t)hip_stream;
    const int path = csr_path();
    // large batches, status only: the span kernel (every line read once), the
    // whole datagram's CRC against the residue; with body CRCs wanted (d_crc)
    // the bucketed batch kernel, which computes them
    if (n >= LNL_BUCKET_MIN_N && !d_crc && path == kPathBucketed)
        return launch_csr_span(*S, a, st, filter ? lnl::kSpanFilter : lnl::kSpanVerify);
    return launch_csr(*S, a, lnl::kModeVerify, st);
}
}  // namespace

// Host-resident batch: chunks of whole datagrams go round-robin over the
// call's streams (lnl_host_opts.streams); each chunk is H2D (bytes + offsets)
// -> kernel (offsets rebased by off0) -> D2H (CRCs / statuses / the wire
// burst).  Stream order makes buffer reuse safe; the streams overlap one
// chunk's copies with the others' kernels and copies in the other direction.
namespace {
// Host-resident CSR batch through `device` (lnl_crc32c_batch_host,
// lnl_inbound_filter_host, lnl_crc32c_append_host and their _ex forms).
enum HostMode : uint32_t { kHostCrc = 0, kHostFilter = 1, kHostAppend = 2 };
// kHostCrc: h_out is u32 CRCs; kHostFilter: u8 inbound status codes;
// kHostAppend: h_out is the wire burst (payload || LE32(CRC) per datagram,
// back to back) and h_crc (optional) the CRCs

// The resolved lnl_host_opts of one call.
struct HostPlan {
    int streams = LNL_HOST_DEFAULT_STREAMS;
    uint32_t chunk_n = 1u << 16;
    size_t chunk_bytes = size_t(64) << 20;
};

int host_plan(const lnl_host_opts* o, HostPlan* p) {
    *p = HostPlan{};
    if (!o) return 0;
    if (o->size < sizeof(lnl_host_opts)) return fail(-EINVAL, "lnl_host_opts.size %u < %zu", o->size, sizeof(lnl_host_opts));
    if (o->reserved) return fail(-EINVAL, "lnl_host_opts.reserved must be 0");
    if (o->streams > (uint32_t)LNL_HOST_MAX_STREAMS)
        return fail(-EINVAL, "lnl_host_opts.streams %u > %d", o->streams, LNL_HOST_MAX_STREAMS);
    if (o->streams) p->streams = (int)o->streams;
    if (o->chunk_datagrams) p->chunk_n = o->chunk_datagrams;
    if (o->chunk_bytes) p->chunk_bytes = (size_t)o->chunk_bytes;
    return 0;
}

// Slot k holds at least these sizes (its stream created on first use; buffers
// regrown only when a call needs more).  Freeing a slot's buffers is safe
// here: the previous call on this device drained every slot's stream.
int slot_ready(HostSlot& s, size_t need_bytes, size_t need_n, size_t need_wire, bool stage) {
    hipError_t e;
    if (!s.stream && (e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess)
        return hip_fail(e, "hipStreamCreate");
    if (need_bytes > s.cap_bytes || need_n > s.cap_n) {
        (void)hipFree(s.d_bytes);
        (void)hipFree(s.d_off);
        (void)hipFree(s.d_out);
        s.d_bytes = nullptr;
        s.d_off = nullptr;
        s.d_out = nullptr;
        s.cap_bytes = s.cap_n = 0;
        const size_t nb = std::max<size_t>(need_bytes, 256);
        if ((e = hipMalloc(&s.d_bytes, nb)) != hipSuccess || (e = hipMalloc(&s.d_off, (need_n + 1) * 8)) != hipSuccess ||
            (e = hipMalloc(&s.d_out, need_n * 4)) != hipSuccess)
            return fail(-ENOMEM, "staging allocation: %s", hipGetErrorString(e));
        s.cap_bytes = nb;
        s.cap_n = need_n;
    }
    if (stage && need_n * 4 > s.cap_stage) {  // pinned result staging: only for a pageable output array
        (void)hipHostFree(s.h_stage);
        s.h_stage = nullptr;
        s.cap_stage = 0;
        if ((e = hipHostMalloc((void**)&s.h_stage, need_n * 4, hipHostMallocDefault)) != hipSuccess)
            return fail(-ENOMEM, "pinned staging allocation: %s", hipGetErrorString(e));
        s.cap_stage = need_n * 4;
    }
    s.pend_dst = nullptr;
    s.pend_bytes = 0;
    if (need_wire > s.cap_wire) {  // the wire staging: append calls only
        (void)hipFree(s.d_wire);
        s.d_wire = nullptr;
        s.cap_wire = 0;
        if ((e = hipMalloc(&s.d_wire, need_wire)) != hipSuccess)
            return fail(-ENOMEM, "wire staging allocation: %s", hipGetErrorString(e));
        s.cap_wire = need_wire;
    }
    return 0;
}

// Page-locked (hipHostMalloc / hipHostRegister) host memory: the DMA engines
// copy into it directly.  Into pageable memory a D2H goes through the runtime's
// own staging and holds up the pipeline (config 5 with a pageable CRC array:
// 50.2 against 53.9 GB/s, tools/host_path_probe.py).
// Both ends of the range are checked (a range that starts in a pinned block
// and runs on into pageable memory stages); a range whose two ends are pinned
// is taken as pinned throughout -- one hipHostMalloc / hipHostRegister block,
// as the callers allocate it.
bool host_pinned(const void* p, size_t bytes) {
    auto one = [](const void* q) {
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, q) != hipSuccess) {
            (void)hipGetLastError();  // (pageable memory: an error, not sticky)
            return false;
        }
        return at.type == hipMemoryTypeHost;
    };
    return one(p) && (bytes <= 1 || one((const uint8_t*)p + bytes - 1));
}

// A slot's staged results of its previous chunk to the caller's array (the
// chunk is done once its stream is)
int host_unstage(HostSlot& s) {
    if (!s.pend_bytes) return 0;
    hipError_t e = hipStreamSynchronize(s.stream);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    memcpy(s.pend_dst, s.h_stage, s.pend_bytes);
    s.pend_dst = nullptr;
    s.pend_bytes = 0;
    return 0;
}

int host_batch(const uint8_t* h_base, const uint64_t* h_off, uint32_t n, void* h_out, int device,
               uint32_t mode, uint32_t* h_crc, const lnl_host_opts* opts) {
    HostPlan plan;
    if (int rc = host_plan(opts, &plan)) return rc;
    if (n == 0) return 0;
    if (!h_base || !h_off || !h_out) return fail(-EINVAL, "NULL argument");
    const uint32_t filter = mode == kHostFilter;
    {
        // (branch-free, so it vectorises: this runs before the first copy is queued)
        bool bad = false;
        for (uint32_t i = 0; i < n; ++i) bad |= h_off[i + 1] < h_off[i];
        if (bad)
            for (uint32_t i = 0; i < n; ++i)
                if (h_off[i + 1] < h_off[i]) return fail(-EINVAL, "offsets decrease at %u", i);
    }
    DeviceState* S;
    if (int rc = device_state(device, &S)) return rc;
    std::lock_guard<std::mutex> lk(S->host_mu);
    int prev = 0;
    (void)hipGetDevice(&prev);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    struct Restore {
        int d;
        ~Restore() { (void)hipSetDevice(d); }
    } restore{prev};

    const int ns = plan.streams;
    // chunk boundaries: <= chunk_n datagrams and <= chunk_bytes bytes (a single
    // larger datagram gets a chunk of its own)
    // (a binary search over the non-decreasing offsets: the last j <= i +
    // chunk_n with off[j] - off[i] <= chunk_bytes)
    auto chunk_end = [&](uint32_t i) {
        const uint32_t hi = (uint32_t)std::min<uint64_t>(n, (uint64_t)i + std::max<uint32_t>(plan.chunk_n, 1u));
        const uint64_t lim = plan.chunk_bytes > UINT64_MAX - h_off[i] ? UINT64_MAX : h_off[i] + plan.chunk_bytes;
        const uint64_t* p = std::upper_bound(h_off + i + 1, h_off + hi + 1, lim);
        const uint32_t j = (uint32_t)(p - h_off) - 1u;
        return j > i ? j : i + 1u;
    };
    size_t need_bytes = 0;
    uint32_t need_n = 0;
    for (uint32_t i = 0; i < n;) {
        const uint32_t j = chunk_end(i);
        need_bytes = std::max<size_t>(need_bytes, h_off[j] - h_off[i]);
        need_n = std::max(need_n, j - i);
        i = j;
    }
    const size_t need_wire = mode == kHostAppend ? need_bytes + (size_t)need_n * LNL_CRC32C_LAYER_EXTRA : 0;
    // the small result arrays (CRCs, statuses, append's optional CRCs) go
    // through the slots' pinned staging when the caller's are pageable
    void* const small_out = mode == kHostAppend ? (void*)h_crc : h_out;
    const bool stage = small_out && !host_pinned(small_out, (size_t)n * (filter ? 1u : 4u));
    for (int k = 0; k < ns; ++k)
        if (int rc = slot_ready(S->slot[k], need_bytes, need_n, need_wire, stage)) return rc;
    // after the first enqueue, every error path drains the streams first: the
    // caller may free h_base / h_out as soon as we return
    auto drained = [&](int rc) {
        for (int s2 = 0; s2 < ns; ++s2) {
            (void)hipStreamSynchronize(S->slot[s2].stream);
            S->slot[s2].pend_bytes = 0;
        }
        return rc;
    };
    uint32_t i = 0;
    int k = 0;
    while (i < n) {
        const uint32_t j = chunk_end(i);
        const uint32_t cn = j - i;
        const size_t cb = h_off[j] - h_off[i];
        HostSlot& s = S->slot[k];
        hipStream_t st = s.stream;
        if (int rc = host_unstage(s)) return drained(rc);  // (its previous chunk: done by now, the others in flight)
        if (cb && (e = hipMemcpyAsync(s.d_bytes, h_base + h_off[i], cb, hipMemcpyHostToDevice, st)) != hipSuccess)
            return drained(hip_fail(e, "H2D bytes"));
        if ((e = hipMemcpyAsync(s.d_off, h_off + i, (size_t)(cn + 1) * 8, hipMemcpyHostToDevice, st)) != hipSuccess)
            return drained(hip_fail(e, "H2D offsets"));
        lnl::BatchArgs a{};
        a.base = s.d_bytes;
        a.off = s.d_off;
        a.off0 = h_off[i];
        a.n = cn;
        const size_t esz = filter ? 1 : 4;  // bytes of output per datagram
        if (mode == kHostAppend) {
            // the chunk's wire burst starts where its first datagram's wire
            // bytes go: (h_off[i] - h_off[0]) + 4 i
            if (int rc = append_csr(*S, a, s.d_wire, s.d_out, st)) return drained(rc);
            uint8_t* dst = (uint8_t*)h_out + (h_off[i] - h_off[0]) + (size_t)i * LNL_CRC32C_LAYER_EXTRA;
            if ((e = hipMemcpyAsync(dst, s.d_wire, cb + (size_t)cn * LNL_CRC32C_LAYER_EXTRA, hipMemcpyDeviceToHost,
                                    st)) != hipSuccess)
                return drained(hip_fail(e, "D2H wire"));
            if (h_crc) {
                void* to = stage ? (void*)s.h_stage : (void*)(h_crc + i);
                if ((e = hipMemcpyAsync(to, s.d_out, (size_t)cn * 4, hipMemcpyDeviceToHost, st)) != hipSuccess)
                    return drained(hip_fail(e, "D2H crc"));
                if (stage) {
                    s.pend_dst = h_crc + i;
                    s.pend_bytes = (size_t)cn * 4;
                }
            }
        } else {
            if (filter) {
                a.ok = (uint8_t*)s.d_out;
                a.filter = 1;
                if (int rc = launch_csr(*S, a, lnl::kModeVerify, st)) return drained(rc);
            } else {
                a.out = s.d_out;
                if (int rc = launch_csr(*S, a, lnl::kModeCsr, st)) return drained(rc);
            }
            uint8_t* const dst = (uint8_t*)h_out + (size_t)i * esz;
            if ((e = hipMemcpyAsync(stage ? (void*)s.h_stage : (void*)dst, s.d_out, (size_t)cn * esz,
                                    hipMemcpyDeviceToHost, st)) != hipSuccess)
                return drained(hip_fail(e, "D2H"));
            if (stage) {
                s.pend_dst = dst;
                s.pend_bytes = (size_t)cn * esz;
            }
        }
        i = j;
        k = (k + 1) % ns;
    }
    for (int s = 0; s < ns; ++s) {
        if ((e = hipStreamSynchronize(S->slot[s].stream)) != hipSuccess)
            return drained(hip_fail(e, "hipStreamSynchronize"));
        if (int rc = host_unstage(S->slot[s])) return drained(rc);
    }
    return 0;
}
}  // namespace

extern "C" int lnl_crc32c_batch_host(const uint8_t* h_base, const uint64_t* h_off, uint32_t n,
                                     uint32_t* h_out, int device) {
    return host_batch(h_base, h_off, n, h_out, device, kHostCrc, nullptr, nullptr);
}

extern "C" int lnl_inbound_filter_host(const uint8_t* h_base, const uint64_t* h_off, uint32_t n,
                                       uint8_t* h_status, int device) {
    return host_batch(h_base, h_off, n, h_status, device, kHostFilter, nullptr, nullptr);
}

extern "C" int lnl_crc32c_append_host(const uint8_t* h_payload, const uint64_t* h_off, uint32_t n, uint8_t* h_wire,
                                      uint32_t* h_crc, int device) {
    return host_batch(h_payload, h_off, n, h_wire, device, kHostAppend, h_crc, nullptr);
}

extern "C" int lnl_crc32c_batch_host_ex(const uint8_t* h_base, const uint64_t* h_off, uint32_t n, uint32_t* h_out,
                                        int device, const lnl_host_opts* opts) {
    return host_batch(h_base, h_off, n, h_out, device, kHostCrc, nullptr, opts);
}

extern "C" int lnl_inbound_filter_host_ex(const uint8_t* h_base, const uint64_t* h_off, uint32_t n,
                                          uint8_t* h_status, int device, const lnl_host_opts* opts) {
    return host_batch(h_base, h_off, n, h_status, device, kHostFilter, nullptr, opts);
}

extern "C" int lnl_crc32c_append_host_ex(const uint8_t* h_payload, const uint64_t* h_off, uint32_t n,
                                         uint8_t* h_wire, uint32_t* h_crc, int device, const lnl_host_opts* opts) {
    return host_batch(h_payload, h_off, n, h_wire, device, kHostAppend, h_crc, opts);
}

namespace {
// lnl_dispatch_opts -> DispatchArgs::tail (NULL: the datagram rule)
int dispatch_tail(const lnl_dispatch_opts* o, uint32_t* tail) {
    *tail = lnl::kDispatchTailDatagram;
    if (!o) return 0;
    if (o->size < sizeof(lnl_dispatch_opts)) return fail(-EINVAL, "lnl_dispatch_opts.size %u", o->size);
    if (o->reserved[0] || o->reserved[1]) return fail(-EINVAL, "lnl_dispatch_opts.reserved must be 0");
    if (o->tail > LNL_DISPATCH_TAIL_LAYER) return fail(-EINVAL, "lnl_dispatch_opts.tail %u", o->tail);
    static_assert(LNL_DISPATCH_TAIL_ZERO == lnl::kDispatchTailZero && LNL_DISPATCH_TAIL_LAYER == lnl::kDispatchTailLayer,
                  "tail modes");
    *tail = o->tail;
    return 0;
}
}  // namespace

extern "C" int lnl_dispatch_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                                    const uint8_t* d_status, uint64_t* d_pkt_start, uint32_t* d_pkt_len,
                                    uint32_t* d_pkt_parent, uint32_t cap, uint32_t* d_total, void* hip_stream) {
    return lnl_dispatch_csr_dev_ex(d_base, d_off, n, d_status, d_pkt_start, d_pkt_len, d_pkt_parent, nullptr, cap,
                                   d_total, nullptr, hip_stream);
}

extern "C" int lnl_dispatch_csr_dev_ex(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                                       const uint8_t* d_status, uint64_t* d_pkt_start, uint32_t* d_pkt_len,
                                       uint32_t* d_pkt_parent, uint32_t* d_pkt_avail, uint32_t cap,
                                       uint32_t* d_total, const lnl_dispatch_opts* opts, void* hip_stream) {
    uint32_t tail = 0;
    if (int rc = dispatch_tail(opts, &tail)) return rc;
    if (!d_total) return fail(-EINVAL, "d_total is NULL");
    hipStream_t st = (hipStream_t)hip_stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_total, 0, 4, st);
        return e == hipSuccess ? 0 : hip_fail(e, "hipMemsetAsync");
    }
    if (!d_base || !d_off || !d_status) return fail(-EINVAL, "NULL argument");
    if (cap && (!d_pkt_start || !d_pkt_len || !d_pkt_parent)) return fail(-EINVAL, "NULL output");
    DeviceState* S;
    if (int rc = current_device(&S)) return rc;
#if LNL_EXPERIMENTS
    // LNL_DISPATCH_ONEPASS=1: one launch with a decoupled look-back (experiment,
    // parity-clean but 0.61 ms against 0.18 for count + scan + emit)
    static const bool onepass = [] {
        const char* e = getenv("LNL_DISPATCH_ONEPASS");
        return e && e[0] == '1';
    }();
    static const uint32_t nt_stores = [] {
        const char* e = getenv("LNL_DISPATCH_NT");
        return e && e[0] == '1' ? 1u : 0u;
    }();
#else
    constexpr bool onepass = false;   // product: count + scan + emit
    constexpr uint32_t nt_stores = 0;  // plain stores (nt measured neutral)
#endif
    if (onepass && !tail && !d_pkt_avail) {
        const size_t nwg = ((size_t)n + 255) / 256;
        void* flags = nullptr;
        hipError_t e = hipMallocAsync(&flags, nwg * 8, st);
        if (e != hipSuccess) return fail(-ENOMEM, "hipMallocAsync(%zu): %s", nwg * 8, hipGetErrorString(e));
        lnl::DispatchArgs a{};
        a.base = d_base;
        a.off = d_off;
        a.n = n;
        a.status = d_status;
        a.look = (uint64_t*)flags;
        a.nt = nt_stores;
        a.pkt_start = d_pkt_start;
        a.pkt_len = d_pkt_len;
        a.pkt_parent = d_pkt_parent;
        a.cap = cap;
        a.total = d_total;
        int rc = 0;
        e = hipMemsetAsync(flags, 0, nwg * 8, st);
        if (e != hipSuccess) rc = hip_fail(e, "hipMemsetAsync");
        if (rc == 0 && (e = lnl::launch_dispatch(a, nullptr, 0, st)) != hipSuccess) rc = hip_fail(e, "dispatch launch");
        e = hipFreeAsync(flags, st);
        if (rc == 0 && e != hipSuccess) rc = hip_fail(e, "hipFreeAsync");
        return rc;
    }
    // batches of up to kDispatchPrefixWgs workgroups: per-workgroup totals
    // (the emit pass sums its predecessors'); larger: a hipCUB scan into first
    const uint32_t nwg = (uint32_t)(((size_t)n + 255) / 256);
    const bool prefix = nwg <= lnl::kDispatchPrefixWgs && !LNL_DISPATCH_SCAN;
    const size_t scan_bytes = prefix ? 0 : lnl::dispatch_scan_bytes(n);
    void* scratch = nullptr;
    const size_t bytes = (2 + (size_t)lnl::kDispatchRec) * n * 4 + scan_bytes + 256;
    hipError_t e = hipMallocAsync(&scratch, bytes, st);
    if (e != hipSuccess) return fail(-ENOMEM, "hipMallocAsync(%zu): %s", bytes, hipGetErrorString(e));
    lnl::DispatchArgs a{};
    a.base = d_base;
    a.off = d_off;
    a.n = n;
    a.status = d_status;
    a.counts = (uint32_t*)scratch;
    a.first = a.counts + n;  // (prefix: its first nwg words are the workgroup totals)
    a.wgsum = prefix ? a.first : nullptr;
    a.rec = a.first + n;
    a.nt = nt_stores;
    a.pkt_start = d_pkt_start;
    a.pkt_len = d_pkt_len;
    a.pkt_parent = d_pkt_parent;
    a.pkt_avail = cap ? d_pkt_avail : nullptr;
    a.tail = tail;
    a.cap = cap;
    a.total = d_total;
    void* tmp = (void*)(((uintptr_t)(a.rec + (size_t)lnl::kDispatchRec * n) + 255) & ~(uintptr_t)255);
    int rc = 0;
    e = lnl::launch_dispatch(a, tmp, scan_bytes, st);
    if (e != hipSuccess) rc = hip_fail(e, "dispatch launch");
    e = hipFreeAsync(scratch, st);
    if (rc == 0 && e != hipSuccess) rc = hip_fail(e, "hipFreeAsync");
    return rc;
}

// lnl_inbound_filter_csr_dev + lnl_dispatch_csr_dev in one pass over the
// bytes: large batches walk their MERGED containers inside the span kernel
// (crc32c_span.hip, WALK), so the dispatch step reads no datagram bytes again;
// small ones run the two calls.
extern "C" int lnl_inbound_filter_dispatch_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                                                   uint8_t* d_status, uint64_t* d_pkt_start, uint32_t* d_pkt_len,
                                                   uint32_t* d_pkt_parent, uint32_t cap, uint32_t* d_total,
                                                   void* hip_stream) {
    return lnl_inbound_filter_dispatch_csr_dev_ex(d_base, d_off, n, d_status, d_pkt_start, d_pkt_len, d_pkt_parent,
                                                  nullptr, cap, d_total, nullptr, hip_stream);
}

extern "C" int lnl_inbound_filter_dispatch_csr_dev_ex(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                                                      uint8_t* d_status, uint64_t* d_pkt_start, uint32_t* d_pkt_len,
                                                      uint32_t* d_pkt_parent, uint32_t* d_pkt_avail, uint32_t cap,
                                                      uint32_t* d_total, const lnl_dispatch_opts* opts,
                                                      void* hip_stream) {
    uint32_t tail = 0;
    if (int rc = dispatch_tail(opts, &tail)) return rc;
    if (!d_total) return fail(-EINVAL, "d_total is NULL");
    hipStream_t st = (hipStream_t)hip_stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_total, 0, 4, st);
        return e == hipSuccess ? 0 : hip_fail(e, "hipMemsetAsync");
    }
    if (!d_base || !d_off || !d_status) return fail(-EINVAL, "NULL argument");
    if (cap && (!d_pkt_start || !d_pkt_len || !d_pkt_parent)) return fail(-EINVAL, "NULL output");
    DeviceState* S;
    if (int rc = current_device(&S)) return rc;
    // (the span kernel indexes walk blocks as 8 k in 32 bits)
    if (n < LNL_BUCKET_MIN_N || n > (1u << 28) || csr_path() != kPathBucketed) {
        if (int rc = lnl_inbound_filter_csr_dev(d_base, d_off, n, d_status, hip_stream)) return rc;
        return lnl_dispatch_csr_dev_ex(d_base, d_off, n, d_status, d_pkt_start, d_pkt_len, d_pkt_parent, d_pkt_avail,
                                       cap, d_total, opts, hip_stream);
    }
    const uint32_t nwg = (uint32_t)(((size_t)n + 255) / 256);
    const bool prefix = nwg <= lnl::kDispatchPrefixWgs && !LNL_DISPATCH_SCAN;
    const size_t scan_bytes = prefix ? 0 : lnl::dispatch_scan_bytes(n);
    void* scratch = nullptr;
    const size_t bytes = (2 + (size_t)lnl::kDispatchRec + lnl::kWalkBlock) * n * 4 + scan_bytes + 512;
    hipError_t e = hipMallocAsync(&scratch, bytes, st);
    if (e != hipSuccess) return fail(-ENOMEM, "hipMallocAsync(%zu): %s", bytes, hipGetErrorString(e));
    lnl::DispatchArgs a{};
    a.base = d_base;
    a.off = d_off;
    a.n = n;
    a.status = d_status;
    a.counts = (uint32_t*)scratch;
    a.first = a.counts + n;  // (prefix: its first nwg words are the workgroup totals)
    a.wgsum = prefix ? a.first : nullptr;
    a.rec = a.first + n;
    a.pkt_start = d_pkt_start;
    a.pkt_len = d_pkt_len;
    a.pkt_parent = d_pkt_parent;
    a.pkt_avail = cap ? d_pkt_avail : nullptr;
    a.tail = tail;
    a.cap = cap;
    a.total = d_total;
    uint32_t* blk = (uint32_t*)(((uintptr_t)(a.rec + (size_t)lnl::kDispatchRec * n) + 255) & ~(uintptr_t)255);
    a.blk = blk;
    void* tmp = (void*)(((uintptr_t)(blk + (size_t)lnl::kWalkBlock * n) + 255) & ~(uintptr_t)255);
    lnl::BatchArgs b{};
    b.base = d_base;
    b.off = d_off;
    b.n = n;
    b.ok = d_status;
    b.filter = 1u;
    int rc = launch_csr_span(*S, b, st, lnl::kSpanFilter, blk, [&](const uint32_t* span_ctl) {
        a.span_ctl = span_ctl;  // [2] != 0: the span kernel walked the batch
        hipError_t le = lnl::launch_dispatch_walked(a, tmp, scan_bytes, st);
        return le == hipSuccess ? 0 : hip_fail(le, "dispatch launch");
    });
    e = hipFreeAsync(scratch, st);
    if (rc == 0 && e != hipSuccess) rc = hip_fail(e, "hipFreeAsync");
    return rc;
}

namespace {
int xor_layer(uint8_t* d_base, const uint64_t* d_off, size_t stride, uint32_t len, uint32_t n,
              const uint8_t* key, size_t key_len, void* hip_stream) {
    if (!key || key_len == 0 || key_len > lnl::kXorMaxKey)
        return fail(-EINVAL, "key_len %zu outside 1..%u", key_len, lnl::kXorMaxKey);
    if (n == 0) return 0;
    if (!d_base) return fail(-EINVAL, "d_base is NULL");
    DeviceState* S;
    if (int rc = current_device(&S)) return rc;
    lnl::XorArgs a{};
    a.base = d_base;
    a.off = d_off;
    a.stride = stride;
    a.len = len;
    a.n = n;
    a.key_len = (uint32_t)key_len;
    memcpy(a.key, key, key_len);
    // contiguous fixed stride (stride == len >= 16), 16-byte aligned: the flat
    // kernel (whole pieces per lane, coalesced).  Strides with gaps take the
    // per-datagram kernel, which never touches the gap bytes (the flat kernel
    // would rewrite them unchanged -- a lost update for a concurrent writer).
#if LNL_EXPERIMENTS
    static const int flat_v = [] {
        const char* e = getenv("LNL_XOR_FLAT");  // 0: per-datagram kernel
        return e ? atoi(e) : 12;
    }();
    static const int flat_wg = [] {
        const char* e = getenv("LNL_XOR_FLAT_WG");  // workgroups per CU
        return e ? std::max(1, atoi(e)) : 8;
    }();
#else
    constexpr int flat_v = 12;  // tiles of 2 x 256 pieces, nontemporal
    constexpr int flat_wg = 8;  // workgroups per CU (persistent forms)
#endif
    const bool flat_on = flat_v > 0;
    const uint64_t span = d_off ? 0 : (uint64_t)(n - 1) * stride + len;
    if (flat_on && !d_off && stride == len && stride >= 16 && stride < (1u << 31) && len >= 1 &&
        ((uintptr_t)d_base & 15u) == 0 && span < (1ull << 35)) {
        lnl::FlatArgs f{};
        f.span = span;
        f.pieces = (uint32_t)((span + 15) / 16);
        f.whole = (uint32_t)(span / 16);
        f.S = (uint32_t)stride;
        f.L = len;
        f.K = (uint32_t)key_len;
        f.n = n;
        f.SK = f.S % f.K;
        const uint32_t per = 256u * 4u;  // pieces per workgroup per step (kThreads x kUnroll)
        uint32_t grid = std::max(1u, std::min((f.pieces + per - 1) / per, (uint32_t)S->cus * (uint32_t)flat_wg));
        uint64_t step = 16ull * grid * 256u;
        if (flat_v > 10) {  // tiles of tu x 256 pieces, one per workgroup, the grid in batch order
            const uint32_t tu = flat_v == 11 || flat_v == 15 ? 1u : flat_v == 13 ? 4u : 2u;
            grid = std::max(1u, (f.pieces + 256u * tu - 1u) / (256u * tu));
            step = 16ull * 256u;
        }
        f.sd = (uint32_t)(step / f.S);
        f.sr = (uint32_t)(step % f.S);
        f.srk = f.sr % f.K;
        hipError_t e = lnl::launch_xor_flat(a, f, (int)grid, flat_v, (hipStream_t)hip_stream);
        return e == hipSuccess ? 0 : hip_fail(e, "xor flat launch");
    }
    // CSR batches: the grid-interleaved CSR kernel (whole pieces per lane over
    // the batch's byte range -- it has no gaps, so no byte outside a datagram
    // is written except by the two edge pieces' byte stores -- chunk c to wave
    // c mod W after a chunk-map kernel).  Experiments build: LNL_XOR_CSR_FLAT=2
    // the streaming run kernel, 1 the flat CSR kernel (round 2), 0 the
    // per-datagram kernel.
#ifndef LNL_XOR_CSR_FLAT
#define LNL_XOR_CSR_FLAT 3
#endif
    // Grid: one workgroup per 32 datagrams, between 16 and 128 per CU (~3 chunks
    // per wave on config 3; the bytes are on the device, so n sizes it).  More
    // waves than a persistent 4 per CU keep the grid inside a narrower window
    // of the batch (round 5).
#ifndef LNL_XOR_GRID_WGS
#define LNL_XOR_GRID_WGS 128u  // workgroups per CU, at most
#endif
#ifndef LNL_XOR_GRID_MIN
#define LNL_XOR_GRID_MIN 16u  // workgroups per CU, at least
#endif
#ifndef LNL_XOR_GRID_PER
#define LNL_XOR_GRID_PER 32u  // datagrams per workgroup (0: always LNL_XOR_GRID_WGS per CU)
#endif
    if (LNL_XOR_CSR_FLAT == 3 && d_off) {
        const uint32_t lo = (uint32_t)S->cus * LNL_XOR_GRID_MIN, hi = (uint32_t)S->cus * LNL_XOR_GRID_WGS;
        const uint32_t want = LNL_XOR_GRID_PER ? (n + LNL_XOR_GRID_PER - 1u) / LNL_XOR_GRID_PER : hi;
        const int grid = (int)std::min(hi, std::max(lo, want));
        return with_xor_map((hipStream_t)hip_stream, (size_t)n + 1u, [&](uint32_t* map) {
            hipError_t e = lnl::launch_xor_csr_grid(a, map, n + 1u, grid, (hipStream_t)hip_stream);
            return e == hipSuccess ? 0 : hip_fail(e, "xor csr grid launch");
        });
    }
#ifndef LNL_XOR_STREAM_WGS
#define LNL_XOR_STREAM_WGS 6  // workgroups per CU
#endif
    if (LNL_XOR_CSR_FLAT == 2 && d_off) {
        hipError_t e = lnl::launch_xor_csr_stream(a, S->cus * LNL_XOR_STREAM_WGS, (hipStream_t)hip_stream);
        return e == hipSuccess ? 0 : hip_fail(e, "xor csr stream launch");
    }
    if (LNL_XOR_CSR_FLAT == 1 && d_off) {
        hipError_t e = lnl::launch_xor_csr_flat(a, S->cus * 8, (hipStream_t)hip_stream);
        return e == hipSuccess ? 0 : hip_fail(e, "xor csr flat launch");
    }
    // lnl::kXorPerWg datagrams per workgroup (uncapped grid: measured faster than persistent)
    const uint32_t wgs = (n + lnl::kXorPerWg - 1u) / lnl::kXorPerWg;
#ifndef LNL_XOR_WG_PER_CU
#define LNL_XOR_WG_PER_CU 0  // 0: one workgroup per kXorPerWg datagrams, no cap
#endif
    const uint32_t cap = LNL_XOR_WG_PER_CU ? (uint32_t)S->cus * LNL_XOR_WG_PER_CU : 0xFFFFFFFFu;
    const int grid = (int)std::max(1u, std::min(wgs, cap));
    hipError_t e = lnl::launch_xor_layer(a, grid, (hipStream_t)hip_stream);
    return e == hipSuccess ? 0 : hip_fail(e, "xor layer launch");
}
}  // namespace

extern "C" int lnl_xor_layer_csr_dev(uint8_t* d_base, const uint64_t* d_off, uint32_t n, const uint8_t* key,
                                     size_t key_len, void* hip_stream) {
    if (n && !d_off) return fail(-EINVAL, "d_off is NULL");
    return xor_layer(d_base, d_off, 0, 0, n, key, key_len, hip_stream);
}

extern "C" int lnl_xor_layer_fixed_dev(uint8_t* d_base, size_t stride, uint32_t len, uint32_t n,
                                       const uint8_t* key, size_t key_len, void* hip_stream) {
    if (n && stride < len) return fail(-EINVAL, "stride %zu < len %u", stride, len);
    return xor_layer(d_base, nullptr, stride, len, n, key, key_len, hip_stream);
}

extern "C" int lnl_crc32c_batch_host_multi(const uint8_t* h_base, const uint64_t* h_off, uint32_t n,
                                           uint32_t* h_out, const int* devices, int ndev) {
    if (n == 0) return 0;
    if (!devices || ndev <= 0) return fail(-EINVAL, "empty device list");
    if (!h_base || !h_off || !h_out) return fail(-EINVAL, "NULL argument");
    const uint32_t per = (uint32_t)(((uint64_t)n + (uint64_t)ndev - 1) / (uint64_t)ndev);
    std::vector<int> rc(ndev, 0);
    std::vector<std::string> err(ndev);
    std::vector<std::thread> th;
    th.reserve(ndev);
    for (int r = 0; r < ndev; ++r) {
        const uint32_t start = (uint32_t)std::min<uint64_t>((uint64_t)r * per, n);
        const uint32_t cnt = std::min(per, n - start);
        if (cnt == 0) continue;
        th.emplace_back([&, r, start, cnt] {
            // the range's offsets stay absolute (h_off[start] may be nonzero)
            rc[r] = lnl_crc32c_batch_host(h_base, h_off + start, cnt, h_out + start, devices[r]);
            if (rc[r]) err[r] = g_err;  // thread_local: copy before the thread ends
        });
    }
    for (auto& t : th) t.join();
    for (int r = 0; r < ndev; ++r)
        if (rc[r]) return fail(rc[r], "range %d (device %d): %s", r, devices[r], err[r].c_str());
    return 0;
}
