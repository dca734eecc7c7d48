// crc32c_span.hip -- CSR batches as line SEGMENTS with a wave-uniform fold
// stash (config 3: 2^20 mixed-length datagrams; any CSR batch of >= 16 Ki
// datagrams).
//
// A CSR batch is one contiguous byte stream (datagram i = base[off[i],
// off[i+1])), so the shape that reads every 128-byte line exactly once with
// every lane busy is the SEGMENT: lane l of wave-batch w owns segment
// g = 64 w + l, R consecutive lines (crc32c_span.h), and reads line g R + t at
// row t.  Measured on the probe (hbm_probe.hip, forms 4 and 7), that shape
// streams at 6.8-6.9 TB/s.  What made the earlier segment kernel VALU-bound
// was the FOLD: datagram ends fall on different rows in every lane, so nearly
// every row paid a divergent 5-level fold (~720 VALU ops) for the few lanes
// that ended a datagram.  Here a lane never folds its own datagram:
//
//  * Row step.  o = A s ^ x for every lane (one generated network,
//    crc32c_bitslice.h).  A lane whose datagram ends in this row at byte b-1
//    has state o ^ F(b), where F(b) is the row from byte b on (pieces before
//    b's piece read from a zero piece, b's piece AND-masked in place in LDS);
//    the next datagram starts with state F(b) ^ C[b] (CRC init as word 0).
//    Further datagrams that start and end inside the row: F(b) ^ F(b') ^ C[b].
//    The row's network runs once whatever the boundaries are.
//  * Stash.  Ended states (32 words) go to a per-wave LDS ring (kCap entries)
//    with their datagram index and e (bytes of the row after the last one).
//    When 64 are waiting, the whole wave folds 64 of them at once -- one per
//    lane, uniform: a table Horner straight to the CRC register (crc32c_span.h,
//    ~200 VALU ops and 128 byte-table lookups), then the final map (two
//    nibble-table products) -- and stores the CRCs.  Fold cost per datagram:
//    one fold, never a divergent one.
//  * Heads and tails.  A datagram that runs in from the previous segment (the
//    head) is folded from state 0; the previous lane folds the part it saw
//    (the tail).  CRC registers are linear:
//    CRC = ~step^(-8e)(step^(1024 m) tail ^ head).  The
//    kernel leaves both per segment (crc32c_span.h record), and the batch
//    kernel's prologue (crc32c_kernels.hip) combines them before it takes the
//    datagrams touching three or more segments (the overflow list).
//
// Memory: rows come in as 16-byte pieces, glds-shaped (load i of lane l is
// piece l & 7 of the row of lane 8 i + l / 8: 8 whole lines per
// wave-instruction), into VGPRs -- two rows in flight -- and are transposed
// through an 8 KiB LDS image per wave (the probe's form 7).  That leaves LDS
// for the stash: 17 KiB of fold tables + 8 waves x (8 KiB image + 66 x 152 B
// stash and meta) = 163,328 B, one 512-thread workgroup per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"
#include "crc32c_kernels.h"
#include "crc32c_span.h"

namespace lnl {

namespace {

using namespace dev;

constexpr int kThreads = kSpanThreads;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kCap = 66;      // stash entries per wave
constexpr uint32_t kFlush = 64;    // fold when this many are waiting
constexpr uint32_t kEntry = 144;   // stash entry stride: 128 B of state + 16 B pad, so that
                                   // consecutive slots start on different banks and the 8
                                   // pieces of an entry sit at immediate offsets
constexpr uint32_t kImageBytes = 8192;
#ifndef LNL_SPAN_WIN1
#define LNL_SPAN_WIN1 12u
#endif
constexpr uint32_t kWin1 = LNL_SPAN_WIN1;  // window chunks (64 offsets each) loaded ahead of the first rows

#ifndef LNL_SPAN_PRIO
#define LNL_SPAN_PRIO 0  // 0: progress-based issue priority; 1: static (experiment); 2: none
#endif
// Round 4 (tools/kvariants.py, config-3 CSR call, one box: 153.8 -> 151.1 us,
// filter 146.6 -> 144.7 us): a wave-batch's first two rows go out behind its
// offset window rather than with its probe, so the probe and the window are not
// queued behind 16 MB of rows (0: round 3's order); a partial flush (the
// segment's end) looks up tables in the lanes that fold only (0: all lanes).
#ifndef LNL_SPAN_ROWS_LATE
#define LNL_SPAN_ROWS_LATE 1
#endif
#ifndef LNL_SPAN_FOLD_MASK
#define LNL_SPAN_FOLD_MASK 1
#endif
#ifndef LNL_SPAN_EARLY_FLUSH
#define LNL_SPAN_EARLY_FLUSH 50  // WALK kernel: fold a stash holding this many entries at a row step's start (0: off)
#endif
// The segment's end (round 4): its tail is folded in registers rather than
// through the stash (1), and the last partial flush in the same pass (2, the
// default; 0: round 3's stash path).  Config-3 call 150.3 -> 148.3 us, filter
// 147.9 -> 143.8, fused walk 337.4 -> 335.4 (tools/kvariants.py, one box);
// the end phase 6.2 -> 4.6 us in the per-wave timeline.
#ifndef LNL_SPAN_TAIL_REG
#define LNL_SPAN_TAIL_REG 2
#endif
#ifndef LNL_SPAN_F_MASK
#define LNL_SPAN_F_MASK 0  // 1: F(b) read by the lanes with a boundary only (experiment)
#endif
#ifndef LNL_SPAN_FIN_LDS
#define LNL_SPAN_FIN_LDS 0  // 1: the heads' final map from the LDS tables (TB, TA), not the global FIN table
#endif
constexpr uint32_t kTabBytes = kSpanTabLds * 4;
// LDS (bytes): the fold tables (crc32c_span.h) first -- the Horner's byte
// lookups then address them with a 16-bit immediate offset -- and a zero
// piece; the waves' row images (8 KiB each, 128-byte aligned, so piece p of a
// swizzled row is r0 ^ 16 p); the stashes and their meta words
constexpr uint32_t kTabOff = 0;
constexpr uint32_t kZeroOff = kTabOff + kTabBytes;
constexpr uint32_t kImageOff = (kZeroOff + 16u + 127u) & ~127u;
constexpr uint32_t kStashOff = kImageOff + kWaves * kImageBytes;
constexpr uint32_t kStashBytes = kCap * kEntry;
constexpr uint32_t kMetaOff = kStashOff + kWaves * kStashBytes;
constexpr uint32_t kProgOff = kMetaOff + kWaves * kCap * 8;  // rows done per wave (issue fairness)
constexpr uint32_t kLdsBytes = kProgOff + kWaves * 4;
static_assert(kLdsBytes <= 160 * 1024, "LDS");
constexpr uint32_t kWinMax = (kStashBytes / 4u) & ~63u;  // window entries the stash holds
static_assert(kWinMax >= 64u * kWin1, "window");
static_assert(kTabBytes % 16 == 0 && kStashOff % 16 == 0 && kMetaOff % 8 == 0, "LDS alignment");

enum : uint32_t { kTypeNormal = 0, kTypeHead = 1, kTypeTail = 2 };

// A datagram's result: its CRC (kSpanCrc) or its LNL_INBOUND_* status from the
// whole-datagram CRC.  (The timeline build, LNL_SPAN_DIAG & 16, stores none:
// out[] carries its stamps.)
__device__ LNL_INLINE void store_result(const SpanArgs& A, uint32_t i, uint32_t crc, uint32_t len, uint32_t hdr) {
#if defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 128)
    if (A.mode == kSpanCrc && crc == 0xFFFFFFFFu && len == 0xFFFFFFFFu) A.out[i] = hdr;  // diagnostic build only: (almost) no CRC stores
    else if (A.mode != kSpanCrc) A.ok[i] = (uint8_t)lnl_span_status(A.mode, crc, len, hdr);
#elif !(defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 16))
    if (A.mode == kSpanCrc)
        A.out[i] = crc;
    else
        A.ok[i] = (uint8_t)lnl_span_status(A.mode, crc, len, hdr);
#endif
}

__device__ LNL_INLINE SpanGeo geometry_of(const SpanArgs& a) {
    const uint64_t b = (uint64_t)(uintptr_t)a.base - a.off0;
    return span_geometry(b + a.off[0], b + a.off[a.n], a.waves);
}


// ---- helpers ------------------------------------------------------------------

__device__ LNL_INLINE void append(uint32_t* cnt, uint32_t* list, bool take, uint32_t value) {
    const uint64_t m = __ballot(take);
    if (m == 0ull) return;
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(cnt, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, (int)leader, 64);
    // rank among the taking lanes (mbcnt: no 64-bit lane mask held in registers)
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (take) list[base + rank] = value;
}

__device__ LNL_INLINE uint32_t clamp16(int64_t v) { return v <= 0 ? 0u : (v >= 0xFFFF ? 0xFFFFu : (uint32_t)v); }

// ---- the span kernel ---------------------------------------------------------

// The lane's upcoming datagram boundaries (byte offsets from its segment's
// first byte, clamped to 0xFFFF), two 16-bit entries per register, the front
// in q[0]'s low half.
struct Queue {
    uint32_t q[8];
    __device__ LNL_INLINE uint32_t front() const { return q[0] & 0xFFFFu; }
    __device__ LNL_INLINE void pop() {
#pragma unroll
        for (int j = 0; j < 7; ++j) q[j] = __builtin_amdgcn_alignbit(q[j + 1], q[j], 16);
        q[7] = (q[7] >> 16) | 0xFFFF0000u;
    }
};

__device__ constexpr uint32_t kZero32[32] = {0u};

// byte b & 15 of a 16-byte piece held in registers
__device__ LNL_INLINE uint32_t piece_byte(const u32x4& v, uint32_t b) {
    const uint32_t w = (b >> 2) & 3u;
    const uint32_t x = w == 0u ? v.x : (w == 1u ? v.y : (w == 2u ? v.z : v.w));
    return (x >> (8u * (b & 3u))) & 0xFFu;
}

// one LDS byte (asm, with its wait: see read_row)
__device__ LNL_INLINE uint32_t lds_read_u8(uint32_t addr) {
    uint32_t v;
    asm volatile("ds_read_u8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

// ~step^(-8e)(r): the final map (two nibble-table products, LDS)
__device__ LNL_INLINE uint32_t final_crc_lds(uint32_t tab_base, uint32_t e, uint32_t r) {
    r = fold_apply_lds(tab_base + 4u * kSpanTabB + 512u * (e & 15u), r);
    r = fold_apply_lds(tab_base + 4u * kSpanTabA + 512u * (e >> 4), r);
    return ~r;
}

// The register value of a 32-word state: lnl_span_phi (crc32c_span.h) with
// the byte tables in LDS -- four independent Horner chains, joined by step^256
__device__ LNL_INLINE uint32_t phi_lds(const uint32_t* T, uint32_t tab_base, const uint32_t* v) {
    uint32_t r0 = 0u, r1 = 0u, r2 = 0u, r3 = 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        r0 = lnl_span_t4(T, r0 ^ v[k]);
        r1 = lnl_span_t4(T, r1 ^ v[8 + k]);
        r2 = lnl_span_t4(T, r2 ^ v[16 + k]);
        r3 = lnl_span_t4(T, r3 ^ v[24 + k]);
    }
    const uint32_t s = tab_base + 4u * kSpanTabS;
    r1 ^= fold_apply_lds(s, r0);
    r2 ^= fold_apply_lds(s, r1);
    return r3 ^ fold_apply_lds(s, r2);
}

// 16 bytes of a row from global memory, nt, in inline asm: the compiler does
// not see these loads, so it inserts no waits for them; row_step waits with a
// counted vmcnt(8) (a row step issues the 8 loads of row t + 2; at row t the
// other buffer's 8 loads of row t + 1 are the younger ones).  Left to the compiler, its vmcnt for one buffer
// counted the other buffer's loads as older and drained both every step.
__device__ LNL_INLINE void row_load(u32x4& v, uint64_t addr) {
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(addr) : "memory");
}

// 8 bytes (one offset) from global memory, in inline asm like row_load: the
// setup's window loads are issued before the first rows' and waited for with a
// counted vmcnt, so that the rows stay in flight meanwhile
__device__ LNL_INLINE void off_load(uint64_t& v, uint64_t addr) {
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(addr) : "memory");
}

// 16 bytes to LDS at addr + OFF (immediate offset)
template <uint32_t OFF>
__device__ LNL_INLINE void ds_write16(uint32_t addr, u32x4 v) {
    asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(OFF) : "memory");
}

// 8 x 16 bytes from LDS at base + 16 p (immediate offsets) + lgkmcnt(0)
__device__ LNL_INLINE void ds_read8(uint32_t base, uint32_t* x) {
    uint4 v0, v1, v2, v3, v4, v5, v6, v7;
    asm volatile(
        "ds_read_b128 %0, %8\n\t"
        "ds_read_b128 %1, %8 offset:16\n\t"
        "ds_read_b128 %2, %8 offset:32\n\t"
        "ds_read_b128 %3, %8 offset:48\n\t"
        "ds_read_b128 %4, %8 offset:64\n\t"
        "ds_read_b128 %5, %8 offset:80\n\t"
        "ds_read_b128 %6, %8 offset:96\n\t"
        "ds_read_b128 %7, %8 offset:112\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(v4), "=&v"(v5), "=&v"(v6), "=&v"(v7)
        : "v"(base)
        : "memory");
    const uint4 v[8] = {v0, v1, v2, v3, v4, v5, v6, v7};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        x[4 * k + 0] = v[k].x;
        x[4 * k + 1] = v[k].y;
        x[4 * k + 2] = v[k].z;
        x[4 * k + 3] = v[k].w;
    }
}

// read_row (crc32c_device.h) plus a ninth piece at pa, same round trip
__device__ LNL_INLINE void read_row_pre(const uint32_t* ad, uint32_t pa, uint32_t* x, u32x4& pre) {
    uint4 v0, v1, v2, v3, v4, v5, v6, v7;
    u32x4 v8;
    asm volatile(
        "ds_read_b128 %0, %9\n\t"
        "ds_read_b128 %1, %10\n\t"
        "ds_read_b128 %2, %11\n\t"
        "ds_read_b128 %3, %12\n\t"
        "ds_read_b128 %4, %13\n\t"
        "ds_read_b128 %5, %14\n\t"
        "ds_read_b128 %6, %15\n\t"
        "ds_read_b128 %7, %16\n\t"
        "ds_read_b128 %8, %17\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(v4), "=&v"(v5), "=&v"(v6), "=&v"(v7), "=&v"(v8)
        : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7]), "v"(pa)
        : "memory");
    const uint4 v[8] = {v0, v1, v2, v3, v4, v5, v6, v7};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        x[4 * k + 0] = v[k].x;
        x[4 * k + 1] = v[k].y;
        x[4 * k + 2] = v[k].z;
        x[4 * k + 3] = v[k].w;
    }
    pre = v8;
}

template <int P>
struct Pieces {  // the 8 pieces of a 32-word state written at base + 16 p
    __device__ static LNL_INLINE void write(uint32_t base, const uint32_t* x, const uint32_t* y) {
        u32x4 w;
        w.x = x[4 * P + 0] ^ y[4 * P + 0];
        w.y = x[4 * P + 1] ^ y[4 * P + 1];
        w.z = x[4 * P + 2] ^ y[4 * P + 2];
        w.w = x[4 * P + 3] ^ y[4 * P + 3];
        ds_write16<16 * P>(base, w);
        Pieces<P + 1>::write(base, x, y);
    }
};
template <>
struct Pieces<8> {
    __device__ static LNL_INLINE void write(uint32_t, const uint32_t*, const uint32_t*) {}
};

template <int I>
struct Transpose {  // load i of the row to the image: even i at we + 1024 i, odd at wo + 1024 i
    __device__ static LNL_INLINE void write(uint32_t we, uint32_t wo, const u32x4* cur) {
        ds_write16<1024 * I>((I & 1) ? wo : we, cur[I]);
        Transpose<I + 1>::write(we, wo, cur);
    }
};
template <>
struct Transpose<8> {
    __device__ static LNL_INLINE void write(uint32_t, uint32_t, const u32x4*) {}
};

// bytes q[0..2] (LE) from the aligned pair of dwords holding them (global memory;
// see lnl_dispatch.hip load3 for why both dwords are inside the batch)
__device__ LNL_INLINE uint32_t global_load3(uint64_t q) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(q & ~(uint64_t)3);
    const uint64_t v = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    return (uint32_t)(v >> ((q & 3u) * 8u));
}

constexpr uint32_t kMergedProperty = 12;  // PACKET_PROPERTY::MERGED, net_enums.h:60

// lnl_packet_verify_hdr (lnl_packet.h) for a packet of size < 2^16 whose first
// byte is b0 & 0xFF, in 32-bit arithmetic
__device__ LNL_INLINE bool verify_hdr16(uint32_t b0, uint32_t size) {
    const uint32_t p = b0 & 0x1Fu;
    const uint32_t hs = lnl_packet_header_size(p < LNL_PACKET_PROPERTY_COUNT ? p : 0u);
    const uint32_t need = (b0 & 0x80u) ? hs + LNL_FRAGMENT_HEADER_SIZE : hs;
    return p < LNL_PACKET_PROPERTY_COUNT && size >= need;
}
// walk flags (WALK): the open datagram started in this lane's segment (the
// lane writes its packet count), is a MERGED container, is still being walked
enum : uint32_t { kWalkOwned = 1, kWalkMerged = 2, kWalkOn = 4 };

// WALK (filter + dispatch): besides the statuses, every datagram whose first
// byte streams through a lane is cut as net_peer::process_packet's MERGED case
// does (/root/reference/src/lnl/net_peer.cpp:164-187; restated in
// lnl_dispatch.hip walk()) while its bytes sit in the lane's LDS row, so the
// dispatch pass does not fetch the size fields again.  Entries whose three
// bytes (u16 size, header byte) are all in the row are taken at the row; one
// that straddles the row end keeps the row's last two bytes for the next row;
// a container still open at the segment's end is finished from global memory.
template <bool WALK>
__global__ __launch_bounds__(kThreads, 1) void crc32c_span_kernel(SpanArgs A) {
    __shared__ __attribute__((aligned(128))) uint8_t lds[kLdsBytes];
    const uint32_t lane = __lane_id();
    const uint32_t wave = uni(threadIdx.x >> 6);
    const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
    const uint32_t tab_base = lds0 + kTabOff;
    const uint32_t* const T = reinterpret_cast<const uint32_t*>(lds + kTabOff) + kSpanTabT;
    const uint32_t zero_addr = lds0 + kZeroOff;
    const uint32_t image = lds0 + kImageOff + wave * kImageBytes;
    const uint32_t stash = lds0 + kStashOff + wave * kStashBytes;
    const uint32_t meta = lds0 + kMetaOff + wave * (kCap * 8u);
    const uint32_t* const ctab = reinterpret_cast<const uint32_t*>(lds + kTabOff) + kSpanTabC;  // C[pad]
    uint32_t* const prog = reinterpret_cast<uint32_t*>(lds + kProgOff);
    uint32_t rows_done = 0;  // rows this wave has streamed (all its wave-batches)

#if defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 16)
    // diagnostic build only: per-wave timeline (s_memrealtime, 100 MHz) into
    // out[8 w ..] instead of CRCs
    uint32_t tl[8];
    tl[0] = (uint32_t)wall_clock64();
#define LNL_TL(i) tl[i] = (uint32_t)wall_clock64()
#else
#define LNL_TL(i) (void)0
#endif
    const uint64_t bsh = (uint64_t)(uintptr_t)A.base - A.off0;
    const SpanGeo G = geometry_of(A);
    const bool runs = span_runs(G, A.waves);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // for the batch kernel and the dispatch fix-up
        A.ctl[2] = runs ? G.NS : 0u;             // 0: the whole batch is the batch kernel's
        A.ctl[3] = G.R;
        // the next call's overflow count (the previous call on this stream,
        // which used that block, has finished: stream order)
        A.ctl_next[1] = 0u;
    }
    if (!runs) return;
    const uint32_t R = G.R, Sb = R << 7, NS = G.NS, nwb = G.nwb;
    if (blockIdx.x * kWaves >= nwb) return;  // whole workgroup idle (before the barrier)
    const uint32_t gw = blockIdx.x * kWaves + wave;
    const uint32_t nw = gridDim.x * kWaves;
    const uint32_t n = A.n;
    // per-lane addressing: load i brings piece pc of the row of lane 8 i + sub;
    // it lands in the image at that lane's row, slot pc ^ swz(8 i + sub)
    // (= pc ^ (sub >> 1) for even i, ^ 4 more for odd i)
    const uint32_t sub = lane >> 3, pc = lane & 7u;
    const uint32_t voff = sub * Sb + 16u * pc;
    const uint32_t we = image + sub * 128u + 16u * (pc ^ (sub >> 1));
    const uint32_t wo = we ^ 64u;
    const uint32_t r0 = image + lane * 128u + 16u * swz(lane);  // piece p of this lane's row: r0 ^ 16 p
    const uint64_t last_line = (G.S0 + G.Pn - 1u) & ~(uint64_t)127;

    // the current wave-batch: its first line, and whether its last rows are
    // clamped to the stream's last line (the last wave-batches)
    uint64_t line0 = 0;
    bool clamp = false;
    uint32_t last_rel = 0;
    auto set_wb = [&](uint32_t wb) {
        line0 = G.S0 + (uint64_t)wb * 64u * Sb;
        clamp = line0 + 64ull * Sb - 128u > last_line;
        last_rel = (uint32_t)(last_line - line0 < 0xFFFFFFFFull ? last_line - line0 : 0xFFFFFFFFull);
    };
    // row t of the wave-batch: load i of this lane is piece pc of line
    // line0 + (8 i + sub) Sb + 128 t (clamped to the stream's last line)
    auto issue = [&](uint32_t t, u32x4* v) {
        if (!clamp) {
            const uint64_t rbase = line0 + ((uint64_t)t << 7);
            uint32_t vo = voff;
            asm volatile("" : "+v"(vo));  // 8 per-load addresses per row, not hoisted into 16 registers
#pragma unroll
            for (int i = 0; i < 8; ++i) row_load(v[i], rbase + (uint64_t)(i * 8u * Sb) + vo);
        } else {
            uint32_t lo = (sub * Sb) + (t << 7);
            asm volatile("" : "+v"(lo));
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t rel = lo + (uint32_t)i * 8u * Sb;
                rel = rel > last_rel ? last_rel : rel;
                row_load(v[i], line0 + rel + 16u * pc);
            }
        }
    };
    // The setup's probe: 64 offsets 64 apart around the datagram whose start the
    // wave-batch's first byte falls on, interpolated from its byte position
    uint32_t pidx = 0;
    uint64_t pv = 0;
    auto probe = [&]() {
        // (fp32: only the probe's centre; a miss costs a 64-ary search, and the
        // error, ~1e-7 n, is far inside the probe's +-2,048 entries)
        const float f = (float)(line0 - G.S0) / (float)G.Pn;
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));  // (not a 64-bit per-lane constant held across the loop)
        const int64_t pi = (int64_t)(f * (float)n) + (int64_t)((int32_t)(ln * 64u) - 32 * 64);
        pidx = pi < 0 ? 0u : (pi > (int64_t)n ? n : (uint32_t)pi);
        off_load(pv, (uint64_t)(uintptr_t)(A.off + pidx));
    };
    u32x4 ra[8], rb[8];
    // The first wave-batch's probe and first two rows go out together with the
    // fold tables' loads -- all inline asm, so the compiler waits for none of
    // them -- and one counted vmcnt then waits for the probe and the tables
    // only: the rows stream while the tables go to LDS and the probe is read.
    {
        const bool has0 = gw < nwb;
        if (has0) {
            set_wb(gw);
            probe();
        }
        constexpr uint32_t kTabPieces = kTabBytes / 16u;
        constexpr uint32_t kTabLoads = (kTabPieces + kThreads - 1u) / kThreads;
        u32x4 tv[kTabLoads];
#pragma unroll
        for (uint32_t j = 0; j < kTabLoads; ++j) {
            const uint32_t i = threadIdx.x + j * kThreads;
            row_load(tv[j], (uint64_t)(uintptr_t)A.tab + 16u * (i < kTabPieces ? i : 0u));
        }
        if (has0 && !LNL_SPAN_ROWS_LATE) {
            issue(0u, ra);
            issue(1u, rb);  // R >= 16
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (uint32_t j = 0; j < kTabLoads; ++j) {
            const uint32_t i = threadIdx.x + j * kThreads;
            if (i < kTabPieces) lds_write_piece(lds0 + kTabOff + 16u * i, tv[j]);
        }
        if (threadIdx.x == 0) lds_write_piece(lds0 + kZeroOff, (u32x4){0u, 0u, 0u, 0u});
        if (threadIdx.x < (uint32_t)kWaves) prog[threadIdx.x] = 0u;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // the wave's stash holds nothing until its first row: the setup's window
    // of offsets goes there (int32, from the wave-batch's first byte)
    int32_t* const win = reinterpret_cast<int32_t*>(lds + kStashOff + wave * kStashBytes);
    LNL_TL(1);
#if LNL_SPAN_PRIO == 1
    if (wave >= 4u) __builtin_amdgcn_s_setprio(1);  // experiment: static priority for the younger waves
#endif

    for (uint32_t wb = gw; wb < nwb; wb += nw) {
        if (wb != gw) {  // a later wave-batch (batches larger than one round): the same start
            set_wb(wb);
            probe();
#if LNL_SPAN_ROWS_LATE
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
            issue(0u, ra);
            issue(1u, rb);
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
#endif
        }
        // ---- this lane's datagrams ----------------------------------------
        // [k0, k1): the datagrams ending in this segment; k0 = #{m >= 1 :
        // pos(off[m]) <= segbase}.  Found without a pre-pass: (1) a = the same
        // for the wave-batch's first byte, to within 64, from one interpolated
        // probe of 64 offsets, loaded with the first two rows (a 64-ary search
        // when the probe misses); (2) the window off[a ..] into LDS; (3)
        // each lane's k0, its datagram's start and the next 16 ends from the
        // window.  A window that does not reach the wave-batch's end (dense
        // batches: > ~2,300 datagrams per wave-batch) leaves those lanes to
        // global-memory searches.
        const uint32_t g = wb * 64u + lane;
        const bool live = g < NS;
        const uint64_t segbase = line0 + (uint64_t)lane * Sb;
        auto rel = [&](uint64_t o) -> int64_t { return (int64_t)(bsh + o - line0); };  // pos(o) - line0
        uint32_t a;
        {
            asm volatile("" : "+v"(pv));  // (arrived: the counted wait above)
            const uint32_t idx = pidx;
            const uint64_t m = __ballot(rel(pv) <= 0);
            const uint32_t idx0 = (uint32_t)__shfl((int)idx, 0, 64), idx63 = (uint32_t)__shfl((int)idx, 63, 64);
            if (m == 0ull && idx0 == 0u) {
                a = 0u;
            } else if (m != 0ull && !(m >> 63)) {  // the probe brackets it (m is a prefix of lanes)
                a = (uint32_t)__shfl((int)idx, 63 - __builtin_clzll(m), 64);
            } else {  // 64-ary search: rel(off[lo]) <= 0 (or lo = 0), rel(off[hi]) > 0
                uint32_t lo = m == 0ull ? 0u : idx63, hi = m == 0ull ? idx0 : n;
                while (hi - lo > 1u) {
                    const uint32_t step = (hi - lo + 63u) >> 6;
                    const uint32_t j = lo + lane * step;
                    const uint64_t mm = __ballot(j < hi && rel(A.off[j]) <= 0);
                    if (mm == 0ull) break;  // (lo = 0 and nothing <= line0)
                    lo += (63u - (uint32_t)__builtin_clzll(mm)) * step;
                    hi = lo + step < hi ? lo + step : hi;
                }
                a = lo;
            }
            a = uni(a);
        }
        auto win_value = [&](uint32_t m, uint64_t o) -> int32_t {  // window entry for off[m] = o
            if (m > n) return 0x7FFFFFFF;
            const int64_t r = rel(o);
            return r > 0x7FFFFFFF ? 0x7FFFFFFF : (r < -0x7FFFFFFF ? -0x7FFFFFFF : (int32_t)r);
        };
        uint32_t wn;  // window entries
        {
            uint64_t wv[kWin1];
#pragma unroll
            for (int c = 0; c < (int)kWin1; ++c) {
                const uint32_t mm = a + 64u * c + lane;
                off_load(wv[c], (uint64_t)(uintptr_t)(A.off + (mm < n ? mm : n)));
            }
#if LNL_SPAN_ROWS_LATE
            // the first two rows go out behind the window: one counted wait
            // for the window, the rows stream on
            issue(0u, ra);
            issue(1u, rb);
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
#else
            // the window (behind the first rows, which land first)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
#pragma unroll
            for (int c = 0; c < (int)kWin1; ++c) {
                asm volatile("" : "+v"(wv[c]));
                win[64u * c + lane] = win_value(a + 64u * c + lane, wv[c]);
            }
        }
        wn = 64u * kWin1;
        const int32_t tend = (int32_t)(64u * Sb);  // the wave-batch's end, from line0
        // more of the window, while it does not reach past the wave-batch's
        // end (these loads wait for the rows too)
        while (wn < kWinMax && __shfl(win[wn - 1u], 0, 64) <= tend) {
            const uint32_t mm = a + wn + lane;
            win[wn + lane] = win_value(mm, A.off[mm < n ? mm : n]);
            wn += 64u;
        }
        __builtin_amdgcn_wave_barrier();
        const int32_t wlast = win[wn - 1u];
        uint32_t wtop = 1u;  // binary-search span: the smallest power of two >= wn
        while (wtop < wn) wtop <<= 1;
        // #{m >= 1 : pos(off[m]) <= line0 + t}: the window when it reaches past
        // t, else a binary search of the offsets
        auto count_le = [&](int32_t t) -> uint32_t {
            if (wlast > t) {
                uint32_t j = 0;
                for (uint32_t step = wtop >> 1; step; step >>= 1)
                    if (j + step < wn && win[j + step] <= t) j += step;
                return a + j;
            }
            uint32_t lo = a, hi = n + 1u;
            while (hi - lo > 1u) {
                const uint32_t mid = (lo + hi) >> 1;
                if (rel(A.off[mid]) <= (int64_t)t) lo = mid; else hi = mid;
            }
            return lo;
        };
        const int32_t tl0 = (int32_t)(lane * Sb);
        const uint32_t k0 = live ? count_le(tl0) : n;
        uint32_t k1 = (uint32_t)__shfl_down((int)k0, 1, 64);
        if (lane == 63u) k1 = live ? count_le(tend) : n;
        if (g == 0u)  // datagrams ending at the stream's first byte: all empty
            for (uint32_t i = 0; i < k0; ++i) {
                store_result(A, i, 0u, 0u, 0u);  // CRC 0; too short for the layer
            }
        Queue Q;
        uint32_t k = k0, kq, qn;
        int32_t cs;  // first byte of datagram k, from the segment's first byte
        uint32_t inj = 0u;
        // verify modes: header byte of datagram k (when it started here); taken
        // from the next row's byte 0 when it starts on a row boundary
        uint32_t chdr = 0u;
        bool hdr_next = false;
        {
            // the datagram's start and the next 16 ends: from the window, or
            // (past it) from global memory, loaded together (indices clamped,
            // values selected; the empty asm keeps the compiler from sinking
            // each load into its own branch, which would wait for them one by one)
            int64_t ov[17];
            if (k0 - a + 17u <= wn) {
#pragma unroll
                for (int j = 0; j < 17; ++j) ov[j] = (int64_t)win[k0 - a + (uint32_t)j] - (int64_t)tl0;
            } else {
                uint64_t ow[17];
#pragma unroll
                for (int j = 0; j < 17; ++j) {
                    const uint32_t kk = k0 + (uint32_t)j;
                    ow[j] = A.off[kk < n ? kk : n];
                }
#pragma unroll
                for (int j = 0; j < 17; ++j) {
                    asm volatile("" : "+v"(ow[j]));
                    ov[j] = (int64_t)(bsh + ow[j]) - (int64_t)segbase;
                }
            }
            const int64_t d0 = k0 < n ? ov[0] : 0;
            cs = d0 < -(int64_t)(2u * Sb + 2u) ? -(int32_t)(2u * Sb + 2u) : (int32_t)d0;
            // the overflow list (datagrams touching three or more segments,
            // span_overflow): each has exactly one segment that no datagram
            // ends in and that it entered from the previous segment
            append(&A.ctl[1], A.ovf, live && k0 == k1 && k0 < n && d0 < 0 && d0 >= -(int64_t)Sb, k0);
            uint32_t qp[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t lo = clamp16(ov[2 * j + 1]);
                const uint32_t hi = clamp16(ov[2 * j + 2]);
                const uint32_t vlo = k0 + 2u * j < n ? lo : 0xFFFFu, vhi = k0 + 2u * j + 1u < n ? hi : 0xFFFFu;
                qp[j] = vlo | (vhi << 16);
            }
            // segment 0: the bytes before the batch's first datagram end a
            // virtual, untracked datagram k0 - 1 at boundary cs (queue shifted
            // by one entry)
            const bool virt = k0 < n && cs > 0;
            Q.q[0] = virt ? ((uint32_t)cs | (qp[0] << 16)) : qp[0];
#pragma unroll
            for (int j = 1; j < 8; ++j) Q.q[j] = virt ? __builtin_amdgcn_alignbit(qp[j], qp[j - 1], 16) : qp[j];
            kq = virt ? k0 + 15u : k0 + 16u;
            qn = 16u;
            if (virt) {
                k = k0 - 1u;
                cs = -(int32_t)(2u * Sb + 2u);
            } else if (k0 < n && cs == 0) {
                inj = 0xFFFFFFFFu;  // C[0]: datagram k0 starts at row 0, byte 0
                hdr_next = true;
            }
        }
        // k0 < n: the lane has a datagram open (k0 - 1 when virtual)
        const bool open0 = k0 < n;
        auto is_open = [&]() { return open0 && (k < n || k == k0 - 1u); };
        auto refill = [&]() {
            // lanes whose queue is empty while a datagram is still open: the
            // next 16 boundaries (rare: > 16 datagrams in one segment)
            const bool need = qn == 0u && is_open() && k <= k1;
            if (__any(need)) {
                if (need) {
                    uint64_t ov[16];
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const uint32_t kk = kq + (uint32_t)j + 1u;
                        ov[j] = A.off[kk < n ? kk : n];
                    }
#pragma unroll
                    for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(ov[j]));
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint32_t ka = kq + 2u * j, kb = ka + 1u;
                        const uint32_t lo = clamp16((int64_t)(bsh + ov[2 * j]) - (int64_t)segbase);
                        const uint32_t hi = clamp16((int64_t)(bsh + ov[2 * j + 1]) - (int64_t)segbase);
                        Q.q[j] = (ka < n ? lo : 0xFFFFu) | ((kb < n ? hi : 0xFFFFu) << 16);
                    }
                    kq += 16u;
                    qn = 16u;
                }
            }
        };


        // ---- MERGED walk (WALK only) ---------------------------------------
        // Two registers (the kernel is at the VGPR budget):
        //   wla = wp | wc << 18: wp, the next entry's u16 size field, bytes from
        //        the segment's first byte (< Sb + 2^16 + 2 < 2^18); wc, entries
        //        taken (< Sb / 3 < 2^14)
        //   wlb = wsv | wfl << 16: wsv, bytes 126, 127 of the previous row; wfl,
        //        the walk flags
        uint32_t wla = 0u, wlb = 0u, wsv_next = 0u;
        // bytes q, q + 1, q + 2 (q >= the row's first byte - 2) of row t
        auto walk_read3 = [&](uint32_t t, int32_t q) -> uint32_t {
            const int32_t j = q - (int32_t)(t << 7);
            uint32_t ad[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const uint32_t u = j + i < 0 ? 0u : (uint32_t)(j + i);
                ad[i] = (r0 ^ (16u * (u >> 4))) + (u & 15u);
            }
            uint32_t v0, v1, v2;
            asm volatile(
                "ds_read_u8 %0, %3\n\t"
                "ds_read_u8 %1, %4\n\t"
                "ds_read_u8 %2, %5\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(v0), "=&v"(v1), "=&v"(v2)
                : "v"(ad[0]), "v"(ad[1]), "v"(ad[2])
                : "memory");
            if (j < 0) v0 = (wlb >> (8 * (j + 2))) & 0xFFu;
            if (j < -1) v1 = (wlb >> 8) & 0xFFu;
            return v0 | (v1 << 8) | (v2 << 16);
        };
        // The datagram's block [count, records 0 .. 6] (crc32c_kernels.h): words
        // 0 .. 3 gather in the lane's 16-byte pad of stash slot `lane` (free:
        // entries use 128 of their 144 bytes) and go out as one 16-byte store
        // with the count; records 3 .. 6 are stored directly (a block per
        // datagram: one sector, where 4-byte stores of the slot-major layout
        // each cost a partly written sector -- 12x the record bytes, measured)
        const uint32_t wpad = stash + lane * kEntry + 128u;
        auto walk_record = [&](uint32_t j, uint32_t r) {
            if (j < 3u)
                asm volatile("ds_write_b32 %0, %1 offset:4" ::"v"(wpad + 4u * j), "v"(r) : "memory");
            else if (j < kWalkBlock - 1u)
                A.wblk[k * kWalkBlock + 1u + j] = r;
        };
        auto walk_block = [&](uint32_t count) {
            asm volatile("ds_write_b32 %0, %1" ::"v"(wpad), "v"(count) : "memory");
            const u32x4 v = lds_read_piece(wpad);
            *reinterpret_cast<uint4*>(A.wblk + k * kWalkBlock) = make_uint4(v.x, v.y, v.z, v.w);
        };
        // take the entries of the owned container (sel) whose three bytes lie
        // before lim; size_end: the container's end without the CRC field
        // (the walk rules of lnl_dispatch.hip walk(), segment-relative)
        auto walk_fields = [&](uint32_t t, bool sel, int32_t size_end, int32_t lim) {
            // a lane has work while walking and its next entry either ends the
            // walk (past the container) or has its three bytes before lim
            auto due = [&]() {
                const int32_t wp = (int32_t)(wla & 0x3FFFFu);
                return sel && (wlb & (kWalkOn << 16)) && (wp + 2 > size_end || wp + 3 <= lim);
            };
            bool act = due();
            while (__any(act)) {
                if (act) {  // one entry, branch-free: the read is harmless when the walk stops here
                    const int32_t wp = (int32_t)(wla & 0x3FFFFu);
                    const uint32_t wc = wla >> 18;
                    const bool in = wp + 2 <= size_end;
                    const uint32_t v = walk_read3(t, in ? wp : (int32_t)(t << 7));
                    const int32_t L = (int32_t)(v & 0xFFFFu), p2 = wp + 2;
                    const bool ok = in && L != 0 && L <= size_end - p2 && verify_hdr16(v >> 16, (uint32_t)L);
                    // record slot wc (slot kDispatchRec is a spare the emit pass never
                    // reads; a slot written as the walk stops is past its count)
                    walk_record(wc, ((uint32_t)(p2 - cs) << 16) | (uint32_t)L);
                    wla = ok ? ((uint32_t)(p2 + L) | ((wc + 1u) << 18)) : wla;
                    wlb = ok ? wlb : (wlb & ~(kWalkOn << 16));
                }
                act = due();
            }
        };
        // datagram k (owned) starts at cs with header byte chdr (k = n: the
        // batch's last datagram has just ended, nothing opens)
        auto walk_open = [&]() {
            wlb = k >= n ? 0u : (kWalkOwned | ((chdr & 0x1Fu) == kMergedProperty ? (kWalkMerged | kWalkOn) : 0u)) << 16;
            wla = (uint32_t)(cs + 1);
        };
        // datagram k ends, len bytes: its packet count (a plain one is one
        // packet, the whole datagram without the CRC field)
        auto walk_close = [&](uint32_t len) {
            if (wlb & (kWalkOwned << 16))  // (a plain datagram's record is the fix-up's: its length)
                walk_block((wlb & (kWalkMerged << 16)) ? wla >> 18 : kWalkPlain);
            wlb = 0u;
        };
        // after row t's boundaries: the open container's entries in row t (an
        // entry that straddles into row t + 1 reads the row's last two bytes
        // from wsv in the next row)
        auto row_walk = [&](uint32_t t) {
#if defined(LNL_WALK_DIAG) && (LNL_WALK_DIAG & 1)
            return;  // diagnostic build only (wrong packets)
#endif
            const int32_t rowend = (int32_t)(t << 7) + 128;
            // (a boundary clamped to 0xFFFF lies beyond the segment: no bound yet)
            const uint32_t qf = Q.front();
            walk_fields(t, true, qf == 0xFFFFu ? 0x7FFFFFFF : (int32_t)qf - 4, rowend);
        };

        // ---- stash (wave-uniform counters) ---------------------------------
        uint32_t st_head = 0, st_tail = 0, head_slot = 0, tail_slot = 0;
        uint32_t hpos = 0, tpos = 0, r_head = 0, r_tail = 0, hk = 0, hinfo = 0, tcs = 0, thdr = 0;
        bool hpend = false, tpend = false, htrack = false;

        // Fold the nf oldest entries, one per lane.  The caller's live state
        // (32 words) waits in the stash meanwhile -- lane l < nf in the slot
        // it has just read, the others in free slots (cnt + 64 - nf <= kCap)
        // -- so the fold's registers do not come on top of it.
        auto flush = [&](uint32_t nf, uint32_t* live_state) {
            const bool act = lane < nf;
            uint32_t slot = act ? head_slot + lane : tail_slot + (lane - nf);
            slot = slot >= kCap ? slot - kCap : slot;
            const uint32_t ea = stash + slot * kEntry;
            uint32_t v[32];
            ds_read8(ea, v);
            uint2 mt;
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(mt) : "v"(meta + slot * 8u) : "memory");
            Pieces<0>::write(ea, live_state, kZero32);
#if defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 1)
            const uint32_t r = v[0] ^ v[31];  // diagnostic build only: no fold (wrong CRCs)
#elif LNL_SPAN_FOLD_MASK
            // only the lanes that fold look up tables: a partial flush (the
            // segment's end) costs LDS in proportion to its entries
            uint32_t r = 0u;
            if (act) r = phi_lds(T, tab_base, v);
#else
            const uint32_t r = phi_lds(T, tab_base, v);
#endif
            const uint32_t type = (mt.y >> 8) & 3u, e = mt.y & 127u;  // mt.y: e | type << 8 | hdr << 10 | len << 18
#if LNL_SPAN_FOLD_MASK
            uint32_t crc = 0u;
            if (act) crc = final_crc_lds(tab_base, e, r);
#else
            const uint32_t crc = final_crc_lds(tab_base, e, r);
#endif
            if (act && type == kTypeNormal && mt.x < n) {  // (the index check only guards the store)
                store_result(A, mt.x, crc, mt.y >> 18, (mt.y >> 10) & 0xFFu);
            }
            // head / tail folds back to the lanes that own them
            const uint32_t hs = hpos - st_head, ts = tpos - st_head;
            const uint32_t rh = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * (hs & 63u)), (int)r);
            const uint32_t rt = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * (ts & 63u)), (int)r);
            if (hpend && hs < nf) {
                r_head = rh;
                hpend = false;
            }
            if (tpend && ts < nf) {
                r_tail = rt;
                tpend = false;
            }
            ds_read8(ea, live_state);
            st_head += nf;
            head_slot += nf;
            head_slot = head_slot >= kCap ? head_slot - kCap : head_slot;
        };
        // append P ^ F (32 words, registers) for the lanes that take
        auto put = [&](bool take, const uint32_t* P, const uint32_t* F, uint32_t info) -> uint32_t {
            const uint64_t m = __ballot(take);
            const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            uint32_t slot = tail_slot + rank;
            slot = slot >= kCap ? slot - kCap : slot;
#if defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 8)
            if (false) {  // diagnostic build only: no stash writes (wrong CRCs)
#else
            if (take) {
#endif
                Pieces<0>::write(stash + slot * kEntry, P, F);
                const uint2 mt = make_uint2(k, info);
                asm volatile("ds_write_b64 %0, %1" ::"v"(meta + slot * 8u), "v"(mt) : "memory");
            }
            const uint32_t pos = st_tail + rank;
            const uint32_t c = (uint32_t)__popcll(m);
            st_tail += c;
            tail_slot += c;
            tail_slot = tail_slot >= kCap ? tail_slot - kCap : tail_slot;
            return pos;
        };

        // One boundary per lane that has one (ev): the datagram open in
        // sout ends at row byte b - 1 -- its state sout ^ F(b) goes to the
        // stash when it is tracked (take) -- and the next one starts at b
        // with state F(b) ^ C[b].  F(b) = the row from byte b on: b's piece
        // AND-masked in place in the image, earlier pieces from a zero piece.
        // (pre: the lane's piece b >> 4 as read with the row, or null: read here)
        auto boundary = [&](uint32_t t, bool ev, bool zero, uint32_t b, bool take, uint32_t* sout, const u32x4* pre) {
            {
                const uint32_t nst = (uint32_t)__popcll(__ballot(take));
                const uint32_t cnt = st_tail - st_head;
                if (nst && (cnt >= kFlush || cnt + nst > kCap)) flush(cnt < kFlush ? cnt : kFlush, sout);
            }
            const bool start = ev && !zero;
            const uint32_t c0 = ctab[b & 127u];
            if (start && b < 128u) {
                // keep the piece's bytes >= d: bits >= 8 d of the 128-bit piece
                const uint32_t d = b & 15u;
                const uint64_t lo = d < 8u ? ~0ull << (8u * d) : 0ull;
                const uint64_t hi = d < 8u ? ~0ull : ~0ull << (8u * (d - 8u));
                const uint32_t m[4] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
                if (pre) {
                    u32x4 v = *pre;
                    v.x &= m[0];
                    v.y &= m[1];
                    v.z &= m[2];
                    v.w &= m[3];
                    lds_write_piece(r0 ^ (16u * (b >> 4)), v);
                } else {
                    patch_piece<0>(r0 ^ (16u * (b >> 4)), m);
                }
            }
            uint32_t F[32];
            {
                const uint32_t bp = start ? (b >> 4) : 8u;
                uint32_t ad[8];
#pragma unroll
                for (int p = 0; p < 8; ++p) ad[p] = (uint32_t)p < bp ? zero_addr : r0 ^ (16u * p);
#if defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 4)
                (void)ad;  // diagnostic build only: no F(b) read (wrong CRCs)
#pragma unroll
                for (int w = 0; w < 32; ++w) F[w] = 0u;
#elif LNL_SPAN_F_MASK
                // only the lanes with a boundary read F: a row's other lanes
                // would move 128 bytes each through the LDS for nothing
                if (ev) read_row<0>(ad, F);
#else
                read_row<0>(ad, F);
#endif
            }
            const bool head = cs < 0;
            // (a normal datagram started in this segment: len < Sb < 2^14)
            const uint32_t len = head ? 0u : (t << 7) + b - (uint32_t)cs;
            const uint32_t pos = put(take, sout, F,
                                     (128u - b) | ((head ? kTypeHead : kTypeNormal) << 8) | (chdr << 10) | (len << 18));
            if (take && head) {
                hpos = pos;
                hpend = true;
                htrack = true;
                hk = k;
                hinfo = (t + 1u) | ((128u - b) << 8);
            }
            if (ev) {
                Q.pop();
                --qn;
                ++k;
            }
            if (start) {
                cs = (int32_t)((t << 7) + b);
                inj = b == 128u ? 0xFFFFFFFFu : 0u;  // C[0] at the next row's word 0
                if (A.mode != kSpanCrc) {  // the new datagram's first byte (intact after the patch)
                    hdr_next = b == 128u;
                    if (b < 128u) chdr = pre ? piece_byte(*pre, b) : lds_read_u8((r0 ^ (16u * (b >> 4))) + (b & 15u));
                }
            }
#pragma unroll
            for (int w = 0; w < 32; ++w) sout[w] = start ? F[w] : sout[w];
            sout[0] ^= start && b < 128u ? c0 : 0u;
        };
        // WALK, around each boundary() call: datagram k ends at row byte
        // b - 1 -- the rest of its walk (its bytes are intact until boundary()
        // masks b's piece), its count; then the next one starts at b (an empty
        // one ended there too: same start and header byte; at b = 128 it
        // opens with the next row)
        auto walk_end = [&](uint32_t t, bool ev, uint32_t b) {
#if defined(LNL_WALK_DIAG) && (LNL_WALK_DIAG & 2)
            return;  // diagnostic build only (wrong packets)
#endif
            const int32_t end = (int32_t)((t << 7) + b);
            walk_fields(t, ev, end - 4, end);
            if (ev) walk_close((uint32_t)(end - cs));
        };

        // ---- rows ---------------------------------------------------------
        // Row step: sout = A sin ^ row, then every datagram boundary in the
        // row (usually at most one per lane): the ended datagram's state
        // sout ^ F(b) goes to the stash, and sout = F(b) ^ C[b] starts the
        // next one.  sin / sout alternate between two arrays (no copies).
        auto row_step = [&](uint32_t t, u32x4* cur, uint32_t* sin, uint32_t* sout) {
            // the row into the image (8 lanes' lines per load), then this
            // buffer takes row t + 2.  The other buffer's 8 loads (row t + 1)
            // are younger; the last row waits for everything, so no row load
            // is in flight once the loop ends (the compiler does not see them
            // and would hand their registers to the epilogue)
            // WALK: the open container's entries in row t - 1 (its image is
            // still there until the transpose below; the last row's are left
            // to the global-memory finish after the loop), while row t's loads
            // land; the straddling entry's bytes 126, 127 of row t - 1 come
            // from wsv_next (taken from the row's registers as it streamed)
            // (measured the same after the wait)
            if constexpr (WALK)
                if (t > 0u) {
                    row_walk(t - 1u);
                    wlb = (wlb & 0xFFFF0000u) | wsv_next;
                }
            // a stash that has filled to the threshold folds here, while the
            // row's loads land, rather than inside a boundary after they have
            // (the boundary's own flush stays for a stash that fills within a
            // row).  Fused walk kernel only: its row steps are the heavy ones
            // (fd workload 339.3 -> 333.7 us at 50; the CRC and filter
            // kernels measured no different)
            if constexpr (WALK && LNL_SPAN_EARLY_FLUSH > 0) {
                const uint32_t cnt = st_tail - st_head;
                if (cnt >= (uint32_t)LNL_SPAN_EARLY_FLUSH) flush(cnt < kFlush ? cnt : kFlush, sin);
            }
            if (t + 1u < R)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            Transpose<0>::write(we, wo, cur);
            if (t + 2u < R) issue(t + 2u, cur);
#if LNL_SPAN_PRIO == 0
            // Issue fairness.  The two waves of a SIMD (wave, wave ^ 4) tie on
            // most issue slots, and ties go to the older wave: left alone, one
            // finishes its rows ~20 % after the other, with the SIMD half idle
            // meanwhile.  The wave that is ahead yields (priority 0), the one
            // behind takes priority 2.
            {
                ++rows_done;
                prog[wave] = rows_done;
                const uint32_t other = uni(prog[wave ^ 4u]);
                if (rows_done > other)
                    __builtin_amdgcn_s_setprio(0);
                else
                    __builtin_amdgcn_s_setprio(2);
            }
#endif
            const uint32_t rowst = t << 7, rowend = rowst + 128u;
#if defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 2)
            bool ev = false;  // diagnostic build only: rows and networks, no datagram boundaries
#else
            bool ev = is_open() && Q.front() <= rowend;
#endif
            const uint32_t b = ev ? Q.front() - rowst : 128u;
            u32x4 pre;  // the piece holding b, read with the row (no separate round trip to mask it)
            {
                uint32_t x[32], rad[8], rr = r0;
                asm volatile("" : "+v"(rr));  // 7 XORs per row rather than 8 registers held
#pragma unroll
                for (int p = 0; p < 8; ++p) rad[p] = rr ^ (16u * p);
                read_row_pre(rad, rr ^ (16u * ((b >> 4) & 7u)), x, pre);
                if (hdr_next) {  // a datagram that started at this row's byte 0
                    chdr = x[0] & 0xFFu;
                    if constexpr (WALK) walk_open();
                }
                hdr_next = false;
                if constexpr (WALK) wsv_next = x[31] >> 16;  // bytes 126, 127
                lnl_net_row_x(sin, x, sout);
            }
            sout[0] ^= inj;
            inj = 0u;
            if (!__any(ev)) return;
            // the first boundary of every lane (straight-line; rows with two or
            // more boundaries in one lane loop below)
            {
                const bool take = ev && cs >= -(int32_t)Sb;  // (a row's first boundary never ends an empty datagram)
                if constexpr (WALK) walk_end(t, ev, b);
                boundary(t, ev, false, b, take, sout, &pre);
                if constexpr (WALK)
                    if (ev && b < 128u) walk_open();
            }
            refill();
            ev = is_open() && Q.front() <= rowend;
#if defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 64)
            ev = false;  // diagnostic build only: a row's second and later boundaries skipped (wrong CRCs)
#endif
            while (__any(ev)) {
                const uint32_t b = ev ? Q.front() - rowst : 128u;
                const bool zero = ev && cs == (int32_t)(rowst + b);  // empty datagram: CRC 0, too short for the layer
                const bool take = ev && !zero;                     // (started in this row: never a head)
                if (zero) {
                    store_result(A, k, 0u, 0u, 0u);
                }
                if constexpr (WALK) walk_end(t, ev, b);
                boundary(t, ev, zero, b, take, sout, nullptr);
                if constexpr (WALK)
                    if (ev && b < 128u) walk_open();
                refill();
                ev = is_open() && Q.front() <= rowend;
            }
        };

        uint32_t sA[32], sB[32];
#pragma unroll
        for (int w = 0; w < 32; ++w) sA[w] = 0u;
        LNL_TL(2);
        for (uint32_t t = 0; t < R; t += 2u) {
            row_step(t, ra, sA, sB);
            if (t + 1u < R)
                row_step(t + 1u, rb, sB, sA);
            else {
#pragma unroll
                for (int w = 0; w < 32; ++w) sA[w] = sB[w];
            }
        }

        LNL_TL(3);
        if constexpr (WALK) {
            // an owned datagram still open runs on into the next segment(s):
            // finish its walk from global memory
            if (wlb & (kWalkOwned << 16)) {
                const uint64_t ds = segbase + (uint64_t)(int64_t)cs;
                const int64_t size = (int64_t)(bsh + A.off[k + 1u] - ds) - 4;
                if (!(wlb & (kWalkMerged << 16))) {
                    walk_block(kWalkPlain);
                } else {
                    int64_t pos = (int64_t)(int32_t)(wla & 0x3FFFFu) - cs;
                    uint32_t c = wla >> 18;
#if defined(LNL_WALK_DIAG) && (LNL_WALK_DIAG & 4)
                    wlb = 0u;  // diagnostic build only (wrong packets)
#endif
                    while ((wlb & (kWalkOn << 16)) && pos + 2 <= size) {
                        const uint32_t v = global_load3(ds + (uint64_t)pos);
                        const int64_t L = (int64_t)(v & 0xFFFFu);
                        pos += 2;
                        if (L > size - pos || L == 0 || !lnl_packet_verify_hdr((uint8_t)(v >> 16), (uint64_t)L)) break;
                        walk_record(c, ((uint32_t)pos << 16) | (uint32_t)L);
                        ++c;
                        pos += L;
                    }
                    walk_block(c);
                }
                wlb = 0u;
            }
        }
        // ---- the tail: the datagram still open, if it started here; then
        // fold everything still waiting.  (One that ends beyond the next
        // segment is an overflow datagram: its tail is folded but not used --
        // the next segment has no head -- and the batch kernel writes its CRC.
        // So no boundary past the segment is needed here.) --------------------
#if LNL_SPAN_TAIL_REG
        // (the tail folded in registers, after what the stash still holds:
        // no stash round trip and no second flush for it)
        {
            const bool tail = is_open() && k < n && cs >= 0 && cs < (int32_t)Sb;
#if LNL_SPAN_TAIL_REG == 2
            // full flushes first; the last partial one folds in the same pass as
            // the tails (the row registers are free now: no parking)
            while (st_tail - st_head >= kFlush) flush(kFlush, sA);
            const uint32_t nf = st_tail - st_head;
            if (nf != 0u) {
                const bool act = lane < nf;
                uint32_t slot = head_slot + lane;
                slot = slot >= kCap ? slot - kCap : slot;
                const uint32_t ea = stash + (act ? slot : 0u) * kEntry;
                uint32_t v[32];
                ds_read8(ea, v);
                uint2 mt;
                asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(mt) : "v"(meta + (act ? slot : 0u) * 8u) : "memory");
                uint32_t r = 0u, rt = 0u;
                if (act) r = phi_lds(T, tab_base, v);
                if (tail) rt = phi_lds(T, tab_base, sA);
                const uint32_t type = (mt.y >> 8) & 3u, e = mt.y & 127u;
                uint32_t crc = 0u;
                if (act) crc = final_crc_lds(tab_base, e, r);
                if (act && type == kTypeNormal && mt.x < n) store_result(A, mt.x, crc, mt.y >> 18, (mt.y >> 10) & 0xFFu);
                const uint32_t hs = hpos - st_head;
                const uint32_t rh = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * (hs & 63u)), (int)r);
                if (hpend && hs < nf) {
                    r_head = rh;
                    hpend = false;
                }
                st_head += nf;
                head_slot += nf;
                head_slot = head_slot >= kCap ? head_slot - kCap : head_slot;
                if (tail) r_tail = rt;
            } else if (tail) {
                r_tail = phi_lds(T, tab_base, sA);
            }
            if (tail) {
                tcs = (uint32_t)cs;
                thdr = chdr;
            }
#else
            for (;;) {
                const uint32_t cnt = st_tail - st_head;
                if (cnt == 0u) break;
                flush(cnt < kFlush ? cnt : kFlush, sA);
            }
            if (tail) {
                r_tail = phi_lds(T, tab_base, sA);
                tcs = (uint32_t)cs;
                thdr = chdr;
            }
#endif
        }
#else
        {
            const bool tail = is_open() && k < n && cs >= 0 && cs < (int32_t)Sb;
            bool tdone = !tail;
            for (;;) {
                const uint32_t nst = (uint32_t)__popcll(__ballot(!tdone));
                const uint32_t cnt = st_tail - st_head;
                if (nst == 0u && cnt == 0u) break;
                if (nst == 0u || cnt >= kFlush || cnt + nst > kCap) {
                    flush(cnt < kFlush ? cnt : kFlush, sA);
                    continue;
                }
                const uint32_t pos = put(!tdone, sA, kZero32, kTypeTail << 8);
                if (!tdone) {
                    tpos = pos;
                    tpend = true;

                    tcs = (uint32_t)cs;
                    thdr = chdr;
                }
                tdone = true;
            }
        }
#endif
        LNL_TL(4);
        // heads: CRC = ~step^(-8e)(step^(1024 m) tail ^ head), the tail from
        // the previous lane; lane 0's from the previous wave-batch (below)
        {
            const int src = (int)(lane - 1u) & 63;
            const uint32_t tprev = (uint32_t)__shfl((int)r_tail, src, 64);
            const uint32_t tcs_prev = (uint32_t)__shfl((int)tcs, src, 64);
            const uint32_t thdr_prev = (uint32_t)__shfl((int)thdr, src, 64);
            if (htrack && lane != 0u && hk < n) {
                const uint32_t m = hinfo & 0xFFu, e = (hinfo >> 8) & 0xFFu;
#if LNL_SPAN_FIN_LDS
                const uint32_t crc = final_crc_lds(tab_base, e, lnl_span_rows(A.tab, m, tprev) ^ r_head);
#else
                const uint32_t crc = lnl_span_final(A.tab, e, lnl_span_rows(A.tab, m, tprev) ^ r_head);
#endif
                // (the head's length: its part in the previous segment and in this one)
                store_result(A, hk, crc, (Sb - tcs_prev) + (m << 7) - e, thdr_prev);
            }
        }
        LNL_TL(5);
        // Wave-batch boundaries: lane 0's head came in from wave-batch wb - 1's
        // lane 63, lane 63's tail goes on to wb + 1's lane 0.  Each side writes
        // its part into the boundary's exchange block (crc32c_span.h kSpanXch*)
        // and then swaps its arrival (the call's epoch and its side) into the
        // block's arrival word; the side whose swap returns the other side's
        // arrival of this epoch has both parts and combines them.  Nothing is
        // reset: a word left by an earlier call (or by an aborted one) holds
        // another epoch and never pairs.  The parts are device-scope (sc1)
        // stores and loads and the arrival a device-scope atomic, ordered by a
        // vmcnt(0) between the stores and the arrival: no L2 writeback or
        // invalidate (an acq_rel fence at agent scope does both on gfx950, per
        // wave, and measured 35 us slower).
        if (live && (lane == 0u || lane == 63u)) {
            const uint32_t w = lane == 0u ? wb : wb + 1u;  // boundary w: segments 64 w - 1 | 64 w
            if (w != 0u && w < nwb) {
                uint32_t* const xb = A.xch + (size_t)w * kSpanXchWords;
                auto put_x = [&](uint32_t i, uint32_t v) {
                    __hip_atomic_store(xb + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                };
                auto get_x = [&](uint32_t i) -> uint32_t {
                    return __hip_atomic_load(xb + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                };
                const uint32_t side = lane == 0u ? kSpanSideHead : kSpanSideTail;
                if (lane == 0u) {
                    put_x(kSpanXchHead, r_head);
                    put_x(kSpanXchHeadIdx, hk);
                    put_x(kSpanXchHeadInfo, hinfo | (htrack ? kSpanHeadBit : 0u));
                } else {
                    put_x(kSpanXchTail, r_tail);
                    put_x(kSpanXchTailInfo, tcs | (thdr << 16));
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the parts are out before the arrival
                // (the epoch through an empty asm here: left alone, the compiler
                // hoists both arrival values out of the wave-batch loop and
                // spills them across the rows)
                uint64_t ep = A.epoch;
                uint32_t sd = side;
                asm volatile("" : "+s"(ep), "+v"(sd));
                const uint64_t prior = __hip_atomic_exchange(reinterpret_cast<uint64_t*>(xb + kSpanXchFlag),
                                                             span_arrival(ep, sd), __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
                if (prior == span_arrival(ep, kSpanSideHead ^ kSpanSideTail ^ sd)) {
                    const uint32_t head = lane == 0u ? r_head : get_x(kSpanXchHead);
                    const uint32_t hidx = lane == 0u ? hk : get_x(kSpanXchHeadIdx);
                    const uint32_t info = lane == 0u ? (hinfo | (htrack ? kSpanHeadBit : 0u)) : get_x(kSpanXchHeadInfo);
                    const uint32_t tail = lane == 63u ? r_tail : get_x(kSpanXchTail);
                    const uint32_t tinf = lane == 63u ? (tcs | (thdr << 16)) : get_x(kSpanXchTailInfo);
                    if ((info & kSpanHeadBit) && hidx < n) {
                        const uint32_t m = info & 0xFFu, e = (info >> 8) & 0xFFu;
#if LNL_SPAN_FIN_LDS
                        const uint32_t crc = final_crc_lds(tab_base, e, lnl_span_rows(A.tab, m, tail) ^ head);
#else
                        const uint32_t crc = lnl_span_final(A.tab, e, lnl_span_rows(A.tab, m, tail) ^ head);
#endif
                        store_result(A, hidx, crc, (Sb - (tinf & 0xFFFFu)) + (m << 7) - e, tinf >> 16);
                    }
                }
            }
        }
    }
#if defined(LNL_SPAN_DIAG) && (LNL_SPAN_DIAG & 16)
    LNL_TL(6);
    if (lane < 7u && 8u * gw + 8u <= n) {
        uint32_t v = tl[0];
#pragma unroll
        for (int i = 1; i < 7; ++i) v = lane == (uint32_t)i ? tl[i] : v;
        A.out[8u * gw + lane] = v;
    }
#endif
}

}  // namespace

// Scratch: two 8-word control blocks (crc32c_span.h kSpanCtl*) and the
// wave-batch boundaries' exchange blocks (kSpanXch*: arrival words of epoch 0
// until a call writes them; all of it zeroed once at allocation), then the
// overflow list.
size_t span_scratch_zero_words(uint32_t waves) {
    return 2 * kSpanCtlWords + (size_t)(span_max_segments(waves) / 64u) * kSpanXchWords;
}

size_t span_scratch_words(uint32_t n, uint32_t waves) { return span_scratch_zero_words(waves) + n; }

void span_scratch_layout(SpanArgs& a, uint32_t* s, uint32_t parity) {
    a.ctl = s + kSpanCtlWords * (parity & 1u);
    a.ctl_next = s + kSpanCtlWords * (~parity & 1u);
    a.xch = s + 2 * kSpanCtlWords;
    a.ovf = s + span_scratch_zero_words(a.waves);
}

hipError_t launch_span(const SpanArgs& a, int grid, hipStream_t stream) {
    if (a.wblk)
        hipLaunchKernelGGL(crc32c_span_kernel<true>, dim3(grid), dim3(kThreads), 0, stream, a);
    else
        hipLaunchKernelGGL(crc32c_span_kernel<false>, dim3(grid), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
