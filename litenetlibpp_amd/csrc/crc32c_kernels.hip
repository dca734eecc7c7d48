// crc32c_kernels.hip -- batched CRC-32C over UDP datagrams for gfx950 (MI355X).
//
// One wavefront owns a BATCH of 64 datagrams, one per lane.  Every datagram is
// processed as end-aligned 128-byte rows (see crc32c_bitslice.h for the
// algebra): the wave streams rows HBM -> LDS with global_load_lds_dwordx4
// (LDS-DMA, no VGPR staging), each lane reads its own row back with
// 8 x ds_read_b128, transposes it into 32 bit-sliced words and runs one
// generated XOR network (S = M_128(S) ^ X) -- ~420 VALU ops per 128 bytes, no
// tables, no bank conflicts, no MFMA (CRC is a GF(2) polynomial remainder, not
// a dense contraction).  After the last row a 5-level bit-sliced tree folds the
// 32 streams and each lane stores one uint32.
//
// Memory pipeline per wave: two 8 KiB LDS row buffers; row s+2 is issued as
// soon as row s has been read into registers, so two rows (16 KiB) per wave and
// 128 KiB per CU (8 waves) are in flight while the wave computes.  HBM access:
// each glds wave-instruction moves 8 datagrams x 128 contiguous bytes; the LDS
// image is XOR-swizzled on the SOURCE address (slot = piece ^ ((row>>1)&7)) so
// that the per-lane ds_read_b128 of a whole row is bank-conflict free.
//
// The row reads are one inline-asm block (8 x ds_read_b128 + lgkmcnt(0)):
// hipcc would otherwise put `s_waitcnt vmcnt(0)` in front of any LDS read that
// follows an LDS-DMA, draining the prefetched rows every step.  Row arrival is
// instead waited for with a counted `s_waitcnt vmcnt(8)` (exactly 8 VMEM
// instructions per row are ever issued, see issue_row).
//
// Waves are persistent (grid = min(batches, CUs x 8 waves)) and stride over
// batches, so rows of the next batch are prefetched under the current batch's
// last rows and its finalize.
//
// Hot path of BASELINE configs 2-4 (fixed stride, CSR, sharded fixed stride)
// and of the batched inbound verify; boundary: include/lnl_crc32c.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_bitslice.h"
#include "crc32c_kernels.h"

namespace lnl {

namespace {

constexpr int kWaves = kBlockThreads / 64;  // waves per workgroup
constexpr int kRowU4 = 8;                   // one 128-byte row = 8 x uint4
constexpr int kBufU4 = 64 * kRowU4;         // one row buffer = 64 rows = 8 KiB
constexpr uint32_t kBufBytes = kBufU4 * 16;

__device__ LNL_INLINE uint32_t swz(uint32_t row) { return (row >> 1) & 7u; }

__device__ LNL_INLINE uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Per-batch parameters.  Wave-uniform fields are kept in SGPRs (readfirstlane).
// "Compute" fields describe the lane's own datagram; "load" fields describe,
// for each of the 8 glds instructions i of a row, the datagram q = 8i + lane/8
// whose 16-byte piece this lane fetches.
struct Batch {
    uint32_t valid;      // uniform: batch exists
    uint32_t rows;       // uniform: max over lanes of ceil(len/128)
    uint32_t max_first;  // uniform: max over lanes of `first`
    uint32_t simple;     // uniform: no idle lane and no near-base datagram
    uint32_t any_nb;     // uniform: some datagram's first window starts before d_base
    // compute lane
    uint32_t p;      // datagram index (>= n: idle lane)
    uint32_t len;    // bytes covered by the CRC
    uint32_t first;  // first real row of this lane (rows before it are virtual zeros)
    uint32_t nb;     // this lane's first window starts before d_base: filled by hand
    int64_t win;     // byte offset (from d_base) of the lane's first real window
    // load lanes: absolute address of row 0 of datagram q (piece included)
    uint64_t ladr[8];
    uint32_t lfirst[8];  // first real row of q | 1<<30 idle | 1<<31 near-base
};

template <int kMode>
__device__ LNL_INLINE void lane_extent(const BatchArgs& a, uint32_t p, uint64_t& start,
                                       uint32_t& len) {
    if (p >= a.n) {
        start = 0;
        len = 0;
        return;
    }
    if constexpr (kMode == kModeFixed) {
        start = (uint64_t)p * a.stride;
        len = a.len;
    } else {
        const uint64_t s = a.off[p], e = a.off[p + 1];
        const uint32_t total = (uint32_t)(e - s);
        start = s - a.off0;
        if constexpr (kMode == kModeVerify)
            len = total >= 5u ? total - 4u : 0u;
        else
            len = total;
    }
}

__device__ LNL_INLINE uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

template <int kMode>
__device__ LNL_INLINE void make_batch(const BatchArgs& a, uint32_t b, uint32_t nbatch, Batch& B) {
    // Branch-free on purpose (every field written on every path keeps the
    // struct in registers).  An invalid batch (b >= nbatch) has only idle lanes.
    const uint32_t lane = __lane_id();
    B.valid = uni(b < nbatch ? 1u : 0u);
    uint64_t start;
    uint32_t len;
    B.p = B.valid ? b * 64u + lane : a.n;
    lane_extent<kMode>(a, B.p, start, len);
    const uint32_t T = (len + 127u) >> 7;
    const uint32_t pad = (T << 7) - len;
    B.len = len;
    if constexpr (kMode == kModeFixed)
        B.rows = uni(B.valid ? (a.len + 127u) >> 7 : 0u);  // idle lanes: last batch only
    else
        B.rows = uni(wave_max(T));
    B.first = B.rows - T;
    B.max_first = uni(wave_max(B.first));
    B.win = (int64_t)start - (int64_t)pad;
    const uint32_t idle = (T == 0u || B.p >= a.n) ? 1u : 0u;
    B.nb = (!idle && (int64_t)start < (int64_t)pad) ? 1u : 0u;
    B.any_nb = uni(__any(B.nb) ? 1u : 0u);
    B.simple = uni(__any(idle | B.nb) ? 0u : 1u);
    // row t of datagram q starts at d_base + win_q + 128 (t - first_q)
    const uint64_t row0 = (uint64_t)(uintptr_t)a.base + (uint64_t)(B.win - ((int64_t)B.first << 7));
    const uint32_t fl = B.first | (idle << 30) | (B.nb << 31);
    const uint32_t sub = lane >> 3, slot = lane & 7u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t q = 8u * i + sub;
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)row0, q, 64);
        const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(row0 >> 32), q, 64);
        B.ladr[i] = (((uint64_t)hi << 32) | lo) + 16u * (slot ^ swz(q));
        B.lfirst[i] = (uint32_t)__shfl((int)fl, q, 64);
    }
}

// Issue the 8 LDS-DMA instructions that bring row t of batch B into `buf`.
// All 8 are issued unconditionally (inactive lanes fetch a 16-byte dummy line
// into a slot that is masked): the counted `s_waitcnt vmcnt(8)` in the main
// loop relies on exactly 8 VMEM instructions per row.
__device__ LNL_INLINE void issue_row(const BatchArgs& a, const Batch& B, uint32_t t, uint4* buf) {
    const uint64_t dt = (uint64_t)t << 7;
    if (B.simple && t > B.max_first) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)(B.ladr[i] + dt),
                                             (void*)(buf + 64 * i), 16, 0, 0);
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t f = B.lfirst[i];
            const uint32_t first = f & 0x3FFFFFFFu;
            bool on = !(f & (1u << 30)) && t >= first;
            if (f & (1u << 31)) on = on && t != first;  // near-base first row: filled by hand
            const uint64_t src = on ? B.ladr[i] + dt : (uint64_t)(uintptr_t)a.dummy;
            __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)src, (void*)(buf + 64 * i), 16,
                                             0, 0);
        }
    }
}

// Rare path: the lane's first window starts before d_base (a datagram within
// 127 bytes of the buffer start).  The glds lanes fetched a dummy line for that
// row; the lane writes its row image itself from in-bounds bytes only (the
// bytes before d_base are virtual padding and get masked anyway).
__device__ LNL_INLINE void fill_near_base_row(const BatchArgs& a, int64_t win, uint4* buf,
                                              uint32_t lane) {
    uint32_t* row = reinterpret_cast<uint32_t*>(buf + lane * kRowU4);
#pragma unroll 1
    for (int w = 0; w < 32; ++w) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int64_t off = win + 4 * w + b;
            const uint32_t byte = off >= 0 ? a.base[off] : 0u;
            v |= byte << (8 * b);
        }
        row[4 * (((uint32_t)w >> 2) ^ swz(lane)) + (w & 3)] = v;
    }
}

// 8 x ds_read_b128 of the lane's row + lgkmcnt(0), as ONE asm statement so that
// no consumer can be scheduled before the wait.  ad[k]: LDS byte address of
// piece k of the row in buffer 0; OFF selects the buffer.
template <uint32_t OFF>
__device__ LNL_INLINE void read_row(const uint32_t* ad, uint32_t* x) {
    uint4 v0, v1, v2, v3, v4, v5, v6, v7;
    asm volatile(
        "ds_read_b128 %0, %8 offset:%16\n\t"
        "ds_read_b128 %1, %9 offset:%16\n\t"
        "ds_read_b128 %2, %10 offset:%16\n\t"
        "ds_read_b128 %3, %11 offset:%16\n\t"
        "ds_read_b128 %4, %12 offset:%16\n\t"
        "ds_read_b128 %5, %13 offset:%16\n\t"
        "ds_read_b128 %6, %14 offset:%16\n\t"
        "ds_read_b128 %7, %15 offset:%16\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(v4), "=&v"(v5), "=&v"(v6), "=&v"(v7)
        : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]),
          "v"(ad[7]), "i"(OFF)
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

template <int kMode>
__device__ LNL_INLINE void store_result(const BatchArgs& a, const Batch& B, uint32_t crc) {
    if (B.p >= a.n) return;
    if constexpr (kMode == kModeVerify) {
        const uint64_t e = a.off[B.p + 1];
        const uint32_t total = (uint32_t)(e - a.off[B.p]);
        uint32_t ok = 0;
        if (total >= 5u) {
            const uint8_t* tail = a.base + (e - a.off0) - 4;
            const uint32_t stored = (uint32_t)tail[0] | ((uint32_t)tail[1] << 8) |
                                    ((uint32_t)tail[2] << 16) | ((uint32_t)tail[3] << 24);
            ok = stored == crc;
        }
        a.ok[B.p] = (uint8_t)ok;
        if (a.out) a.out[B.p] = crc;
    } else {
        a.out[B.p] = crc;
    }
}

template <int kMode>
__global__ __launch_bounds__(kBlockThreads, 2) void crc32c_batch_kernel(BatchArgs a) {
    __shared__ __attribute__((aligned(16))) uint4 lds[kWaves][2][kBufU4];
    const uint32_t lane = __lane_id();
    const uint32_t wave = uni(threadIdx.x >> 6);
    uint4* const buf_base = &lds[0][0][0] + wave * (2 * kBufU4);
    const uint32_t nbatch = (a.n + 63u) >> 6;
    const uint32_t gw = blockIdx.x * kWaves + wave;
    const uint32_t nw = gridDim.x * kWaves;

    // LDS byte addresses of this lane's 8 row pieces in buffer 0
    uint32_t rad[8];
    {
        const uint32_t rowb = (uint32_t)(uintptr_t)(buf_base + lane * kRowU4);
#pragma unroll
        for (int k = 0; k < 8; ++k) rad[k] = rowb + 16u * ((uint32_t)k ^ swz(lane));
    }

    Batch cur, nxt;
    uint32_t b = gw;
    make_batch<kMode>(a, b, nbatch, cur);
    if (!cur.valid) return;
    make_batch<kMode>(a, b + nw, nbatch, nxt);

    // Row pipeline.  `step` counts computed rows; row `step` lives in buffer
    // step & 1.  have0: row `step` has been issued; have1: row step+1 has been
    // issued.  Rows are normally issued two steps ahead; a row that could not be
    // (it belongs to the batch after `nxt`) is issued on demand.
    uint32_t step = 0, t = 0;
    uint32_t have0 = 0, have1 = 0;
    uint32_t s[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) s[k] = 0;
    if (cur.rows > 0) {
        issue_row(a, cur, 0, buf_base);
        have0 = 1;
        if (cur.rows > 1) {
            issue_row(a, cur, 1, buf_base + kBufU4);
            have1 = 1;
        } else if (nxt.valid && nxt.rows > 0) {
            issue_row(a, nxt, 0, buf_base + kBufU4);
            have1 = 1;
        }
    }

    while (true) {
        if (cur.rows == 0) {
            // every datagram of this batch is empty: CRC = crc32c("") = 0, and
            // in verify mode none has the 5 bytes a valid datagram needs
            store_result<kMode>(a, cur, 0u);
            b += nw;
            cur = nxt;
            if (!cur.valid) break;
            make_batch<kMode>(a, b + nw, nbatch, nxt);
            have0 = 0;  // nothing can have been issued for it
            have1 = 0;
            continue;
        }
        const uint32_t odd = uni(step & 1u);
        uint4* const buf = buf_base + odd * kBufU4;
        if (!have0) {
            issue_row(a, cur, t, buf);
            have1 = 0;  // drain everything below
        }
        if (have1)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (cur.any_nb && t <= cur.max_first) {
            if (cur.nb && t == cur.first) fill_near_base_row(a, cur.win, buf, lane);
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
        uint32_t x[32];
        if (odd)
            read_row<kBufBytes>(rad, x);
        else
            read_row<0>(rad, x);
        // prefetch row step+2 into the buffer just drained
        uint32_t have2 = 0;
        {
            const uint32_t t2 = t + 2;
            if (t2 < cur.rows) {
                issue_row(a, cur, t2, buf);
                have2 = 1;
            } else if (nxt.valid && t2 - cur.rows < nxt.rows) {
                issue_row(a, nxt, t2 - cur.rows, buf);
                have2 = 1;
            }
        }
        have0 = have1;
        have1 = have2;

        lnl_transpose32(x);
        if (t <= cur.max_first + 1u) {
            uint32_t keep[4], inv0[4], inv1[4];
            lnl_first_row_masks((cur.rows - cur.first) * 128u - cur.len, cur.len, keep, inv0, inv1);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t kq = t < cur.first ? 0u : (t == cur.first ? keep[q] : 0xFFFFFFFFu);
                const uint32_t iq = t == cur.first ? inv0[q] : (t == cur.first + 1u ? inv1[q] : 0u);
                keep[q] = kq;
                inv0[q] = iq;
            }
            lnl_apply_masks(x, keep, inv0);
        }
        uint32_t o[32];
        lnl_net_adv128_x(s, x, o);
#pragma unroll
        for (int k = 0; k < 32; ++k) s[k] = o[k];

        ++step;
        if (++t == cur.rows) {
            store_result<kMode>(a, cur, lnl_finalize(s) ^ lnl_final_xor(cur.len));
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] = 0;
            t = 0;
            b += nw;
            cur = nxt;
            if (!cur.valid) break;
            make_batch<kMode>(a, b + nw, nbatch, nxt);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

hipError_t launch_crc32c_batch(const BatchArgs& a, int mode, int grid, hipStream_t stream) {
    switch (mode) {
        case kModeFixed:
            hipLaunchKernelGGL(crc32c_batch_kernel<kModeFixed>, dim3(grid), dim3(kBlockThreads), 0,
                               stream, a);
            break;
        case kModeCsr:
            hipLaunchKernelGGL(crc32c_batch_kernel<kModeCsr>, dim3(grid), dim3(kBlockThreads), 0,
                               stream, a);
            break;
        case kModeVerify:
            hipLaunchKernelGGL(crc32c_batch_kernel<kModeVerify>, dim3(grid), dim3(kBlockThreads), 0,
                               stream, a);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace lnl
