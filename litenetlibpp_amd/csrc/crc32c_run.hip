// crc32c_run.hip -- fixed-stride batches as LANE RUNS (configs 2 and 4).
//
// The any-layout batch kernel (crc32c_kernels.hip) gives every lane one
// datagram, so every lane pays the framing of its own first and last line,
// the wave waits for its longest datagram, the line two neighbouring datagrams
// share is fetched twice (8 % extra HBM traffic at 1400 B), and every datagram
// pays a full 5-level fold.  For a fixed stride S all of that can be removed:
//
//  * A lane owns a RUN of K consecutive datagrams and streams the lines the run
//    covers exactly once, datagram after datagram: the line where one datagram
//    ends and the next begins is fetched once and split between them.
//  * The lanes of a wave are spaced Q datagrams apart, with Q * S a multiple of
//    128 (Q = max(K, 128 / gcd(S, 128))).  Every lane then has the same offset
//    within its 128-byte line, so the whole line schedule -- which row ends
//    datagram k, which row starts datagram k+1, the byte masks, the CRC init
//    word, the final correction table -- is WAVE-UNIFORM: scalar compares and
//    scalar masks, no per-lane framing, no zero-line fetches, no idle lanes.
//    A superblock of 64 Q datagrams is covered by Q / K waves (slices): wave
//    (g, j), lane l owns datagrams g*64Q + l*Q + j*K + [0, K).
//  * Folds are paired: datagrams 2i and 2i+1 of a run share fold levels 2..5
//    (lnl_fold_pair), ~40 % fewer fold ops per datagram.
//
// Requirements (checked by the host planner, crc32c_api.cpp): len >= 129 (a
// datagram's first and last byte are in different lines), S >= len (at most
// one start and one end per line), K even.  Datagrams beyond the last whole
// superblock go to the batch kernel.
//
// Memory pipeline, LDS layout and inline-asm row reads are the batch
// kernel's (crc32c_device.h); the loads use an SGPR line base that advances by
// 128 bytes per row plus a per-lane 32-bit offset fixed for the whole kernel,
// so issuing a row costs no VALU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"
#include "crc32c_kernels.h"

// cache policy of the row loads (0 default, 2 nt)
#ifndef LNL_RUN_AUX
#define LNL_RUN_AUX 2
#endif

namespace lnl {

namespace {

using namespace dev;

// issue fairness between the two waves of a SIMD (needs both in one
// workgroup: LNL_RUN_THREADS 512); see crc32c_span.hip
#ifndef LNL_RUN_PRIO
#define LNL_RUN_PRIO 0
#endif
constexpr int kWaves = kRunThreads / 64;
constexpr int kBufsU4 = kWaves * 2 * kBufU4;  // the waves' row buffers
constexpr int kFoldLdsU4 = kFoldU4 + 1;       // the tables + one uint4: per-wave progress words
#ifndef LNL_RUN_EARLY_ROWS
#define LNL_RUN_EARLY_ROWS 1  // first rows issued before the tables land (0: after, as before round 3)
#endif
static_assert(!LNL_RUN_PRIO || kWaves == 8, "priority balancing pairs wave w with w ^ 4");

// Wave-uniform description of one lane-run batch.
struct RunBatch {
    uint64_t line;  // address of row 0 of lane 0 (128-byte aligned)
    uint32_t d0;    // datagram index of lane 0's first datagram
    uint32_t ph;    // offset of every lane's first datagram in its row 0
    uint32_t rows;  // rows per lane
};

__device__ LNL_INLINE RunBatch run_batch(const RunArgs& a, uint32_t wb) {
    RunBatch B;
    const uint32_t g = wb / a.slices, j = wb - g * a.slices;
    B.d0 = g * 64u * a.q + j * a.k;
    const uint64_t A0 = (uint64_t)(uintptr_t)a.base + (uint64_t)B.d0 * a.stride;
    B.ph = (uint32_t)A0 & 127u;
    B.line = A0 - B.ph;
    B.rows = (B.ph + (a.k - 1u) * (uint32_t)a.stride + a.len + 127u) >> 7;
    return B;
}

// The 8 LDS-DMA instructions of row t (64 lanes' lines) into buf.  glds
// instruction i, this lane: piece (lane & 7) of the row of lane q = 8i + lane/8,
// whose run starts q*Q*S bytes after lane 0's (same line offset).  The slot
// swizzle of q = 8i + sub is swz(sub) for even i and swz(sub) ^ 4 for odd i, so
// the per-lane part is one of two offsets (off[0] / off[1]) and the 8i*Q*S part
// goes into the scalar base.
__device__ LNL_INLINE void issue_run_row(const RunBatch& B, uint32_t t, const uint32_t* off, uint32_t qs8,
                                         uint4* buf) {
    const uint8_t* row = (const uint8_t*)(uintptr_t)(B.line + ((uint64_t)t << 7));
#pragma unroll
    for (int i = 0; i < 8; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(row + (uint64_t)i * qs8 + off[i & 1]),
                                         (void*)(buf + 64 * i), 16, 0, LNL_RUN_AUX);
}

// Scalar (SGPR) byte masks of row word w for a datagram END at row byte be
// (keep bytes <= be) and a START at row byte bs (keep bytes >= bs): all-ones /
// zero away from the boundary word, a partial mask on it.  Inline asm so they
// stay on the scalar unit (as plain C the compiler picks VALU clamps and parks
// the 32 constants in VGPRs); crc32c_bitslice.h's lnl_word_keep_le/ge are the
// same masks (the CPU emulation checks those).
struct EdgeMask {
    uint32_t wi;  // boundary word
    uint32_t pm;  // mask of the boundary word
};
__device__ LNL_INLINE EdgeMask end_mask(uint32_t be) {
    return {be >> 2, (be & 3u) == 3u ? 0xFFFFFFFFu : (1u << (8u * ((be & 3u) + 1u))) - 1u};
}
__device__ LNL_INLINE EdgeMask start_mask(uint32_t bs) {
    return {bs >> 2, 0xFFFFFFFFu << (8u * (bs & 3u))};
}
template <int W>
__device__ LNL_INLINE uint32_t word_keep_le(const EdgeMask& m) {  // W < wi: ~0, W == wi: pm, else 0
    uint32_t r;
    asm("s_cmp_lt_u32 %1, %2\n\ts_cselect_b32 %0, -1, 0\n\ts_cmp_eq_u32 %1, %2\n\ts_cselect_b32 %0, %3, %0"
        : "=&s"(r) : "i"(W), "s"(m.wi), "s"(m.pm) : "scc");
    return r;
}
template <int W>
__device__ LNL_INLINE uint32_t word_keep_ge(const EdgeMask& m) {  // W > wi: ~0, W == wi: pm, else 0
    uint32_t r;
    asm("s_cmp_gt_u32 %1, %2\n\ts_cselect_b32 %0, -1, 0\n\ts_cmp_eq_u32 %1, %2\n\ts_cselect_b32 %0, %3, %0"
        : "=&s"(r) : "i"(W), "s"(m.wi), "s"(m.pm) : "scc");
    return r;
}

template <int W>
struct MaskLoop {  // x[w] &= keep(w) for w = W..31 (compile-time word index for the asm)
    template <bool kEnd>
    __device__ static LNL_INLINE void apply(const uint32_t* x, uint32_t* y, const EdgeMask& m) {
        y[W] = x[W] & (kEnd ? word_keep_le<W>(m) : word_keep_ge<W>(m));
        MaskLoop<W + 1>::template apply<kEnd>(x, y, m);
    }
};
template <>
struct MaskLoop<32> {
    template <bool kEnd>
    __device__ static LNL_INLINE void apply(const uint32_t*, uint32_t*, const EdgeMask&) {}
};

__device__ LNL_INLINE uint32_t final_map(uint32_t fold_base, uint32_t e, uint32_t r) {
    r = fold_apply_lds(fold_base + 512u * lnl_table_b(e), r);
    r = fold_apply_lds(fold_base + 512u * lnl_table_a(e), r);
    return ~r;
}

__global__ __launch_bounds__(kRunThreads, 512 / kRunThreads) void crc32c_run_kernel(RunArgs a) {
    // row buffers and tables in separate LDS arrays: the tables' LDS writes
    // then provably do not touch the LDS-DMA destinations, and the wait before
    // them can leave the first rows in flight
    __shared__ __attribute__((aligned(128))) uint4 bufs[kBufsU4];
    __shared__ __attribute__((aligned(16))) uint4 fold_arr[kFoldLdsU4];
    const uint32_t lane = __lane_id();
    const uint32_t wave = uni(threadIdx.x >> 6);
    uint4* const buf_base = bufs + wave * (2 * kBufU4);
    uint4* const fold_lds = fold_arr;
    const uint32_t fold_base = (uint32_t)(uintptr_t)fold_lds;
    uint32_t* const prog = reinterpret_cast<uint32_t*>(fold_lds + kFoldU4);
    uint32_t rows_done = 0;
    (void)prog;
    (void)rows_done;
    const uint32_t gw = blockIdx.x * kWaves + wave;
    const uint32_t nw = gridDim.x * kWaves;
    const bool active = gw < a.nb;

    uint32_t off[2];
    const uint32_t qs8 = 8u * a.q * (uint32_t)a.stride;
    {
        const uint32_t sub = lane >> 3, slot = lane & 7u;
        off[0] = sub * a.q * (uint32_t)a.stride + 16u * (slot ^ swz(sub));
        off[1] = sub * a.q * (uint32_t)a.stride + 16u * (slot ^ swz(sub) ^ 4u);
    }
    // LDS address of piece k of this lane's row: r0 ^ 16k (the row is 128-byte
    // aligned, so the slot swizzle is an XOR on address bits 4..6); recomputed
    // per row -- 7 VALU -- instead of holding 8 registers across the fold
    const uint32_t r0 = (uint32_t)(uintptr_t)(buf_base + lane * kRowU4) | (16u * swz(lane));
    const uint32_t S = (uint32_t)a.stride, L = a.len, K = a.k;
    const bool contiguous = S == L;

    uint32_t wb = gw;
    RunBatch cur{}, nxt{};
    bool has_nxt = false;
    // The tables' loads go out first, then this wave's first two rows (rows >= 2
    // always: len >= 129), then the tables go to LDS: the wait before those LDS
    // writes counts the 16 row loads issued after them, so the rows stream
    // while the tables land (before round 3 the rows waited for the tables).
    {
        constexpr int kPer = (kFoldU4 + kRunThreads - 1) / kRunThreads;
        u32x4 tv[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {  // (inline asm: the compiler inserts no wait for them)
            const int i = (int)threadIdx.x + j * kRunThreads;
            const uint64_t at = (uint64_t)(uintptr_t)a.fold + 16u * (uint32_t)(i < kFoldU4 ? i : kFoldU4 - 1);
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(tv[j]) : "v"(at) : "memory");
        }
        auto first_rows = [&]() {
            if (!active) return;
            cur = run_batch(a, wb);
            has_nxt = wb + nw < a.nb;
            if (has_nxt) nxt = run_batch(a, wb + nw);
            issue_run_row(cur, 0, off, qs8, buf_base);
            issue_run_row(cur, 1, off, qs8, buf_base + kBufU4);
        };
#if LNL_RUN_EARLY_ROWS
        first_rows();
        if (active)
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // the tables only
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int i = (int)threadIdx.x + j * kRunThreads;
            asm volatile("" : "+v"(tv[j]));
            if (i < kFoldU4) lds_write_piece(fold_base + 16u * (uint32_t)i, tv[j]);
        }
        if (threadIdx.x == 0) lds_write_piece(fold_base + 16u * (uint32_t)kFoldU4, u32x4{0u, 0u, 0u, 0u});
        // the tables are in LDS (lgkmcnt) before the barrier; a plain s_barrier,
        // not __syncthreads, whose fence would also wait for the rows in flight
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#if !LNL_RUN_EARLY_ROWS
        first_rows();
#endif
    }
    if (!active) return;

    uint32_t s[32], P[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) s[k] = P[k] = 0;
    // line schedule of the current batch (scalar): next datagram to start /
    // end, byte offsets (from row 0) of its first / last byte
    uint32_t ks = 0, ke = 0, sb = cur.ph, eb = cur.ph + L - 1u, eprev = 0;
    uint32_t dl = cur.d0 + lane * a.q;  // this lane's first datagram
    uint32_t step = 0, t = 0, have1 = 1;

    while (true) {
        const uint32_t odd = step & 1u;
        uint4* const buf = buf_base + odd * kBufU4;
        if (have1)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t x[32];
        {
            uint32_t rad[8], rb = r0;
            asm volatile("" : "+v"(rb));  // keep the 7 XORs in the loop (no hoisting)
#pragma unroll
            for (int k = 0; k < 8; ++k) rad[k] = rb ^ (16u * k);
            if (odd)
                read_row<kBufBytes>(rad, x);
            else
                read_row<0>(rad, x);
        }
        {
            const uint32_t t2 = t + 2u;
            have1 = 0;
            if (t2 < cur.rows) {
                issue_run_row(cur, t2, off, qs8, buf);
                have1 = 1;
            } else if (has_nxt) {
                issue_run_row(nxt, t2 - cur.rows, off, qs8, buf);
                have1 = 1;
            }
        }
#if LNL_RUN_PRIO
        {  // the wave ahead of its SIMD partner yields
            ++rows_done;
            prog[wave & 7u] = rows_done;
            const uint32_t other = uni(prog[(wave & 7u) ^ 4u]);
            if (rows_done > other)
                __builtin_amdgcn_s_setprio(0);
            else
                __builtin_amdgcn_s_setprio(2);
        }
#endif

        const bool st = ks < K && (sb >> 7) == t;
        const bool en = ke < K && (eb >> 7) == t;
        if (!(st || en)) {
#if defined(LNL_DIAG_NO_COMPUTE)
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] ^= x[k];
#else
            uint32_t o[32];
            lnl_net_row_x(s, x, o);
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] = o[k];
#endif
        } else if (!en) {
            // datagram ks starts in this row (after a gap row or at row 0)
            const uint32_t bs = sb & 127u;
            MaskLoop<0>::apply<false>(x, s, start_mask(bs));
            s[0] ^= lds_read_u32(fold_base + 4u * (LNL_TABLE_C_OFF + bs));  // CRC init as word 0
            ++ks;
            sb += S;
        } else {
            // datagram ke ends in this row (and maybe ks starts after it)
            const uint32_t be = eb & 127u;
            uint32_t o[32], xe[32];
            MaskLoop<0>::apply<true>(x, xe, end_mask(be));
            if (st) {  // the start part first, so x dies before the network
                const uint32_t bs = sb & 127u;
                if (contiguous) {
#pragma unroll
                    for (int w = 0; w < 32; ++w) x[w] ^= xe[w];
                } else {
                    MaskLoop<0>::apply<false>(x, x, start_mask(bs));
                }
                x[0] ^= lds_read_u32(fold_base + 4u * (LNL_TABLE_C_OFF + bs));
                ++ks;
                sb += S;
            }
            lnl_net_row_x(s, xe, o);
            if (st) {
#pragma unroll
                for (int w = 0; w < 32; ++w) s[w] = x[w];
            }
            uint32_t f[32];
            lnl_fold_level1(o, f);
            if ((ke & 1u) == 0u) {
#pragma unroll
                for (int k = 0; k < 32; ++k) P[k] = f[k];
                eprev = 127u - be;
            } else {
                uint32_t ra, rb;
                lnl_fold_pair(P, f, ra, rb);
                a.out[dl + ke - 1u] = final_map(fold_base, eprev, ra);
                a.out[dl + ke] = final_map(fold_base, 127u - be, rb);
            }
            ++ke;
            eb += S;
        }

        ++step;
        if (++t == cur.rows) {
            wb += nw;
            if (!has_nxt) break;
            cur = nxt;
            has_nxt = wb + nw < a.nb;
            if (has_nxt) nxt = run_batch(a, wb + nw);
            t = 0;
            ks = ke = 0;
            sb = cur.ph;
            eb = cur.ph + L - 1u;
            dl = cur.d0 + lane * a.q;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

hipError_t launch_crc32c_run(const RunArgs& a, int grid, hipStream_t stream) {
    hipLaunchKernelGGL(crc32c_run_kernel, dim3(grid), dim3(kRunThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
