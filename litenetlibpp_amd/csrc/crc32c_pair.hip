// crc32c_pair.hip -- CSR batches as datagram PAIRS (config 3).
//
// CSR datagrams are contiguous: datagram i ends where i+1 begins.  A lane of
// the any-layout batch kernel owns one datagram, so the line two neighbours
// share is fetched twice (+13 % HBM traffic at 64..1400 B), and every datagram
// pays a full 5-level fold.  Here a lane owns the PAIR (2j, 2j+1) = (a, b) and
// streams the lines from a's first to b's last once:
//
//  * the line where a ends and b begins is read once and split: a's part xe
//    (bytes <= a's last byte: the piece holding it AND-masked in LDS, later
//    pieces read from a zero piece) and b's part x ^ xe;
//  * a's and b's level-1 fold results are interleaved and folded together
//    (lnl_fold_pair), as in the lane-run kernel.
//
// The row schedule of a pair depends only on (Ta, Tb, shared): the lines a and
// b touch and whether they share one.  The bucket pre-pass
// (crc32c_bucket.hip) sorts pairs by that key into 64-entry-aligned groups,
// so every wave's lanes have the same schedule: which row starts a, ends a,
// starts b, ends b is WAVE-UNIFORM.  Only the byte offsets inside those rows
// are per lane (LDS patches, as in the batch kernel).  Pairs whose datagrams
// touch more than kPairMaxT lines go to the batch kernel instead.
//
// Memory pipeline: the batch kernel's (two 8 KiB LDS row buffers per wave,
// rows issued two ahead, counted vmcnt, inline-asm row reads).  Whole pieces
// outside the run (first / last row) come from the zero line.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"
#include "crc32c_kernels.h"

#ifndef LNL_PAIR_AUX
#define LNL_PAIR_AUX 2  // interior rows: nt
#endif
#ifndef LNL_PAIR_EDGE_AUX
#define LNL_PAIR_EDGE_AUX 0  // first / last row: lines shared with the neighbouring pairs
#endif

namespace lnl {

namespace {

using namespace dev;

// One 512-thread workgroup per CU (8 waves): the tables are staged once per CU,
// which leaves room for each wave's 1 KiB descriptor slot.
constexpr int kThreads = kPairThreads;
constexpr int kWaves = kThreads / 64;
constexpr int kFoldOffU4 = kWaves * 2 * kBufU4;
constexpr int kDescOffU4 = kFoldOffU4 + kFoldU4;      // 64 descriptors per wave
constexpr int kZeroU4 = kDescOffU4 + kWaves * 64;     // one zero piece
constexpr int kLdsU4 = kZeroU4 + 1;
static_assert(kLdsU4 * 16 <= 160 * 1024, "LDS");

// A batch: wave-uniform schedule + this lane's descriptor (PairArgs).
struct Pair {
    uint32_t valid;   // batch exists
    uint32_t Ta, Tb;  // lines a / b touch (0: empty)
    uint32_t shared;  // a's last line is b's first
    uint32_t steps;   // Ta + Tb: the shared line is read at two consecutive steps
    uint4 d;          // x: run's first line, y: pad_a | be_a | pad_b | be_b, z: a, w: hasb | key
    uint32_t lline[8];  // run's first line of lane q = 8i + lane/8 (glds instruction i)
};

__device__ LNL_INLINE uint32_t byte_of(uint32_t v, int k) { return (v >> (8 * k)) & 0xFFu; }

// A batch from its lanes' descriptors.  The bucket makes (Ta, Tb, shared)
// equal on every lane (padding lanes carry the group's key).
__device__ LNL_INLINE void make_pair(const uint4& d, uint32_t valid, Pair& P) {
    P.valid = valid;
    const uint32_t key = uni(d.w) >> 8;
    P.shared = key & 1u;
    P.Tb = (key >> 1) % (kPairMaxT + 1u);
    P.Ta = (key >> 1) / (kPairMaxT + 1u);
    P.steps = valid ? P.Ta + P.Tb : 0u;
    P.d = d;
    if (!valid) P.d.z = 0xFFFFFFFFu;
    const uint32_t sub = __lane_id() >> 3;
#pragma unroll
    for (int i = 0; i < 8; ++i) P.lline[i] = (uint32_t)__shfl((int)d.x, 8 * i + (int)sub, 64);
}


__device__ LNL_INLINE uint4 load_desc(const PairArgs& A, uint32_t wb, uint32_t nwb) {
    return wb < nwb ? A.desc[wb * 64u + __lane_id()] : make_uint4(0u, 0u, 0xFFFFFFFFu, 0u);
}

// The descriptors of a later batch go HBM -> the wave's LDS slot by LDS-DMA,
// issued before a step's row prefetch, so the next step's counted
// `s_waitcnt vmcnt(8)` (or any vmcnt(0)) covers them like a row; they are read
// back (asm ds_read) at the batch change.  No compiler-visible register is
// written asynchronously.
__device__ LNL_INLINE void load_desc_lds(const PairArgs& A, uint32_t wb, uint32_t nwb, uint4* slot) {
    const uint32_t idx = wb < nwb ? wb * 64u + __lane_id() : __lane_id();  // any readable entry
    __builtin_amdgcn_global_load_lds((const void*)(A.desc + idx), (void*)slot, 16, 0, 0);
}

__device__ LNL_INLINE uint4 read_desc_lds(uint32_t slot_addr) {
    const u32x4 v = lds_read_piece(slot_addr + 16u * __lane_id());
    return make_uint4(v.x, v.y, v.z, v.w);
}

// The 8 LDS-DMA instructions of step u (64 lanes' lines) into buf.  Whole
// lines always (every byte a run needs is in them; framing happens at read
// time).  Piece of glds i for this lane: slot ^ swz(8i + sub) = pc0 for even
// i, pc0 ^ 4 for odd i.  The shared line is read at steps Ta-1 and Ta; both
// fetches use the default cache policy so the second is served by L2.
__device__ LNL_INLINE void issue_pair_step(const Pair& P, uint64_t base_line, uint32_t max_line, uint32_t pc0,
                                           uint32_t u, uint4* buf) {
    const uint32_t line = u - (P.shared && u >= P.Ta ? 1u : 0u);
    const bool dflt = P.shared && (u + 1u == P.Ta || u == P.Ta);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        // a run never leaves the buffer; the clamp only guards the fetch
        const uint32_t ln = min(P.lline[i] + line, max_line);
        const uint64_t src = ((base_line + ln) << 7) + 16u * (pc0 ^ (4u * (i & 1)));
        if (dflt)
            __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)src, (void*)(buf + 64 * i), 16, 0,
                                             LNL_PAIR_EDGE_AUX);
        else
            __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)src, (void*)(buf + 64 * i), 16, 0,
                                             LNL_PAIR_AUX);
    }
}

__device__ LNL_INLINE uint32_t final_crc(uint32_t fold_base, uint32_t e, uint32_t r) {
    r = fold_apply_lds(fold_base + 512u * lnl_table_b(e), r);
    r = fold_apply_lds(fold_base + 512u * lnl_table_a(e), r);
    return ~r;
}

__device__ LNL_INLINE uint32_t init_word(uint32_t fold_base, uint32_t pad) {
    return lds_read_u32(fold_base + 4u * (LNL_TABLE_C_OFF + pad));  // C[pad]
}

// Read the lane's row keeping bytes lo..hi only: the partial pieces at either
// end AND-masked in LDS first, whole pieces outside read from the zero piece.
__device__ LNL_INLINE void read_row_framed(uint32_t rowb, uint32_t sw, uint32_t zero_addr, uint32_t lo,
                                           uint32_t hi, uint32_t* x) {
    uint32_t hp, tp, hm[4], tm[4];
    lnl_piece_masks(true, true, lo, 127u - hi, hp, tp, hm, tm);
    patch_piece<0>(rowb + 16u * (hp ^ sw), hm);
    patch_piece<0>(rowb + 16u * (tp ^ sw), tm);
    uint32_t ad[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        ad[k] = ((uint32_t)k < hp || (uint32_t)k > tp) ? zero_addr : (rowb + 16u * ((uint32_t)k ^ sw));
    read_row<0>(ad, x);
}

__global__ __launch_bounds__(kThreads, 1) void crc32c_pair_kernel(PairArgs A) {
    __shared__ __attribute__((aligned(16))) uint4 lds[kLdsU4];
    const uint32_t lane = __lane_id();
    const uint32_t wave = uni(threadIdx.x >> 6);
    uint4* const buf_base = lds + wave * (2 * kBufU4);
    uint4* const fold_lds = lds + kFoldOffU4;
    uint4* const desc_slot = lds + kDescOffU4 + wave * 64;
    const uint32_t desc_addr = (uint32_t)(uintptr_t)desc_slot;
    const uint32_t fold_base = (uint32_t)(uintptr_t)fold_lds;
    const uint32_t zero_addr = (uint32_t)(uintptr_t)(lds + kZeroU4);
    const uint32_t nwb = uni(A.ctl[0]);
    const uint32_t max_line = uni(A.ctl[3]);
    if (blockIdx.x * kWaves >= nwb) return;  // whole workgroup idle (before the barrier)
    {
        const uint4* g = reinterpret_cast<const uint4*>(A.fold);
        for (int i = threadIdx.x; i < kFoldU4; i += kThreads) fold_lds[i] = g[i];
        if (threadIdx.x == 0) lds[kZeroU4] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
    }
    const uint32_t gw = blockIdx.x * kWaves + wave;
    const uint32_t nw = gridDim.x * kWaves;
    if (gw >= nwb) return;

    const uint64_t base_line = ((uint64_t)(uintptr_t)A.base) >> 7;  // lines are indexed from here
    const uint32_t sw = swz(lane);
    const uint32_t pc0 = (lane & 7u) ^ swz(lane >> 3);
    const uint32_t row0 = (uint32_t)(uintptr_t)(buf_base + lane * kRowU4);  // lane's row, buffer 0

    Pair cur, nxt;
    uint32_t wb = gw;
    make_pair(load_desc(A, wb, nwb), 1u, cur);
    make_pair(load_desc(A, wb + nw, nwb), uni(wb + nw < nwb ? 1u : 0u), nxt);
    uint32_t raw_step = 0;  // step at which the slot's load (batch after nxt) was issued

    // step pipeline as in the batch kernel: step s lives in buffer s & 1,
    // issued two steps ahead (into the next batch near the end of this one)
    uint32_t step = 0, u = 0, have0 = 0, have1 = 0;
    uint32_t s[32], Pf[16];  // Pf: a's level-1 fold, packed (lnl_pack_level1)
#pragma unroll
    for (int k = 0; k < 32; ++k) s[k] = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) Pf[k] = 0;
    if (cur.steps > 0) {
        issue_pair_step(cur, base_line, max_line, pc0, 0, buf_base);
        have0 = 1;
        if (cur.steps > 1) {
            issue_pair_step(cur, base_line, max_line, pc0, 1, buf_base + kBufU4);
            have1 = 1;
        } else if (nxt.valid && nxt.steps > 0) {
            issue_pair_step(nxt, base_line, max_line, pc0, 0, buf_base + kBufU4);
            have1 = 1;
        }
    }

    while (true) {
        if (cur.steps == 0) {
            // every pair of this batch is two empty datagrams: CRC 0
            if (cur.d.z < A.n) {
                A.out[cur.d.z] = 0u;
                if (cur.d.w & 1u) A.out[cur.d.z + 1u] = 0u;
            }
            wb += nw;
            cur = nxt;
            if (!cur.valid) break;
            const uint4 d = load_desc(A, wb + nw, nwb);  // rare: a plain (waited) load
            make_pair(d, uni(wb + nw < nwb ? 1u : 0u), nxt);
            have0 = 0;
            have1 = 0;
            continue;
        }
        const uint32_t odd = uni(step & 1u);
        uint4* const buf = buf_base + odd * kBufU4;
        const uint32_t rowb = row0 + odd * kBufBytes;
        if (!have0) {
            issue_pair_step(cur, base_line, max_line, pc0, u, buf);
            have1 = 0;
        }
        if (have1)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

        // events of this step (wave-uniform)
        const bool inA = u < cur.Ta;
        const bool start = u == 0u || u == cur.Ta;   // a's or b's first row
        const bool end = u + 1u == cur.Ta || u + 1u == cur.steps;
        uint32_t x[32];
        if (start || end) {
            const uint32_t lo = start ? byte_of(cur.d.y, inA ? 0 : 2) : 0u;
            const uint32_t hi = end ? byte_of(cur.d.y, inA ? 1 : 3) : 127u;
            read_row_framed(rowb, sw, zero_addr, lo, hi, x);
        } else {
            uint32_t ad[8], rb = rowb;
            asm volatile("" : "+v"(rb));  // keep the address math in the loop
#pragma unroll
            for (int k = 0; k < 8; ++k) ad[k] = rb + 16u * ((uint32_t)k ^ sw);
            read_row<0>(ad, x);
        }
        if (u == 0u) {
            load_desc_lds(A, wb + 2u * nw, nwb, desc_slot);
            raw_step = step;
        }
        // prefetch step+2 into the buffer just drained
        uint32_t have2 = 0;
        {
            const uint32_t u2 = u + 2u;
            if (u2 < cur.steps) {
                issue_pair_step(cur, base_line, max_line, pc0, u2, buf);
                have2 = 1;
            } else if (nxt.valid && u2 - cur.steps < nxt.steps) {
                issue_pair_step(nxt, base_line, max_line, pc0, u2 - cur.steps, buf);
                have2 = 1;
            }
        }
        have0 = have1;
        have1 = have2;

        if (start) {
            // a fresh state: V = X, the CRC init as the row's word 0
            x[0] ^= init_word(fold_base, byte_of(cur.d.y, inA ? 0 : 2));
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] = x[k];
        } else {
            uint32_t o[32];
            lnl_net_row_x(s, x, o);
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] = o[k];
        }
        if (end) {
            // the datagram's state goes into the fold; the next datagram starts
            // fresh, so s is dead from here (zeroed to tell the compiler)
            uint32_t f[32];
            lnl_fold_level1(s, f);
            if (inA) {
                lnl_pack_level1(f, Pf);
#pragma unroll
                for (int k = 0; k < 32; ++k) f[k] = 0;
            }
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] = 0;
            if (!inA || !cur.Tb) {  // the pair is complete
                uint32_t ra, rb;
                lnl_fold_pair_packed(Pf, f, ra, rb);
                const uint32_t ca = final_crc(fold_base, 127u - byte_of(cur.d.y, 1), ra);
                const uint32_t cb = final_crc(fold_base, 127u - byte_of(cur.d.y, 3), rb);
                if (cur.d.z < A.n) {
                    A.out[cur.d.z] = cur.Ta ? ca : 0u;
                    if (cur.d.w & 1u) A.out[cur.d.z + 1u] = cur.Tb ? cb : 0u;
                }
            }
        }

        ++step;
        if (++u == cur.steps) {
            // the batch's pairs are stored: Pf is dead (zeroed so the compiler
            // knows, and so an empty a folds as zero next time)
#pragma unroll
            for (int k = 0; k < 16; ++k) Pf[k] = 0;
            u = 0;
            wb += nw;
            cur = nxt;
            if (!cur.valid) break;
            // the slot was loaded at this batch's step 0; a later step's
            // counted wait covers it unless the batch had a single step
            if (step - raw_step < 2u) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            make_pair(read_desc_lds(desc_addr), uni(wb + nw < nwb ? 1u : 0u), nxt);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

hipError_t launch_crc32c_pair(const PairArgs& a, int grid, hipStream_t stream) {
    hipLaunchKernelGGL(crc32c_pair_kernel, dim3(grid), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
