// crc32c_csr.hip -- CSR batches (config 3) as UNIFORM line-count batches whose
// shared boundary lines are fetched once.
//
// The any-layout batch kernel (crc32c_kernels.hip) gives a lane one datagram
// and fetches every line the datagram touches.  In a packed CSR batch the line
// where datagram i ends is the line where i+1 starts, so ~1 line per datagram
// (config 3: 7.04 M row slots for 6.0 M distinct lines) is fetched twice -- and
// the kernel is bound by row slots (measured: a zero-line slot costs about
// what an HBM slot does).  Here the shared line is fetched ONCE, by the lane of
// datagram i+1 (its first row), and split there by linearity:
//
//   * the state after i's last row is A V' ^ X_tail (V': after i's last fully
//     owned line, X_tail: the first k = pad(i+1) bytes of the shared line);
//   * the fold, the matrix A (= L^-1 step^1024 L) and the final map are
//     linear and A commutes with the fold (both are conjugates of powers of
//     step), so CRC(i) = ~F_e(A fold(V')) ^ F_e(fold(X_tail)), F_e = the final
//     map for the e = 128 - k bytes after i in that line;
//   * lane i ("drop") stops one line early and writes ~F_e(A fold(V')) to
//     out[i]; lane i+1 ("take") fetches the whole shared line, moves its first
//     k bytes into a second state, folds it and writes F_e(fold(X_tail)) to
//     tail[i]; the epilogue XORs tail into out.
//
// A datagram shares its last line when it touches >= 2 lines (its init word
// then sits in a row it fetches itself), the next datagram is non-empty, starts
// mid-line, and neither is an overflow datagram (> kCsrMaxRows lines).
//
// Plan pre-pass (two kernels over the offsets): key = fetched lines
// (T - drop, 1..kCsrMaxRows).  Datagrams are grouped by key into batches of 64
// padded with idle entries, so every batch is UNIFORM: all lanes start at row
// 0 and end at row R-1 together (no leading zero rows, no wave max), and the
// framing work happens only on rows 0 and R-1, for the whole wave at once.
// Empty datagrams get CRC 0 from the pre-pass; overflow datagrams go to the
// batch kernel (perm list), whose launch also applies the tail XOR.
//
// Memory pipeline (LDS-DMA rows, 2 x 8 KiB buffers per wave, counted vmcnt,
// inline-asm LDS reads) as in crc32c_kernels.hip / crc32c_device.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"
#include "crc32c_kernels.h"

// cache policy of the middle rows / of rows 0 and R-1 (0 default, 2 nt)
#ifndef LNL_CSR_AUX
#define LNL_CSR_AUX 2
#endif
#ifndef LNL_CSR_EDGE_AUX
#define LNL_CSR_EDGE_AUX 0
#endif

namespace lnl {

namespace {

using namespace dev;

constexpr int kPlanThreads = 256;
constexpr int kPlanPerThread = 4;
constexpr uint32_t kPlanPerBlock = kPlanThreads * kPlanPerThread;

// ---- plan ---------------------------------------------------------------

struct Dg {
    uint32_t len;   // bytes
    uint32_t T;     // 128-byte lines touched (0: empty)
    uint32_t pad;   // offset of the first byte in its first line
    uint32_t be;    // offset of the last byte in its last line
    uint64_t line;  // first line, counted from base's line
};

__device__ inline Dg dg_of(const CsrPlanArgs& a, uint32_t i) {
    const uint64_t s = a.off[i] - a.off0, e = a.off[i + 1] - a.off0;
    Dg d;
    d.len = (uint32_t)(e - s);
    const uint64_t b0 = (uint64_t)(uintptr_t)a.base;
    const uint64_t abs0 = b0 + s, abs1 = abs0 + d.len - 1u;
    d.T = d.len ? (uint32_t)((abs1 >> 7) - (abs0 >> 7)) + 1u : 0u;
    if (d.len > (uint32_t)(kCsrMaxRows + 1) * 128u) d.T = kCsrMaxRows + 1;  // (no 32-bit overflow)
    d.pad = (uint32_t)abs0 & 127u;
    d.be = (uint32_t)abs1 & 127u;
    d.line = (abs0 >> 7) - (b0 >> 7);
    return d;
}

// too long for a uniform batch, or beyond the kernel's 32-bit line offsets
__device__ inline bool dg_ovf(const Dg& d) { return d.T > kCsrMaxRows || d.line >= kCsrMaxLine; }

// datagram a (followed by b) hands its last line to b
__device__ inline bool dg_share(const Dg& a, const Dg& b) {
    return a.T >= 2u && !dg_ovf(a) && b.len != 0u && !dg_ovf(b) && b.pad != 0u;
}

struct DgPlan {
    Dg d;
    uint32_t key;   // fetched lines; 0: not in a uniform batch (empty / overflow)
    uint32_t take;  // fetches the previous datagram's tail
    uint32_t drop;  // leaves its last line to the next datagram
};

__device__ inline DgPlan plan_of(const CsrPlanArgs& a, uint32_t i) {
    DgPlan P;
    P.d = dg_of(a, i);
    P.drop = 0;
    P.take = 0;
    if (i + 1u < a.n) P.drop = dg_share(P.d, dg_of(a, i + 1u)) ? 1u : 0u;
    if (i > 0u) P.take = dg_share(dg_of(a, i - 1u), P.d) ? 1u : 0u;
    P.key = (P.d.T == 0u || dg_ovf(P.d)) ? 0u : P.d.T - P.drop;
    return P;
}

__global__ __launch_bounds__(kPlanThreads) void csr_plan_count_kernel(CsrPlanArgs a) {
    constexpr int kW = kPlanThreads / 64;
    __shared__ uint32_t hist[kW][kBuckets];
    __shared__ uint32_t novf, ovf_base;
    for (int k = threadIdx.x; k < kW * kBuckets; k += kPlanThreads) (&hist[0][0])[k] = 0;
    if (threadIdx.x == 0) novf = 0;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * kPlanPerBlock + threadIdx.x;
    uint32_t key[kPlanPerThread], oslot[kPlanPerThread];
#pragma unroll
    for (int j = 0; j < kPlanPerThread; ++j) {
        const uint32_t i = i0 + j * kPlanThreads;
        key[j] = kBuckets;
        oslot[j] = 0xFFFFFFFFu;
        if (i < a.n) {
            const DgPlan P = plan_of(a, i);
            if (!P.drop) a.tail[i] = 0u;          // no tail contribution for i
            if (P.d.T == 0u) a.out[i] = 0u;       // CRC-32C of zero bytes
            if (P.key) key[j] = P.key;
            else if (P.d.T) oslot[j] = atomicAdd(&novf, 1u);  // overflow
        }
    }
    uint32_t* h = hist[threadIdx.x >> 6];
#pragma unroll
    for (int j = 0; j < kPlanPerThread; ++j)
        if (key[j] < kBuckets) atomicAdd(&h[key[j]], 1u);
    __syncthreads();
    if (threadIdx.x < kBuckets) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kW; ++w) c += hist[w][threadIdx.x];
        if (c) atomicAdd(&a.counts[(blockIdx.x % kCounterCopies) * kBuckets + threadIdx.x], c);
    }
    if (threadIdx.x == 0) ovf_base = novf ? atomicAdd(&a.ctl[1], novf) : 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPlanPerThread; ++j)
        if (oslot[j] != 0xFFFFFFFFu) a.ovf[ovf_base + oslot[j]] = i0 + j * kPlanThreads;
}

__global__ __launch_bounds__(kPlanThreads) void csr_plan_scatter_kernel(CsrPlanArgs a) {
    __shared__ uint32_t hist[kBuckets], base[kBuckets], tot[kBuckets], part[kBuckets], bb[kBuckets + 1];
    const uint32_t copy = blockIdx.x % kCounterCopies;
    if (threadIdx.x < kBuckets) {
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
    if (threadIdx.x == 0) {  // first batch of each key (keys padded to whole batches)
        uint32_t nb = 0;
        for (int k = 0; k < kBuckets; ++k) {
            bb[k] = nb;
            nb += (tot[k] + 63u) >> 6;
        }
        bb[kBuckets] = nb;
        if (blockIdx.x == 0) a.ctl[0] = nb;
    }
    const uint32_t i0 = blockIdx.x * kPlanPerBlock + threadIdx.x;
    uint32_t key[kPlanPerThread], rank[kPlanPerThread];
    uint4 d[kPlanPerThread];
#pragma unroll
    for (int j = 0; j < kPlanPerThread; ++j) {
        const uint32_t i = i0 + j * kPlanThreads;
        key[j] = 0;
        if (i < a.n) {
            const DgPlan P = plan_of(a, i);
            key[j] = P.key;
            d[j] = make_uint4(i, (uint32_t)P.d.line,
                              P.d.pad | (P.d.be << 8) | (P.take << 16) | (P.drop << 17) | (P.key << 20), 0u);
        }
    }
#pragma unroll
    for (int j = 0; j < kPlanPerThread; ++j) rank[j] = key[j] ? atomicAdd(&hist[key[j]], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x < kBuckets) {
        const uint32_t h = hist[threadIdx.x];
        base[threadIdx.x] = 64u * bb[threadIdx.x] + part[threadIdx.x] +
                            (h ? atomicAdd(&a.fill[copy * kBuckets + threadIdx.x], h) : 0u);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPlanPerThread; ++j)
        if (key[j]) a.desc[base[key[j]] + rank[j]] = d[j];
    if (blockIdx.x == 0) {  // idle entries padding every key to whole batches
        for (int k = 1; k < kBuckets; ++k) {
            const uint32_t pad = ((tot[k] + 63u) & ~63u) - tot[k];
            if (threadIdx.x < pad)
                a.desc[64u * bb[k] + tot[k] + threadIdx.x] = make_uint4(0xFFFFFFFFu, 0u, (uint32_t)k << 20, 0u);
        }
    }
}

// ---- uniform batch kernel -----------------------------------------------

// One 512-thread workgroup per CU (8 waves, 2 per SIMD): one copy of the
// tables per CU leaves LDS room for two 1 KiB descriptor slots per wave.
constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kAU4 = 32;    // the matrix A as 8 nibble tables (128 words)
constexpr int kDescU4 = 64;  // one batch's descriptors
constexpr int kLdsU4 = kWaves * 2 * kBufU4 + kFoldU4 + kAU4 + kWaves * 2 * kDescU4;  // 160,768 B

struct CBatch {
    uint32_t valid;     // uniform
    uint32_t R;         // uniform: rows (fetched lines per lane)
    uint32_t full;      // uniform: no idle lane
    uint32_t any_take;  // uniform
    // compute lane: datagram, framing pad | be << 8 | take << 16 | drop << 17 | idle << 18
    uint32_t p, fr;
    // load lanes: byte offset (from base's line) of row 0 of datagram
    // q = 8i + lane/8, plus this lane's piece
    uint32_t lofs[8];
    uint32_t m;  // bit i: glds i fetches on row 0; bit 8+i: on row R-1; bit 16+i: on other rows
};
__device__ LNL_INLINE uint32_t f_pad(uint32_t fr) { return fr & 127u; }
__device__ LNL_INLINE uint32_t f_be(uint32_t fr) { return (fr >> 8) & 127u; }
__device__ LNL_INLINE bool f_take(uint32_t fr) { return (fr >> 16) & 1u; }
__device__ LNL_INLINE bool f_drop(uint32_t fr) { return (fr >> 17) & 1u; }
__device__ LNL_INLINE bool f_idle(uint32_t fr) { return (fr >> 18) & 1u; }

// Descriptors of batch b -> LDS slot (one LDS-DMA instruction; no-op past the end).
__device__ LNL_INLINE void desc_dma(const CsrArgs& a, uint32_t b, uint32_t nb, uint4* slot) {
    if (b < nb)
        __builtin_amdgcn_global_load_lds((const void*)(a.desc + 64u * b + __lane_id()), (void*)slot, 16, 0, 0);
}

// Batch b from its descriptors in LDS slot `slot_addr` (already arrived).
__device__ LNL_INLINE void make_cbatch(uint32_t b, uint32_t nb, uint32_t slot_addr, CBatch& B) {
    const uint32_t lane = __lane_id();
    B.valid = uni(b < nb ? 1u : 0u);
    uint4 d = make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
    if (B.valid) {
        const u32x4 v = lds_read_piece(slot_addr + 16u * lane);
        d = make_uint4(v.x, v.y, v.z, v.w);
    }
    B.p = d.x;
    const uint32_t idle = d.x == 0xFFFFFFFFu ? 1u : 0u;
    B.R = uni((d.z >> 20) & 63u);  // lane 0 is never padding
    B.fr = (d.z & (idle ? 0xFF7Fu : 0x3FFFFu)) | (idle << 18);  // (idle: no take)
    B.full = uni(__any(idle) ? 0u : 1u);
    B.any_take = uni(__any(f_take(B.fr)) ? 1u : 0u);
    const uint32_t row0 = d.y << 7;
    const uint32_t sub = lane >> 3, slot = lane & 7u;
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t q = 8u * i + sub;
        const uint32_t f = (uint32_t)__shfl((int)B.fr, q, 64);
        const uint32_t pc = slot ^ swz(q);
        B.lofs[i] = (uint32_t)__shfl((int)row0, q, 64) + 16u * pc;
        const bool busy = !((f >> 18) & 1u);
        const bool head_ok = ((f >> 16) & 1u) || pc >= ((f & 127u) >> 4);
        const bool tail_ok = ((f >> 17) & 1u) || pc <= (((f >> 8) & 127u) >> 4);
        m |= (busy && head_ok && (B.R > 1u || tail_ok) ? 1u : 0u) << i;
        m |= (busy && tail_ok ? 1u : 0u) << (8 + i);
        m |= (busy ? 1u : 0u) << (16 + i);
    }
    B.m = m;
}

// row t: line base (SGPR) + t * 128 + the lane's 32-bit offset
__device__ LNL_INLINE void issue_crow(const CsrArgs& a, const CBatch& B, uint32_t t, uint4* buf) {
    const uint8_t* row = (const uint8_t*)(((uintptr_t)a.base & ~(uintptr_t)127) + ((uintptr_t)t << 7));
    if (B.full && t > 0u && t + 1u < B.R) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(row + B.lofs[i]), (void*)(buf + 64 * i), 16, 0,
                                             LNL_CSR_AUX);
    } else {
        const uint32_t mb = (t == 0u ? B.m : (t + 1u == B.R ? B.m >> 8 : B.m >> 16)) & 0xFFu;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint8_t* src = (mb >> i) & 1u ? row + B.lofs[i] : a.dummy;
            __builtin_amdgcn_global_load_lds((const void*)src, (void*)(buf + 64 * i), 16, 0, LNL_CSR_EDGE_AUX);
        }
    }
}

// bytes 4w..4w+3 of a row: mask of the bytes at row offsets < n (n in 0..128)
__device__ LNL_INLINE uint32_t below_mask(int32_t w, uint32_t n) { return lnl_low_bits(8 * (int32_t)n - 32 * w); }

__device__ LNL_INLINE uint32_t final_map(uint32_t fold_base, uint32_t e, uint32_t r) {
    r = fold_apply_lds(fold_base + 512u * lnl_table_b(e), r);
    return fold_apply_lds(fold_base + 512u * lnl_table_a(e), r);
}

__global__ __launch_bounds__(kThreads, 2) void crc32c_csr_kernel(CsrArgs a) {
    __shared__ __attribute__((aligned(16))) uint4 lds[kLdsU4];
    const uint32_t lane = __lane_id();
    const uint32_t wave = uni(threadIdx.x >> 6);
    uint4* const buf_base = lds + wave * (2 * kBufU4);
    uint4* const fold_lds = lds + kWaves * 2 * kBufU4;
    uint4* const a_lds = fold_lds + kFoldU4;
    uint4* const slot_lds = a_lds + kAU4 + wave * (2 * kDescU4);  // this wave's 2 descriptor slots
    const uint32_t fold_base = (uint32_t)(uintptr_t)fold_lds;
    const uint32_t a_base = (uint32_t)(uintptr_t)a_lds;

    const uint32_t nb = uni(a.ctl[0]);
    if (blockIdx.x * kWaves >= nb) return;  // whole workgroup idle (before the barrier)
    {
        const uint4* g = reinterpret_cast<const uint4*>(a.fold);
        for (int i = threadIdx.x; i < kFoldU4; i += kThreads) fold_lds[i] = g[i];
        const uint4* ga = reinterpret_cast<const uint4*>(a.amat);
        for (int i = threadIdx.x; i < kAU4; i += kThreads) a_lds[i] = ga[i];
        __syncthreads();
    }
    const uint32_t gw = blockIdx.x * kWaves + wave;
    const uint32_t nw = gridDim.x * kWaves;

    // LDS address of piece k of this lane's row: r0 ^ 16k (see crc32c_run.hip)
    const uint32_t r0 = (uint32_t)(uintptr_t)(buf_base + lane * kRowU4) | (16u * swz(lane));

    // Descriptor pipeline: cur and nxt live in registers, the descriptors of
    // the batch after nxt are in flight (LDS-DMA into slot ps) -- so a batch
    // switch never waits on a global load with rows in flight.  A slot is
    // safe to read once the counted row wait two steps after its DMA has
    // passed (`dready`); short batches that switch sooner wait for it.
    const uint32_t slot0 = (uint32_t)(uintptr_t)slot_lds, slot1 = slot0 + 16u * kDescU4;
    CBatch cur, nxt;
    uint32_t b = gw;
    desc_dma(a, b, nb, slot_lds);
    desc_dma(a, b + nw, nb, slot_lds + kDescU4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    make_cbatch(b, nb, slot0, cur);
    if (!cur.valid) return;
    make_cbatch(b + nw, nb, slot1, nxt);
    uint32_t ps = 0, dready = 0;  // slot of the batch in flight; step from which it has arrived
    desc_dma(a, b + 2u * nw, nb, slot_lds);

    // Row pipeline (as in crc32c_kernels.hip): `step` counts computed rows,
    // row `step` lives in buffer step & 1; have0 / have1: rows step / step+1
    // have been issued.  Rows are issued two steps ahead, into nxt when cur
    // ends; a row of the batch after nxt is issued on demand.  R >= 1 always.
    uint32_t step = 0, t = 0;
    uint32_t have0 = 1, have1 = 0;
    issue_crow(a, cur, 0, buf_base);
    if (cur.R > 1u) {
        issue_crow(a, cur, 1, buf_base + kBufU4);
        have1 = 1;
    } else if (nxt.valid) {
        issue_crow(a, nxt, 0, buf_base + kBufU4);
        have1 = 1;
    }
    uint32_t s[32];

    while (true) {
        const uint32_t odd = uni(step & 1u);
        uint4* const buf = buf_base + odd * kBufU4;
        if (!have0) {
            issue_crow(a, cur, t, buf);
            have1 = 0;  // drain everything below
        }
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
            uint32_t have2 = 0;
            if (t2 < cur.R) {
                issue_crow(a, cur, t2, buf);
                have2 = 1;
            } else if (nxt.valid && t2 - cur.R < nxt.R) {
                issue_crow(a, nxt, t2 - cur.R, buf);
                have2 = 1;
            }
            have0 = have1;
            have1 = have2;
        }
        const bool last = t + 1u == cur.R;
#if defined(LNL_CSR_DIAG_MEMONLY)  // diagnostic build: rows loaded and read, no framing / network / fold
#pragma unroll
        for (int k = 0; k < 32; ++k) s[k] = (t == 0u ? 0u : s[k]) ^ x[k];
        ++step;
        if (last) {
            if (!f_idle(cur.fr)) a.out[cur.p] = s[0] ^ s[31];
#else
        if (last) {  // the datagram's end (lanes that keep their last line)
#pragma unroll
            for (int w = 0; w < 32; ++w) x[w] &= f_drop(cur.fr) ? 0xFFFFFFFFu : below_mask(w, f_be(cur.fr) + 1u);
        }
        if (t == 0u) {
            // first row: the state is zero, so it becomes the masked row itself;
            // take lanes first move the previous datagram's tail bytes out
            const uint32_t pad = f_pad(cur.fr);
            if (cur.any_take) {
                const bool take = f_take(cur.fr);
                uint32_t xt[32];
#pragma unroll
                for (int w = 0; w < 32; ++w) {
                    const uint32_t lo = below_mask(w, pad);
                    xt[w] = take ? x[w] & lo : 0u;
                    x[w] &= ~lo;
                }
                const uint32_t r = final_map(fold_base, 128u - pad, lnl_fold_tree(xt));
                if (take) a.tail[cur.p - 1u] = r;
            } else {
#pragma unroll
                for (int w = 0; w < 32; ++w) x[w] &= ~below_mask(w, pad);
            }
            x[0] ^= lds_read_u32(fold_base + 4u * (LNL_TABLE_C_OFF + pad));  // CRC init, as word 0
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] = x[k];
        } else {
#if defined(LNL_DIAG_NO_COMPUTE)
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] ^= x[k];
#else
            uint32_t o[32];
            lnl_net_row_x(s, x, o);
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] = o[k];
#endif
        }
        ++step;
        if (last) {
            uint32_t r = lnl_fold_tree(s);
            const uint32_t ra = fold_apply_lds(a_base, r);  // one more (zero) line: the dropped one
            r = f_drop(cur.fr) ? ra : r;
            r = final_map(fold_base, 127u - f_be(cur.fr), r);
            if (!f_idle(cur.fr)) a.out[cur.p] = ~r;
#endif
            t = 0;
            b += nw;
            cur = nxt;
            if (!cur.valid) break;
            if (step < dready) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (short batches)
            make_cbatch(b + nw, nb, ps ? slot1 : slot0, nxt);
            desc_dma(a, b + 2u * nw, nb, slot_lds + (ps ^ 1u) * kDescU4);
            ps ^= 1u;
            dready = step + 2u;
        } else {
            ++t;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

void csr_plan_layout(CsrPlanArgs& a, uint32_t* w) {
    a.counts = w;
    a.fill = a.counts + kCounterCopies * kBuckets;
    a.ctl = a.counts + kBucketCounterWords;  // 4 words: [0] batches, [1] overflow datagrams
    a.desc = (uint4*)(a.ctl + 4);            // 16-byte aligned: kBucketCounterWords + 4 is a multiple of 4
    uint32_t* d = (uint32_t*)(a.desc + ((size_t)a.n + 64u * kBuckets));
    a.tail = d;
    a.ovf = d + a.n;
}

size_t csr_plan_scratch_words(uint32_t n) {
    return kBucketCounterWords + 4 + 4 * ((size_t)n + 64u * kBuckets) + 2 * (size_t)n;
}

hipError_t launch_csr_uniform(const CsrPlanArgs& p, const CsrArgs& c, int grid, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(p.counts, 0, (kBucketCounterWords + 4) * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const dim3 pg((p.n + kPlanPerBlock - 1) / kPlanPerBlock);
    hipLaunchKernelGGL(csr_plan_count_kernel, pg, dim3(kPlanThreads), 0, stream, p);
    hipLaunchKernelGGL(csr_plan_scatter_kernel, pg, dim3(kPlanThreads), 0, stream, p);
    hipLaunchKernelGGL(crc32c_csr_kernel, dim3(grid), dim3(kThreads), 0, stream, c);
    return hipGetLastError();
}

}  // namespace lnl
