// crc32c_seg.hip -- CSR batches as uniform LINE SEGMENTS (config 3; also the
// batched inbound verify and the host-streaming path).
//
// CSR datagrams are contiguous: datagram i is base[P_i, P_{i+1}).  The
// any-layout batch kernel gives a lane one datagram, so it fetches the line two
// neighbours share twice (+13 % HBM traffic at 64..1400 B), needs a bucket
// pre-pass so that a wave's lanes touch equal line counts, and idles lanes on
// the rows of a wave's shorter datagrams.  This kernel reads every line of the
// batch exactly once, with every lane busy on every row:
//
//  * The batch's lines are cut into SEGMENTS of R lines (crc32c_seg.h, R about
//    lines / (64 x resident waves)).  Lane l of wave-batch w owns segment
//    g = 64 w + l and reads line g R + t at row t: the row schedule is uniform,
//    so a row's 8 LDS-DMA loads are an SGPR base plus one of two per-lane
//    offsets (the lane-run kernel's addressing).
//  * A lane checksums the datagrams that END in its segment.  At a datagram's
//    last row the lane splits the row: the piece holding the last byte is
//    AND-masked in LDS and later pieces are read from a zero piece (the
//    ending datagram's part); the rest of the row starts the next datagram
//    (CRC init as its word 0).  One row network per row either way.
//  * The datagram that runs in from the previous segment (the HEAD) is only a
//    suffix here: the lane folds it from state 0 and the previous lane folds
//    the prefix it saw (its TAIL).  CRC registers are linear, so
//        r = A^m r_tail ^ r_head      (m = the suffix's rows, A = one row)
//    and the end's owner combines the two after the row loop: the tail value
//    arrives by a lane shuffle, A^m from LDS tables of A^(2^b).  Lane 0's head
//    (prefix in the previous wave-batch) is combined by seg_fixup_kernel.
//  * Datagrams touching three or more segments, and the datagrams of a segment
//    with more than kSegTrack ends, are left to the batch kernel (overflow
//    list).  Empty datagrams get CRC 0 from the pre-pass.
//
// Memory pipeline: the batch kernel's (two 8 KiB LDS row buffers per wave, rows
// issued two ahead, counted vmcnt, inline-asm LDS reads).  One 512-thread
// workgroup per CU shares one copy of the tables.  Grid: CUs workgroups; the
// geometry (crc32c_seg.h) is derived from off[0] and off[n] by the pre-pass,
// the kernel and the fix-up alike, so the host never reads the offsets.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"
#include "crc32c_kernels.h"
#include "crc32c_seg.h"

#ifndef LNL_SEG_AUX
#define LNL_SEG_AUX 2  // nt: every line is read exactly once
#endif

namespace lnl {

namespace {

using namespace dev;

constexpr int kThreads = kSegThreads;
constexpr int kWaves = kThreads / 64;
constexpr int kFoldOffU4 = kWaves * 2 * kBufU4;
constexpr int kPowOffU4 = kFoldOffU4 + kFoldU4;
constexpr int kPowU4 = (int)kSegPowTables * 128 / 4;
constexpr int kZeroU4 = kPowOffU4 + kPowU4;
constexpr int kLdsU4 = kZeroU4 + 1;
static_assert(kLdsU4 * 16 <= 160 * 1024, "LDS");

__device__ LNL_INLINE SegGeo geometry_of(const SegArgs& a) {
    const uint64_t b = (uint64_t)(uintptr_t)a.base - a.off0;
    return seg_geometry(b + a.off[0], b + a.off[a.n], a.waves);
}

__device__ LNL_INLINE bool seg_runs(const SegGeo& G, uint32_t waves) {
    return G.NS != 0u && G.NS <= seg_max_segments(waves);
}

// ---- pre-pass ---------------------------------------------------------------

// Append `value` for the lanes with `take` (one atomic per wave).
__device__ LNL_INLINE void append(uint32_t* cnt, uint32_t* list, bool take, uint32_t value) {
    const uint64_t m = __ballot(take);
    if (m == 0ull) return;
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(cnt, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, (int)leader, 64);
    if (take) list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = value;
}

// One thread per datagram: first[g] = min{ i : P_{i+1} > g Sb } (the datagram
// holding segment g's first byte, or the first one after it) for the g in
// [ceil(P_i / Sb), ceil(P_{i+1} / Sb)), first[NS] = n; CRC 0 for empty
// datagrams; the overflow list.  A batch with more segments than the kernel
// takes goes to the batch kernel whole.
__global__ __launch_bounds__(256) void seg_prep_kernel(SegArgs a) {
    const uint64_t b = (uint64_t)(uintptr_t)a.base - a.off0;
    const SegGeo G = geometry_of(a);
    const bool whole = !seg_runs(G, a.waves);
    const uint32_t stride = gridDim.x * 256u;
    if (whole && blockIdx.x == 0 && threadIdx.x == 0) a.ctl[1] = a.n;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < a.n; i += stride) {
        if (whole) {
            a.ovf[i] = i;
            continue;
        }
        const uint64_t Pi = b + a.off[i] - G.S0, Pj = b + a.off[i + 1] - G.S0;
        if (Pi == Pj) a.out[i] = 0u;  // CRC-32C of zero bytes
        append(&a.ctl[1], a.ovf, Pj > Pi && seg_overflow(Pi, Pj, G.R), i);
        const uint32_t lo = i == 0 ? 0u : seg_ceil(Pi, G.R), hi = seg_ceil(Pj, G.R);
        for (uint32_t g = lo; g < hi; ++g) a.first[g] = i;
        if (i + 1u == a.n) a.first[G.NS] = a.n;
    }
}

// ---- segment kernel ---------------------------------------------------------

// The lane's upcoming datagram ends: 16-bit offsets from its segment's first
// byte (clamped to 0xFFFF), two per register, the front in q[0]'s low half.
struct EndQueue {
    uint32_t q[kSegQueue / 2];
    __device__ LNL_INLINE uint32_t front() const { return q[0] & 0xFFFFu; }
    __device__ LNL_INLINE void pop() {
#pragma unroll
        for (int j = 0; j + 1 < (int)kSegQueue / 2; ++j) q[j] = __builtin_amdgcn_alignbit(q[j + 1], q[j], 16);
        q[kSegQueue / 2 - 1] >>= 16;
    }
};

// The 8 LDS-DMA instructions of row t: glds i loads piece (lane & 7) of the
// row of lane q = 8 i + lane / 8, i.e. line (64 wb + q) R + t; the per-lane
// part of the address is off[i & 1] (slot swizzle as in the lane-run kernel).
__device__ LNL_INLINE void issue_seg_row(uint64_t line0, uint32_t t, const uint32_t* off, uint32_t rs8,
                                         uint4* buf) {
    const uint8_t* row = (const uint8_t*)(uintptr_t)(line0 + ((uint64_t)t << 7));
#pragma unroll
    for (int i = 0; i < 8; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(row + (uint64_t)i * rs8 + off[i & 1]), (void*)(buf + 64 * i),
                                         16, 0, LNL_SEG_AUX);
}

// The same for the batch's last wave-batches: lines past the batch's last line
// are clamped to it (in bounds; no datagram of the lane uses them).
__device__ LNL_INLINE void issue_seg_row_clamped(uint64_t line0, uint32_t t, uint32_t R, uint64_t last_line,
                                                 uint32_t pc0, uint4* buf) {
    const uint32_t sub = __lane_id() >> 3;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t a = line0 + ((uint64_t)((8u * i + sub) * R + t) << 7);
        a = a > last_line ? last_line : a;
        __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)(a + 16u * (pc0 ^ (4u * (i & 1)))),
                                         (void*)(buf + 64 * i), 16, 0, LNL_SEG_AUX);
    }
}

// xe = the lane's row up to row byte be: the piece holding be AND-masked in LDS
// (the bytes after be are not read from LDS again), later pieces from the zero
// piece.
template <uint32_t OFF>
__device__ LNL_INLINE void read_row_upto(uint32_t rowb, uint32_t sw, uint32_t zero_addr, uint32_t be,
                                         uint32_t* xe) {
    const uint32_t tp = be >> 4;
    const int32_t keep = (int32_t)(be & 15u) + 1;
    uint32_t tm[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) tm[w] = lnl_keep_below(keep - 4 * w);
    patch_piece<OFF>(rowb + 16u * (tp ^ sw), tm);
    uint32_t ad[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) ad[k] = (uint32_t)k > tp ? zero_addr - OFF : rowb + 16u * ((uint32_t)k ^ sw);
    read_row<OFF>(ad, xe);
}

__device__ LNL_INLINE uint32_t final_crc(uint32_t fold_base, uint32_t e, uint32_t r) {
    r = fold_apply_lds(fold_base + 512u * lnl_table_b(e), r);
    r = fold_apply_lds(fold_base + 512u * lnl_table_a(e), r);
    return ~r;
}

__device__ LNL_INLINE uint32_t init_word(uint32_t fold_base, uint32_t pad) {
    return lds_read_u32(fold_base + 4u * (LNL_TABLE_C_OFF + pad));  // C[pad]
}

// The fold at a datagram end.  Diagnostic build only (-DLNL_SEG_DIAG_NOFOLD):
// a 2-op stand-in (wrong CRCs), to measure what the folds cost.
__device__ LNL_INLINE uint32_t seg_fold(uint32_t* s) {
#if defined(LNL_SEG_DIAG_NOFOLD)
    return s[0] ^ s[31];
#else
    return lnl_fold_tree(s);
#endif
}

// A^m r (m < 2^kSegPowTables)
__device__ LNL_INLINE uint32_t pow_apply(uint32_t pow_base, uint32_t m, uint32_t r) {
#pragma unroll
    for (int b = 0; b < (int)kSegPowTables; ++b)
        if ((m >> b) & 1u) r = fold_apply_lds(pow_base + 512u * b, r);
    return r;
}

__global__ __launch_bounds__(kThreads, 1) void crc32c_seg_kernel(SegArgs A) {
    __shared__ __attribute__((aligned(16))) uint4 lds[kLdsU4];
    const uint32_t lane = __lane_id();
    const uint32_t wave = uni(threadIdx.x >> 6);
    uint4* const buf_base = lds + wave * (2 * kBufU4);
    const uint32_t fold_base = (uint32_t)(uintptr_t)(lds + kFoldOffU4);
    const uint32_t pow_base = (uint32_t)(uintptr_t)(lds + kPowOffU4);
    const uint32_t zero_addr = (uint32_t)(uintptr_t)(lds + kZeroU4);

    const uint64_t bsh = (uint64_t)(uintptr_t)A.base - A.off0;
    const SegGeo G = geometry_of(A);
    if (!seg_runs(G, A.waves)) return;
    const uint32_t R = G.R, NS = G.NS, Sb = R << 7;
    const uint32_t nwb = (NS + 63u) >> 6;
    if (blockIdx.x * kWaves >= nwb) return;  // whole workgroup idle (before the barrier)
    {
        const uint4* f = reinterpret_cast<const uint4*>(A.fold);
        for (int i = threadIdx.x; i < kFoldU4; i += kThreads) lds[kFoldOffU4 + i] = f[i];
        const uint4* p = reinterpret_cast<const uint4*>(A.pow);
        for (int i = threadIdx.x; i < kPowU4; i += kThreads) lds[kPowOffU4 + i] = p[i];
        if (threadIdx.x == 0) lds[kZeroU4] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
    }
    const uint32_t gw = blockIdx.x * kWaves + wave;
    const uint32_t nw = gridDim.x * kWaves;

    const uint32_t sub = lane >> 3, pc0 = (lane & 7u) ^ (sub >> 1);
    uint32_t off[2];
    off[0] = sub * Sb + 16u * pc0;
    off[1] = sub * Sb + 16u * (pc0 ^ 4u);
    const uint32_t rs8 = 8u * Sb;
    const uint32_t sw = swz(lane);
    const uint32_t rowb = (uint32_t)(uintptr_t)(buf_base + lane * kRowU4);
    const uint32_t r0 = rowb | (16u * sw);
    const uint64_t last_line = (G.S0 + G.Pn - 1u) & ~(uint64_t)127;

    for (uint32_t wb = gw; wb < nwb; wb += nw) {
        const uint64_t line0 = G.S0 + (uint64_t)wb * 64u * Sb;
        const bool clamp = line0 + 64ull * Sb - 128u > last_line;
#define LNL_SEG_ISSUE(T, BUF)                                          \
    do {                                                               \
        if (clamp)                                                     \
            issue_seg_row_clamped(line0, (T), R, last_line, pc0, BUF); \
        else                                                           \
            issue_seg_row(line0, (T), off, rs8, BUF);                  \
    } while (0)
        LNL_SEG_ISSUE(0u, buf_base);  // R >= 16: rows 0 and 1 exist
        LNL_SEG_ISSUE(1u, buf_base + kBufU4);

        // ---- this lane's datagrams --------------------------------------
        const uint32_t g = wb * 64u + lane;
        const bool live = g < NS;
        const uint64_t segbase = G.S0 + (uint64_t)g * Sb;
        uint32_t h0 = 0, h1 = 0, hp = 0;
        if (live) {
            h0 = A.first[g];
            h1 = A.first[g + 1u];
            hp = g ? A.first[g - 1u] : h0;
        }
        const uint32_t cnt = h1 - h0;  // datagrams ending here (the head included)
        const bool excess = cnt > kSegTrack;
        const bool prev_excess = h0 - hp > kSegTrack;  // the previous lane left our head to the batch kernel
        // queued ends: those of h0 .. (at most kSegTrack), then, if the lane
        // keeps them all, the end of the datagram running out of the segment
        const uint32_t E = !live ? 0u : (excess ? kSegTrack : cnt + (h1 < A.n ? 1u : 0u));
        uint64_t pv[kSegQueue + 1];
#pragma unroll
        for (int k = 0; k <= (int)kSegQueue; ++k) pv[k] = (uint32_t)k <= E && live ? A.off[h0 + k] : 0ull;
        EndQueue Q;
#pragma unroll
        for (int j = 0; j < (int)kSegQueue / 2; ++j) {
            uint32_t v[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint64_t p = bsh + pv[2 * j + 1 + h];
                v[h] = p <= segbase ? 0u : (p - segbase >= 0xFFFFull ? 0xFFFFu : (uint32_t)(p - segbase));
            }
            Q.q[j] = v[0] | (v[1] << 16);
        }
        int32_t cs;  // first byte of the current datagram, from the segment's first byte
        {
            const int64_t d = (int64_t)(bsh + pv[0]) - (int64_t)segbase;
            cs = d < -(int64_t)(2u * Sb) ? -(int32_t)(2u * Sb) : (int32_t)d;
        }
        if (live && excess) {
            // the lane checksums the first kSegTrack datagrams ending here; the
            // rest, and the one running out of the segment, go to the batch kernel
            bool tail = false;
            if (h1 < A.n) {
                const uint64_t p0 = bsh + A.off[h1] - G.S0, p1 = bsh + A.off[h1 + 1u] - G.S0;
                tail = G.S0 + p0 < segbase + Sb && p1 > p0 && !seg_overflow(p0, p1, R);
            }
            const uint32_t k0 = h0 + kSegTrack, nx = h1 - k0 + (tail ? 1u : 0u);
            const uint32_t at = atomicAdd(&A.ctl[1], nx);
            for (uint32_t k = 0; k < nx; ++k) A.ovf[at + k] = k0 + k;
        }

        uint32_t left = E, cid = h0, ce = 0u, inj = 0u;
        bool active = false, track = false, head = false;
        // the current datagram ended at ce: the next queued one (skipping empty
        // datagrams, whose CRC the pre-pass wrote)
        auto advance = [&]() {
            do {
                cs = (int32_t)ce;
                ++cid;
                head = false;
                if (left == 0u) {
                    active = false;
                    return;
                }
                ce = Q.front();
                Q.pop();
                --left;
                track = ce <= 2u * Sb;  // it starts here: overflow iff it reaches a third segment
            } while (ce == (uint32_t)cs);
        };
        if (live && cs > 0) {
            // segment 0: the bytes before the batch's first datagram end a
            // virtual untracked datagram
            active = true;
            ce = (uint32_t)cs;
            cid = h0 - 1u;
        } else if (live && left) {
            active = true;
            ce = Q.front();
            Q.pop();
            --left;
            head = cs < 0;
            track = head ? (cs >= -(int32_t)Sb && ce <= Sb && !prev_excess) : ce <= 2u * Sb;
            if (ce == (uint32_t)cs) advance();  // empty first datagram (only at the batch start)
            if (active && !head && cs == 0 && track) inj = 0xFFFFFFFFu;  // C[0]: starts at row 0, byte 0
        }

        // ---- rows ---------------------------------------------------------
        uint32_t s[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) s[k] = 0u;
        uint32_t r_head = 0u, m_head = 0u, e_head = 0u, id_head = 0u;
        bool has_head = false;
        for (uint32_t t = 0; t < R; ++t) {
            const uint32_t odd = t & 1u;
            uint4* const buf = buf_base + odd * kBufU4;
            if (t + 1u < R)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint32_t x[32];
            {
                uint32_t rad[8], rb = r0;
                asm volatile("" : "+v"(rb));  // keep the 7 XORs in the loop
#pragma unroll
                for (int k = 0; k < 8; ++k) rad[k] = rb ^ (16u * k);
                if (odd)
                    read_row<kBufBytes>(rad, x);
                else
                    read_row<0>(rad, x);
            }
            const uint32_t rowst = t << 7, rowend = rowst + 128u;
            const bool ev0 = active && ce <= rowend;
            const bool any_ev = __any(ev0);
            // v: lanes with an end in this row: the row's bytes after it (the
            // next datagrams'); the other lanes: their state after this row.
            // One array for both keeps the register count down.
            uint32_t v[32];
            uint32_t be = 0u;
            if (any_ev && ev0) {
                // the current datagram ends in this row: x keeps its bytes
                be = ce - 1u - rowst;
                uint32_t xe[32];
                if (odd)
                    read_row_upto<kBufBytes>(rowb, sw, zero_addr, be, xe);
                else
                    read_row_upto<0>(rowb, sw, zero_addr, be, xe);
#pragma unroll
                for (int w = 0; w < 32; ++w) {
                    v[w] = x[w] ^ xe[w];
                    x[w] = xe[w];
                }
            }
            // the row is in registers: prefetch row t+2 into its buffer
            if (t + 2u < R) LNL_SEG_ISSUE(t + 2u, buf);
            x[0] ^= inj;  // CRC init of a datagram starting at this row's byte 0
            inj = 0u;
            uint32_t o[32];
            lnl_net_row_x(s, x, o);
            if (!any_ev) {
#pragma unroll
                for (int k = 0; k < 32; ++k) s[k] = o[k];
                continue;
            }
            uint32_t ini = 0u;
            if (ev0) {
                if (track) {
                    const uint32_t r = seg_fold(o);
                    if (head) {
                        r_head = r;
                        m_head = t + 1u;
                        e_head = 127u - be;
                        id_head = cid;
                        has_head = true;
                    } else {
                        A.out[cid] = final_crc(fold_base, 127u - be, r);
                    }
                }
                advance();
                ini = active && track && cs < (int32_t)rowend ? init_word(fold_base, (uint32_t)cs - rowst) : 0u;
            } else {
#pragma unroll
                for (int k = 0; k < 32; ++k) v[k] = o[k];
            }
            // datagrams that start and end inside this row
            bool ev = ev0 && active && ce <= rowend;
            while (__any(ev)) {
                if (ev) {
                    const uint32_t be2 = ce - 1u - rowst;
                    uint32_t xe[32];
#pragma unroll
                    for (int w = 0; w < 32; ++w) {
                        const uint32_t m = lnl_word_keep_le(w, be2);
                        xe[w] = v[w] & m;
                        v[w] &= ~m;
                    }
                    xe[0] ^= ini;
                    if (track) A.out[cid] = final_crc(fold_base, 127u - be2, seg_fold(xe));
                    advance();
                    ini = active && track && cs < (int32_t)rowend ? init_word(fold_base, (uint32_t)cs - rowst) : 0u;
                    ev = active && ce <= rowend;
                }
            }
            if (ev0) {
                // the state of the datagram now open after this row
                if (active && cs < (int32_t)rowend) {
                    v[0] ^= ini;
                } else {
#pragma unroll
                    for (int k = 0; k < 32; ++k) v[k] = 0u;
                    inj = active && track && cs == (int32_t)rowend ? 0xFFFFFFFFu : 0u;  // starts at the next row
                }
            }
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] = v[k];
        }
#undef LNL_SEG_ISSUE

        // ---- head / tail ------------------------------------------------------
        // the datagram still open at the segment's end is the next lane's head
        uint32_t r_tail;
        {
            uint32_t f[32];
#pragma unroll
            for (int k = 0; k < 32; ++k) f[k] = s[k];
            r_tail = lnl_fold_tree(f);
        }
        const uint32_t prev = __shfl_up(r_tail, 1u, 64);
        if (lane == 0u) {
            // the head's prefix is the previous wave-batch's lane 63: fix-up kernel
            A.fix[wb] = make_uint4(r_head, m_head | (e_head << 8), id_head, has_head ? 1u : 0u);
        } else if (has_head) {
            A.out[id_head] = final_crc(fold_base, e_head, pow_apply(pow_base, m_head, prev) ^ r_head);
        }
        if (lane == 63u) A.carry[wb] = r_tail;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- fix-up -----------------------------------------------------------------
// Lane 0's head of wave-batch w (prefix = wave-batch w-1's lane-63 tail).  One
// thread per wave-batch; tables staged in LDS.
__global__ __launch_bounds__(256) void seg_fixup_kernel(SegArgs a) {
    __shared__ uint32_t tab[LNL_TABLE_WORDS + kSegPowTables * 128];
    const SegGeo G = geometry_of(a);
    if (!seg_runs(G, a.waves)) return;
    const uint32_t nwb = (G.NS + 63u) >> 6;
    if (blockIdx.x * 256u >= nwb) return;
    for (uint32_t i = threadIdx.x; i < LNL_TABLE_WORDS; i += 256u) tab[i] = a.fold[i];
    for (uint32_t i = threadIdx.x; i < kSegPowTables * 128u; i += 256u) tab[LNL_TABLE_WORDS + i] = a.pow[i];
    __syncthreads();
    const uint32_t w = blockIdx.x * 256u + threadIdx.x;
    if (w == 0u || w >= nwb) return;
    const uint4 f = a.fix[w];
    if (!f.w) return;
    uint32_t r = a.carry[w - 1u];
    const uint32_t m = f.y & 0xFFu, e = (f.y >> 8) & 0xFFu;
    for (uint32_t b = 0; b < kSegPowTables; ++b)
        if ((m >> b) & 1u) r = lnl_table_apply(tab + LNL_TABLE_WORDS + 128u * b, r);
    r ^= f.x;
    r = lnl_table_apply(tab + 128u * lnl_table_b(e), r);
    r = lnl_table_apply(tab + 128u * lnl_table_a(e), r);
    a.out[f.z] = ~r;
}

}  // namespace

size_t seg_scratch_words(uint32_t n, uint32_t waves) {
    const size_t ns = seg_max_segments(waves), nb = ns / 64;
    size_t w = 4 + (ns + 1) + n + nb;
    w = (w + 3) & ~(size_t)3;  // fix[] is 16-byte aligned
    return w + 4 * nb;
}

void seg_scratch_layout(SegArgs& a, uint32_t* s) {
    const size_t ns = seg_max_segments(a.waves), nb = ns / 64;
    a.ctl = s;
    a.first = s + 4;
    a.ovf = a.first + ns + 1;
    a.carry = a.ovf + a.n;
    size_t w = 4 + (ns + 1) + a.n + nb;
    w = (w + 3) & ~(size_t)3;
    a.fix = reinterpret_cast<uint4*>(s + w);
}

hipError_t launch_seg(const SegArgs& a, int grid, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(a.ctl, 0, 4 * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const uint32_t blocks = (a.n + 255u) / 256u;
    const uint32_t prep = blocks < 8192u ? blocks : 8192u;
    hipLaunchKernelGGL(seg_prep_kernel, dim3(prep), dim3(256), 0, stream, a);
    hipLaunchKernelGGL(crc32c_seg_kernel, dim3(grid), dim3(kThreads), 0, stream, a);
    const uint32_t nb = seg_max_segments(a.waves) / 64u;
    hipLaunchKernelGGL(seg_fixup_kernel, dim3((nb + 255u) / 256u), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
