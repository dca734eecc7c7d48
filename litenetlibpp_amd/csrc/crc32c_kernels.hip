// crc32c_kernels.hip -- batched CRC-32C over UDP datagrams for gfx950 (MI355X).
//
// One wavefront owns a BATCH of 64 datagrams, one per lane.  Every datagram is
// processed as the 128-byte-aligned memory lines it touches (see
// crc32c_bitslice.h for the algebra): the wave streams lines HBM -> LDS with
// global_load_lds_dwordx4 (LDS-DMA, no VGPR staging), each lane reads its own
// row back with 8 x ds_read_b128 -- 32 words that ARE the bit-sliced state
// input (stream j = bit j of every word, no transpose) -- and runs one
// generated XOR network (V = A V ^ X) -- ~165 VALU ops per 128 bytes, no
// tables in the row loop, no bank conflicts, no MFMA (CRC is a GF(2)
// polynomial remainder, not a dense contraction).  After the last row a
// 5-level bit-sliced tree folds the 32 streams, two nibble-table lookups map
// the result back to a CRC register and undo the line padding, and each lane
// stores one uint32.
//
// Why lines: a row that straddles two 128-byte lines makes the LDS-DMA fetch
// both lines (measured: 2^20 x 1408 B rows 128-B aligned 250 us, the same
// shifted by 4..64 bytes 280 us; with nt loads 223 us vs 400 us).  Rows are
// therefore the aligned lines themselves; whole 16-byte pieces of a
// datagram's first/last line that lie outside it are fetched from a zero line
// instead, and each lane masks the one partial piece at either end.  A
// 128-byte-aligned line never crosses a page, so reading the whole first/last
// line of a datagram is always safe even at the ends of the caller's buffer
// (those bytes are read, never written, and masked).
//
// Memory pipeline per wave: two 8 KiB LDS row buffers; row s+2 is issued as
// soon as row s has been read into registers, so two rows (16 KiB) per wave and
// 128 KiB per CU (8 waves) are in flight while the wave computes.  Each glds
// wave-instruction moves 8 datagrams x 1 line; the LDS image is XOR-swizzled
// on the SOURCE address (slot = piece ^ ((row>>1)&7)) so that the per-lane
// ds_read_b128 of a whole row is bank-conflict free.
//
// LDS reads are inline asm (8 x ds_read_b128 + lgkmcnt(0) in ONE statement):
// hipcc would otherwise put `s_waitcnt vmcnt(0)` in front of any LDS read that
// follows an LDS-DMA, draining the prefetched rows every step.  Row arrival is
// waited for with a counted `s_waitcnt vmcnt(8)` (exactly 8 VMEM instructions
// per row are ever issued, see issue_row).
//
// Waves are persistent (grid = min(batches, CUs x 8 waves)) and stride over
// batches, so rows of the next batch are prefetched under the current batch's
// last rows and its fold.
//
// Hot path of BASELINE configs 2-4 (fixed stride, CSR, sharded fixed stride)
// and of the batched inbound verify; boundary: include/lnl_crc32c.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device.h"
#include "crc32c_kernels.h"
#include "lnl_packet.h"
#include "crc32c_span.h"

// Build knobs (defaults are the shipped configuration):
//   LNL_GLDS_AUX   cache-policy bits of the LDS-DMA loads (0 = default, 2 = nt)
//   LNL_EDGE_AUX   the same for the first/last rows of a batch
//   LNL_DIAG_NO_COMPUTE  diagnostic build only: rows are loaded and read but the
//                  framing/network is replaced by an XOR (wrong CRCs) -- used
//                  to measure the memory pipeline's own ceiling.
#ifndef LNL_GLDS_AUX
#define LNL_GLDS_AUX 2
#endif
// cache policy of the first/last rows (the boundary line two neighbouring
// datagrams share is fetched once by each)
#ifndef LNL_EDGE_AUX
#define LNL_EDGE_AUX 0
#endif

namespace lnl {

namespace {

constexpr int kWaves = kBlockThreads / 64;  // waves per workgroup
using namespace dev;
constexpr int kLdsU4 = kWaves * 2 * kBufU4 + kFoldU4;

// Per-batch parameters.  Wave-uniform fields are kept in SGPRs (readfirstlane).
// "Compute" fields describe the lane's own datagram; "load" fields describe,
// for each of the 8 glds instructions i of a row, the datagram q = 8i + lane/8
// whose 16-byte piece this lane fetches.
struct Batch {
    uint32_t valid;      // uniform: batch exists
    uint32_t rows;       // uniform: max over lanes of T
    uint32_t max_first;  // uniform: max over lanes of `first`
    uint32_t simple;     // uniform: no idle lane
    // compute lane
    uint32_t p;      // datagram index (>= n: idle lane)
    uint32_t len;    // bytes covered by the CRC
    const uint8_t* dptr;  // the datagram's first byte (verify mode: header byte, trailing CRC at dptr + len)
    uint32_t T;      // lines the datagram touches (0: idle)
    uint32_t first;  // first real row of this lane (rows before it are virtual)
    uint32_t pad;    // bytes of the first line before the datagram
    uint32_t e;      // bytes of the last line after the datagram
    uint32_t c0;     // CRC init as the first row's word 0 (table C[pad])
    // load lanes: absolute address of row 0 (line of datagram q minus first_q
    // lines), piece included, and the framing of q:
    // first_q | head piece hp_q << 20 | tail piece tp_q << 23 | idle << 30
    uint64_t ladr[8];
    uint32_t lfirst[8];
    // uniform: every lane busy and starting at row 0 (the common case once CSR
    // batches are bucketed by line count): the only edge rows are 0 and rows-1
    uint32_t uedge;
    // load lanes, uedge batches: bit i = fetch piece of glds i on the head row,
    // bit 8 + i = on the tail row (else the zero line)
    uint32_t ebits;
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
__device__ LNL_INLINE void make_batch(const BatchArgs& a, uint32_t b, uint32_t nbatch, uint32_t nperm,
                                      uint32_t tab_base, Batch& B) {
    // Branch-free on purpose (every field written on every path keeps the
    // struct in registers).  An invalid batch (b >= nbatch) has only idle lanes.
    const uint32_t lane = __lane_id();
    B.valid = uni(b < nbatch ? 1u : 0u);
    uint64_t start;
    uint32_t len;
    const uint32_t idx = b * 64u + lane;
    const bool real = B.valid && idx < nperm;
    if (kMode != kModeFixed && a.desc) {  // uniform branch: bucketed CSR / verify
        const uint4 d = real ? a.desc[idx] : make_uint4(a.n, 0u, 0u, 0u);
        B.p = d.x;
        len = d.y;
        start = (uint64_t)d.z | ((uint64_t)d.w << 32);
    } else {
        B.p = real ? (a.perm ? a.perm[idx] : idx) : a.n;
        lane_extent<kMode>(a, B.p, start, len);
    }
    const uint64_t abs0 = (uint64_t)(uintptr_t)a.base + start;
    const uint64_t abs1 = abs0 + len - 1u;  // last byte (unused when len == 0)
    const uint32_t idle = len == 0u ? 1u : 0u;
    B.len = len;
    B.dptr = a.base + start;
    B.T = idle ? 0u : (uint32_t)((abs1 >> 7) - (abs0 >> 7)) + 1u;
    B.pad = (uint32_t)abs0 & 127u;
    B.e = 127u - ((uint32_t)abs1 & 127u);
    B.c0 = lds_read_u32(tab_base + 4u * (LNL_TABLE_C_OFF + B.pad));
    B.rows = uni(wave_max(B.T));
    B.first = B.rows - B.T;
    B.max_first = uni(wave_max(idle ? 0u : B.first));
    B.simple = uni(__any(idle) ? 0u : 1u);
    // row t of datagram q is line (abs0_q >> 7) + t - first_q
    const uint64_t row0 = ((abs0 >> 7) << 7) - ((uint64_t)B.first << 7);
    const uint32_t fl = B.first | ((B.pad >> 4) << 20) | (((127u - B.e) >> 4) << 23) | (idle << 30);
    const uint32_t sub = lane >> 3, slot = lane & 7u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t q = 8u * i + sub;
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)row0, q, 64);
        const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(row0 >> 32), q, 64);
        B.ladr[i] = (((uint64_t)hi << 32) | lo) + 16u * (slot ^ swz(q));
        B.lfirst[i] = (uint32_t)__shfl((int)fl, q, 64);
    }
    B.uedge = uni(B.simple && B.max_first == 0u ? 1u : 0u);
    uint32_t eb = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t f = B.lfirst[i];
        const uint32_t piece = slot ^ swz(8u * i + sub);
        eb |= (piece >= ((f >> 20) & 7u) ? 1u : 0u) << i;
        eb |= (piece <= ((f >> 23) & 7u) ? 1u : 0u) << (8 + i);
    }
    B.ebits = eb;
}

// Issue the 8 LDS-DMA instructions that bring row t of batch B into `buf`.
// All 8 are issued unconditionally -- lanes of idle datagrams, of virtual rows
// and of whole pieces outside the datagram fetch the 16-byte zero line: the
// counted `s_waitcnt vmcnt(8)` in the main loop relies on exactly 8 VMEM
// instructions per row, and the algebra wants those bytes zero.
__device__ LNL_INLINE void issue_row(const BatchArgs& a, const Batch& B, uint32_t t, uint4* buf) {
    const uint64_t dt = (uint64_t)t << 7;
    const uint32_t lane = __lane_id();
    if (B.simple && t > B.max_first && t + 1u < B.rows) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)(B.ladr[i] + dt),
                                             (void*)(buf + 64 * i), 16, 0, LNL_GLDS_AUX);
    } else if (B.uedge) {
        // rows 0 and rows-1 of a batch whose lanes all start at row 0
        const uint32_t m = (t == 0u ? B.ebits : 0xFFu) & (t + 1u == B.rows ? (B.ebits >> 8) : 0xFFu);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t src = (m >> i) & 1u ? B.ladr[i] + dt : (uint64_t)(uintptr_t)a.dummy;
            __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)src, (void*)(buf + 64 * i), 16,
                                             0, LNL_EDGE_AUX);
        }
    } else {
        const bool last = t + 1u == B.rows;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t f = B.lfirst[i];
            const uint32_t first = f & 0xFFFFFu;
            const uint32_t piece = (lane & 7u) ^ swz(8u * i + (lane >> 3));
            const bool on = !(f & (1u << 30)) && t >= first &&
                            !(t == first && piece < ((f >> 20) & 7u)) &&
                            !(last && piece > ((f >> 23) & 7u));
            const uint64_t src = on ? B.ladr[i] + dt : (uint64_t)(uintptr_t)a.dummy;
            __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)src, (void*)(buf + 64 * i), 16,
                                             0, LNL_EDGE_AUX);
        }
    }
}

template <int kMode>
__device__ LNL_INLINE void store_result(const BatchArgs& a, const Batch& B, uint32_t crc) {
    if (B.p >= a.n) return;
    if constexpr (kMode == kModeVerify) {
        // B.len = total - 4 for datagrams of >= 5 bytes, else 0 (lane_extent,
        // bucket_of): the trailing CRC follows the covered bytes
        uint32_t ok = 0;
        if (B.len) {
            const uint8_t* tail = B.dptr + B.len;
            const uint32_t stored = (uint32_t)tail[0] | ((uint32_t)tail[1] << 8) |
                                    ((uint32_t)tail[2] << 16) | ((uint32_t)tail[3] << 24);
            ok = stored == crc;
            // inbound filter: the CRC layer passed it, now net_packet::verify()
            // on the stripped packet (net_manager.cpp:343)
            if (ok && a.filter) ok = lnl_packet_verify_hdr(B.dptr[0], B.len) ? 1u : 2u;
        }
        a.ok[B.p] = (uint8_t)ok;
        if (a.out) a.out[B.p] = crc;
    } else {
        a.out[B.p] = crc;
    }
}

template <int kMode>
__global__ __launch_bounds__(kBlockThreads, 2) void crc32c_batch_kernel(BatchArgs a) {
    __shared__ __attribute__((aligned(16))) uint4 lds[kLdsU4];
    const uint32_t lane = __lane_id();
    const uint32_t wave = uni(threadIdx.x >> 6);
    uint4* const buf_base = lds + wave * (2 * kBufU4);
    uint4* const fold_lds = lds + kWaves * 2 * kBufU4;
    const uint32_t fold_base = (uint32_t)(uintptr_t)fold_lds;

    // CSR uniform path epilogue: fold the tail contributions into out (a
    // datagram this launch computes itself has tail 0 and is not touched)
    if (a.tail_xor) {
        for (uint32_t i = blockIdx.x * kBlockThreads + threadIdx.x; i < a.xor_n; i += gridDim.x * kBlockThreads) {
            const uint32_t v = a.tail_xor[i];
            if (v) a.out[i] ^= v;
        }
    }
    // CSR span path (the span kernel combined the cross-segment heads itself
    // and zeroed the next call's overflow count): the overflow list, or the
    // whole batch when the span kernel did not take it -- [1] and [2] of its
    // control block in one load
    uint32_t nperm;
    if (a.span_ctl) {
        const uint4 c = *reinterpret_cast<const uint4*>(a.span_ctl);  // (32-byte aligned control blocks)
        const bool taken = uni(c.z) != 0u;
        nperm = taken ? uni(c.y) : a.n;
        if (!taken) {
            a.perm = nullptr;
            a.perm_n = nullptr;
        }
    } else {
        // entries to process: n, or a device-side count of perm entries
        nperm = a.perm_n ? uni(*a.perm_n) : a.n;
    }
    const uint32_t nbatch = (nperm + 63u) >> 6;
    if (blockIdx.x * kWaves >= nbatch) return;  // whole workgroup idle (before the barrier)

    // stage the tables (before any LDS-DMA is in flight)
    {
        const uint4* g = reinterpret_cast<const uint4*>(a.fold);
        for (int i = threadIdx.x; i < kFoldU4; i += kBlockThreads) fold_lds[i] = g[i];
        __syncthreads();
    }
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
    make_batch<kMode>(a, b, nbatch, nperm, fold_base, cur);
    if (!cur.valid) return;
    make_batch<kMode>(a, b + nw, nbatch, nperm, fold_base, nxt);

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
            make_batch<kMode>(a, b + nw, nbatch, nperm, fold_base, nxt);
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
        // framing of the datagrams' first/last rows: the partial 16-byte piece
        // at either end is masked in LDS (whole pieces outside the datagram
        // were fetched from the zero line)
        const bool edge = t <= cur.max_first || t + 1u == cur.rows;
        const bool head = edge && t == cur.first && cur.T != 0u;
#if !defined(LNL_MASK_IN_REGS)
        if (edge) {
            uint32_t hp, tp, hm[4], tm[4];
            lnl_piece_masks(head, t + 1u == cur.rows, cur.pad, cur.e, hp, tp, hm, tm);
            const uint32_t sw = swz(lane);
            // lanes with no partial piece on this row patch piece 0 with all-ones
            const uint32_t rowb = rad[0] - 16u * sw;  // piece 0 sits at slot sw
            const uint32_t hsel = hp < 8u ? hp : 0u, tsel = tp < 8u ? tp : 0u;
            uint32_t hmk[4], tmk[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                hmk[w] = hp < 8u ? hm[w] : 0xFFFFFFFFu;
                tmk[w] = tp < 8u ? tm[w] : 0xFFFFFFFFu;
            }
            const uint32_t haddr = rowb + 16u * (hsel ^ sw), taddr = rowb + 16u * (tsel ^ sw);
            if (odd) {
                patch_piece<kBufBytes>(haddr, hmk);
                patch_piece<kBufBytes>(taddr, tmk);
            } else {
                patch_piece<0>(haddr, hmk);
                patch_piece<0>(taddr, tmk);
            }
        }
#endif
        uint32_t x[32];
        if (odd)
            read_row<kBufBytes>(rad, x);
        else
            read_row<0>(rad, x);
#if defined(LNL_MASK_IN_REGS)
        if (edge) {
            uint32_t hp, tp, hm[4], tm[4];
            lnl_piece_masks(head, t + 1u == cur.rows, cur.pad, cur.e, hp, tp, hm, tm);
            lnl_mask_row(x, hp, tp, hm, tm);
        }
#endif
        if (edge) x[0] ^= head ? cur.c0 : 0u;  // CRC init, as the first row's word 0
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

#if defined(LNL_DIAG_NO_COMPUTE)
#pragma unroll
        for (int k = 0; k < 32; ++k) s[k] ^= x[k];
#else
        uint32_t o[32];
        lnl_net_row_x(s, x, o);
#pragma unroll
        for (int k = 0; k < 32; ++k) s[k] = o[k];
#endif

        ++step;
        if (++t == cur.rows) {
            uint32_t r = lnl_fold_tree(s);
            r = fold_apply_lds(fold_base + 512u * lnl_table_b(cur.e), r);
            r = fold_apply_lds(fold_base + 512u * lnl_table_a(cur.e), r);
            store_result<kMode>(a, cur, cur.T ? ~r : 0u);
#pragma unroll
            for (int k = 0; k < 32; ++k) s[k] = 0;
            t = 0;
            b += nw;
            cur = nxt;
            if (!cur.valid) break;
            make_batch<kMode>(a, b + nw, nbatch, nperm, fold_base, nxt);
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
