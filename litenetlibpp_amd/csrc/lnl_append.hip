// lnl_append.hip -- the outbound CRC-32C layer for a device-resident burst
// (lnl_crc32c_append_csr_dev, include/lnl_crc32c.h): datagram i of a CSR burst
// is written to dst + (off[i] - off[0]) + 4 i as payload || LE32(crc_i), the
// wire form net_manager::send_raw puts on the socket with the layer on
// (/root/reference/src/lnl/net_manager.cpp:515-521).
//
// The product (LNL_APPEND_MODE 0): the CSR CRC pass (crc32c_span.hip) into
// crc[], then append_copy_kernel below -- 32 lanes per datagram, whole 16-byte
// destination chunks, up to three chunk loads in flight per lane.
//
// Experiments build only (tools/kvariants.py app_1pass*, app_team): the layer
// in ONE pass over the payload (crc32c_append.h has the algebra and the
// ownership rule).  A team of 32 lanes takes one datagram; lane q loads the
// 16 source bytes of destination chunks V0 + 16 v, v = q, q + 32, ... (a
// dwordx4 + dword at any byte shift, aligned with v_alignbyte), stores the
// chunks that lie inside the payload straight from those registers, and
// folds the same bytes into its CRC register: slicing-by-2 from LDS tables
// laid out one bank per lane, a Horner step of 512 bytes between its pieces.
// The team then shifts each lane's register to the datagram's end (one
// nibble-table product per lane, its own table), XORs the 32 registers
// together, and writes the chunks that hold the CRC -- whole 16-byte stores,
// the next datagram's first bytes included, whenever it knows all 16 -- and,
// only where a chunk is shared with a datagram of < 12 bytes or lies at the
// burst's edges, single bytes.  One 1024-thread workgroup per CU (the tables
// take 104 KiB of LDS).  Parity-green, and 752-845 us per config-3 call
// against the two passes' 467: its per-datagram work runs on all 32 lanes
// at 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_append.h"
#include "crc32c_device.h"
#include "crc32c_kernels.h"

#ifndef LNL_APPEND_MODE
#define LNL_APPEND_MODE 0  // 0: CSR CRC pass + the copy kernel (the product); experiments build only:
                           // 1 one pass (the team computes the CRCs), 2 CSR CRC pass + the team copy
#endif

namespace lnl {

namespace {

using dev::u32x4;

#define LNL_G LNL_GLOBAL  // crc32c_device.h

struct __attribute__((packed, aligned(4))) U4a {  // 16 bytes at a 4-byte aligned address
    uint32_t x, y, z, w;
};

#ifndef LNL_APPEND_THREADS
#define LNL_APPEND_THREADS 1024
#endif
[[maybe_unused]] constexpr int kThreads = LNL_APPEND_THREADS;  // the one-pass form's workgroup
#ifndef LNL_APPEND_GROUP
#define LNL_APPEND_GROUP 3  // pieces per lane loaded before any is folded (3: a 1,536-byte datagram at once)
#endif
constexpr uint32_t kGroup = LNL_APPEND_GROUP;

// 16-byte chunk store (asm: the compiler then keeps the loop rolled and the
// wave reaches its next loads sooner)
__device__ LNL_INLINE void store16(uint64_t a, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(a), "v"(u32x4{x, y, z, w}) : "memory");
}

// The N source dwords from the aligned dword holding byte sa on, zero where a
// dword lies outside [lo, hi) (the 128-byte lines the burst's bytes touch: a
// kernel may read there, include/lnl_crc32c.h).  Only the bursts' first and
// last datagrams ever need the guarded form.
template <int N>
__device__ LNL_INLINE void load_dwords(uint64_t sa, uint64_t lo, uint64_t hi, uint32_t* d) {
    const uint64_t ab = sa & ~(uint64_t)3;
    if (ab >= lo && ab + 4u * N <= hi) {
        const U4a v = *LNL_G(const U4a, ab);
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
#pragma unroll
        for (int j = 4; j < N; ++j) d[j] = *LNL_G(const uint32_t, ab + 4u * j);
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const uint64_t a = ab + 4u * j;
            d[j] = (a >= lo && a + 4u <= hi) ? *LNL_G(const uint32_t, a) : 0u;
        }
    }
}

// bytes kept of the 4 at [4 m, 4 m + 4) of a piece whose payload is [lo, hi)
[[maybe_unused]] __device__ LNL_INLINE uint32_t keep_word(int32_t lo, int32_t hi, uint32_t m) {
    auto low = [](int32_t b) -> uint32_t { return b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : (1u << (8 * b)) - 1u); };
    return low(hi - 4 * (int32_t)m) & ~low(lo - 4 * (int32_t)m);
}

#ifndef LNL_APPEND_COPY_THREADS
#define LNL_APPEND_COPY_THREADS 256
#endif
#ifndef LNL_APPEND_COPY_WGS
#define LNL_APPEND_COPY_WGS 8  // copy kernel: workgroups per CU (persistent grid)
#endif
[[maybe_unused]] constexpr int kCopyTeamThreads = LNL_APPEND_COPY_THREADS;

// CRC: the one-pass form (the team computes each datagram's CRC from the
// pieces it copies; LDS tables); otherwise the copy after the CSR CRC pass
// (a.crc in), the same pieces, ownership rule and tail-chunk assembly.
template <bool CRC, int THREADS>
__global__ __launch_bounds__(THREADS, CRC ? 1 : 2) void append_team_kernel(AppendArgs a) {
    constexpr uint32_t kTeamsPerWg = THREADS / kAppTeam;
    __shared__ __attribute__((aligned(16))) uint32_t T[CRC ? kAppTabWords : 4];
    if constexpr (CRC) {
        for (uint32_t i = threadIdx.x; i < kAppTabWords / 4; i += THREADS)
            reinterpret_cast<uint4*>(T)[i] = reinterpret_cast<const uint4*>(a.tab)[i];
        __syncthreads();
    }

    const uint32_t q = threadIdx.x % kAppTeam;  // lane within the team = bank of its table reads
    const uint32_t copy = q % kAppRepl;
    const uint32_t team = blockIdx.x * kTeamsPerWg + threadIdx.x / kAppTeam;
    const uint32_t nteams = gridDim.x * kTeamsPerWg;
    const uint32_t n = a.n;
    const uint64_t o0 = a.off[0];
    const uint64_t dstb = (uint64_t)(uintptr_t)a.dst, srcb = (uint64_t)(uintptr_t)a.base - a.off0;
    const uint64_t lo = (srcb + o0) & ~(uint64_t)127, hi = (srcb + a.off[n] + 127u) & ~(uint64_t)127;

    // the lane algebra on the LDS tables (crc32c_append.h)
    auto t2 = [&](uint32_t r, uint32_t h) -> uint32_t {
        const uint32_t x = r ^ h;
        return (r >> 16) ^ T[kAppT2 + (x & 255u) * kAppRepl + copy] ^
               T[kAppT2 + (256u + ((x >> 8) & 255u)) * kAppRepl + copy];
    };
    auto nib = [&](uint32_t base, uint32_t stride, uint32_t col, uint32_t v) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) r ^= T[base + (k * 16u + ((v >> (4 * k)) & 15u)) * stride + col];
        return r;
    };

    // A datagram's geometry, from off[i - 1 .. i + 2] (fetched one datagram
    // ahead of its pieces' loads, which go out one datagram ahead of its CRC)
    struct Dg {
        AppGeo g;
        uint64_t delta;  // destination - source of every payload byte
        uint64_t P0p;    // previous datagram's P0 (has_prev only)
        uint64_t P1n;    // next datagram's payload end (has_next only)
        uint64_t nload;  // pieces loaded: the payload's, then through the tail chunks (ct, ct + 16)
        uint32_t sh;     // source byte shift of every piece
        uint32_t t;      // piece index of the first tail chunk ct = P1 & ~15
        uint32_t crc;    // (copy form)
        bool has_prev, has_next, nonempty;
    };
    uint64_t f0 = 0, f1 = 0, f2 = 0, f3 = 0;
    uint32_t fc = 0;  // (copy form) the datagram's CRC from the CSR pass
    auto fetch = [&](uint32_t i) {
        f0 = a.off[i ? i - 1u : 0u];
        f1 = a.off[i];
        f2 = a.off[i + 1u];
        f3 = a.off[i + 2u <= n ? i + 2u : n];
        if constexpr (!CRC) fc = a.crc[i];
    };
    auto make = [&](uint32_t i) -> Dg {
        Dg D;
        const uint64_t P0 = dstb + (f1 - o0) + 4ull * i;
        D.g = lnl_app_geo(P0, f2 - f1);
        D.delta = P0 - (srcb + f1);
        D.P0p = P0 - 4u - (f1 - f0);
        D.P1n = D.g.P2 + (f3 - f2);
        D.has_prev = i > 0u;
        D.has_next = i + 1u < n;
        D.nonempty = f2 != f1;
        D.sh = (uint32_t)((D.g.V0 - D.delta) & 3u);
        D.t = (uint32_t)(((D.g.P1 & ~(uint64_t)15) - D.g.V0) >> 4);
        D.nload = D.g.nv > (uint64_t)D.t + 2u ? D.g.nv : (uint64_t)D.t + 2u;
        D.crc = fc;
        return D;
    };
    uint32_t d[kGroup][5];  // raw source dwords of the lane's pieces of one group
    auto issue = [&](const Dg& D, uint64_t vb) {
#pragma unroll
        for (uint32_t j = 0; j < kGroup; ++j) {
            const uint64_t v = vb + kAppTeam * j + q;
            if (v < D.nload) load_dwords<5>(D.g.V0 + 16u * v - D.delta, lo, hi, d[j]);
        }
    };

    Dg cur{};
    if (team < n) {
        fetch(team);
        cur = make(team);
        issue(cur, 0);
        if (team + nteams < n) fetch(team + nteams);
    }
    for (uint32_t i = team; i < n; i += nteams) {
        const AppGeo& g = cur.g;

        // ---- pieces: copy + lane CRC; the tail chunks' source words kept --------
        uint32_t acc = 0, vlast = 0;
        bool has = false;
        uint32_t A[5] = {0u, 0u, 0u, 0u, 0u};  // this lane's tail chunk, if it holds one (crc32c_append.h)
        uint32_t tc = 0xFFFFFFFFu;             // ... its piece index
        uint32_t carry_w3 = 0;                 // word 3 of the piece before this group's first (lane 0's view)
        for (uint64_t vb = 0; vb < cur.nload; vb += kAppTeam * kGroup) {
            if (vb) issue(cur, vb);  // (datagrams over 1.5 KiB: the later groups load in place)
            uint32_t w[kGroup][4], pw3[kGroup];
#pragma unroll
            for (uint32_t j = 0; j < kGroup; ++j)
#pragma unroll
                for (int m = 0; m < 4; ++m) w[j][m] = __builtin_amdgcn_alignbyte(d[j][m + 1], d[j][m], cur.sh);
            // word 3 of the previous piece: lane q - 1's, or lane 31's of the previous slot
#pragma unroll
            for (uint32_t j = 0; j < kGroup; ++j) pw3[j] = (uint32_t)__shfl((int)w[j][3], (int)((q + 31u) & 31u), 32);
            const uint32_t next_carry = (uint32_t)__shfl((int)w[kGroup - 1][3], 31, 32);
#pragma unroll
            for (uint32_t j = kGroup - 1; j > 0; --j)
                if (q == 0u) pw3[j] = pw3[j - 1];
            if (q == 0u) pw3[0] = carry_w3;
            carry_w3 = next_carry;
#pragma unroll
            for (uint32_t j = 0; j < kGroup; ++j) {
                const uint64_t v = vb + kAppTeam * j + q;
                if (v == cur.t || v == (uint64_t)cur.t + 1u) {  // a tail chunk: its 20 source bytes
                    A[0] = pw3[j];
                    A[1] = w[j][0];
                    A[2] = w[j][1];
                    A[3] = w[j][2];
                    A[4] = w[j][3];
                    tc = (uint32_t)v;
                }
                if (v >= g.nv) continue;
                uint32_t p[4] = {w[j][0], w[j][1], w[j][2], w[j][3]};
                const uint64_t c = g.V0 + 16u * v;
                if (c >= g.P0 && c + 16u <= g.P1) store16(c, p[0], p[1], p[2], p[3]);  // a payload chunk it owns
                if constexpr (!CRC) continue;
                const int32_t plo = (int32_t)((int64_t)g.P0 - (int64_t)c), phi = (int32_t)((int64_t)g.P1 - (int64_t)c);
                if (plo > 0 || phi < 16) {  // first / last piece: only the payload's bytes count
#pragma unroll
                    for (uint32_t m = 0; m < 4; ++m) p[m] &= keep_word(plo, phi < 16 ? phi : 16, m);
                }
                if (v == 0) p[0] ^= T[kAppC + g.pad];  // the CRC init, placed at P0
                uint32_t r = 0;
#if LNL_APP_SLICE16
#pragma unroll
                for (uint32_t b = 0; b < 16; ++b) r ^= T[kAppT2 + b * 256u + ((p[b >> 2] >> (8 * (b & 3))) & 255u)];
#else
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    r = t2(r, p[m] & 0xFFFFu);
                    r = t2(r, p[m] >> 16);
                }
#endif
                acc = has ? nib(kAppS512, kAppRepl, copy, acc) ^ r : r;
                has = true;
                vlast = (uint32_t)v;
            }
        }
        const Dg D = cur;
        // ---- the next datagram's first pieces go out now, under this one's combine
        if (i + nteams < n) {
            cur = make(i + nteams);
            issue(cur, 0);
            if (i + 2u * nteams < n) fetch(i + 2u * nteams);
        }

        // ---- team combine: each register shifted to the payload's end, XORed
        uint32_t crc = D.crc;
        if constexpr (CRC) {
            uint32_t x = has ? nib(kAppM, 32u, (uint32_t)(D.g.nv - 1u - vlast), acc) : 0u;
#pragma unroll
            for (int k = 16; k >= 1; k >>= 1) x ^= (uint32_t)__shfl_xor((int)x, k, 64);
            crc = D.nonempty ? ~nib(kAppTB + D.g.Z * 128u, 1u, 0u, x) : 0u;
            if (a.crc && q == 0u) a.crc[i] = crc;
        }

        // ---- the chunks holding the CRC, whole when the owner knows all 16 bytes
        // (by the lanes that hold their pieces)
        if (tc != 0xFFFFFFFFu) {
            const uint64_t c = D.g.V0 + 16u * tc;
            if (c >= D.g.P0 && c < D.g.P2 && lnl_app_full_own(c, D.g.P2, D.has_next, D.P1n)) {
                uint32_t o[4];
#pragma unroll
                for (uint32_t m = 0; m < 4; ++m)
                    o[m] = lnl_app_tail_word(A, m, (int64_t)D.g.P1 - (int64_t)(c + 4u * m),
                                             (int64_t)D.g.P2 - (int64_t)(c + 4u * m), crc);
                store16(c, o[0], o[1], o[2], o[3]);
            }
        }
        const AppGeo& gg = D.g;
        const uint64_t delta = D.delta, P0p = D.P0p, P1n = D.P1n;
        const bool has_prev = D.has_prev, has_next = D.has_next;
        const uint64_t ct = gg.P1 & ~(uint64_t)15;
        // ---- single bytes: the head chunk's and the tail's, of chunks not stored whole
        const uint64_t hc = gg.P0 & ~(uint64_t)15;
        const uint64_t tb = ct > gg.P0 ? ct : gg.P0;
        for (uint32_t k = q; k < 36u; k += kAppTeam) {
            const uint64_t xb = k < 16u ? gg.P0 + k : tb + (k - 16u);
            bool want = xb < gg.P2;
            if (k < 16u) want = want && hc < gg.P0 && xb < hc + 16u;
            else want = want && !(hc < gg.P0 && xb < hc + 16u);  // (the head candidates took it)
            want = want && !lnl_app_byte_in_full_chunk(xb, gg.P0, gg.P1, gg.P2, has_prev, P0p, has_next, P1n);
            if (want) {
                const uint8_t v = xb < gg.P1 ? *LNL_G(const uint8_t, xb - delta)
                                             : (uint8_t)(crc >> (8u * (uint32_t)(xb - gg.P1)));
                *LNL_G(uint8_t, xb) = v;
            }
        }
    }
}

#if LNL_APPEND_MODE == 0
// ---- the product: the copy kernel after the CSR CRC pass ------------------------
// A team of 32 lanes per datagram writes its whole 16-byte destination chunks
// from a dwordx4 + dword source load (v_alignbyte to any byte shift); the
// head chunk and the tail (payload remainder + CRC), which share chunks with
// the neighbouring datagrams, go one byte per lane.  Each lane issues the
// loads of up to kCopyU chunks before it stores any (round 3 issued one, then
// stored it: one memory round trip per 512 bytes of a datagram).  20-odd
// VGPRs, 8 waves per SIMD: the one-pass and team-copy kernels above hold more
// state per lane and lose on occupancy.
#ifndef LNL_APPEND_COPY_U
#define LNL_APPEND_COPY_U 3  // chunk loads in flight per lane (1: round 3's kernel)
#endif
constexpr uint32_t kCopyU = LNL_APPEND_COPY_U;
#ifndef LNL_APPEND_COPY_DPP
#define LNL_APPEND_COPY_DPP 0  // 1: aligned source chunks, the next lane's by DPP (experiment: parity-green,
                               // 499 vs 466 us per config-3 call -- the unaligned loads are not what bounds the copy)
#endif
constexpr int kCopyThreads = 256;
__device__ inline uint8_t out_byte(uint64_t x, uint64_t P1, uint64_t delta, uint32_t crc) {
    return x < P1 ? *LNL_G(const uint8_t, x - delta) : (uint8_t)(crc >> (8u * (uint32_t)(x - P1)));
}
__global__ __launch_bounds__(kCopyThreads) void append_copy_kernel(AppendArgs a) {
    const uint32_t t = (blockIdx.x * kCopyThreads + threadIdx.x) / kAppTeam;
    const uint32_t nt = gridDim.x * (kCopyThreads / kAppTeam);
    const uint32_t q = threadIdx.x % kAppTeam;
    const uint64_t o0 = a.off[0];
    const uint64_t dstb = (uint64_t)(uintptr_t)a.dst, srcb = (uint64_t)(uintptr_t)a.base - a.off0;
    // the next datagram's offsets and CRC are fetched one datagram ahead
    uint64_t ns = 0, ne = 0;
    uint32_t ncrc = 0;
    if (t < a.n) {
        ns = a.off[t];
        ne = a.off[t + 1];
        ncrc = a.crc[t];
    }
    for (uint32_t i = t; i < a.n; i += nt) {
        const uint64_t s = ns, e = ne;
        const uint32_t crc = ncrc;
        if (i + nt < a.n) {
            ns = a.off[i + nt];
            ne = a.off[i + nt + 1];
            ncrc = a.crc[i + nt];
        }
        const uint64_t P0 = dstb + (s - o0) + 4ull * i, P1 = P0 + (e - s), P2 = P1 + 4u;
        const uint64_t delta = P0 - (srcb + s);
        const uint64_t c0 = (P0 + 15u) & ~(uint64_t)15, c1 = P1 & ~(uint64_t)15;
        if (c0 >= c1) {
            for (uint64_t x = P0 + q; x < P2; x += kAppTeam) *LNL_G(uint8_t, x) = out_byte(x, P1, delta, crc);
            continue;
        }
        // the head chunk [P0, c0) and the tail [c1, P2), one byte per lane,
        // loaded before the chunks so that their latency overlaps them
        const uint64_t x0 = P0 + q, x1 = c1 + q;
        const bool b0 = x0 < c0, b1 = x1 < P2;
        const uint8_t v0 = b0 ? out_byte(x0, P1, delta, crc) : 0;
        const uint8_t v1 = b1 ? out_byte(x1, P1, delta, crc) : 0;
#if LNL_APPEND_COPY_DPP
        // Experiment: every lane loads the 16-byte ALIGNED source chunk under its
        // destination chunk; the bytes past it are the next lane's chunk,
        // taken with a DPP wave shift (the team's last lane loads its own), so
        // each chunk is one aligned dwordx4 instead of an unaligned dwordx4 +
        // dword.  Lanes past the payload's end still load (their chunk holds
        // payload bytes its left neighbour needs) when it starts inside it.
        {
            const uint32_t off = (uint32_t)((c0 - delta) & 15u), kd = off >> 2, cb = off & 3u;
            const uint64_t send = srcb + e;  // one past the payload's last source byte
            for (uint64_t wb = c0 + 16ull * q; wb - 16ull * q < c1; wb += 16ull * kAppTeam * kCopyU) {
                uint32_t d[kCopyU][8];
#pragma unroll
                for (uint32_t u = 0; u < kCopyU; ++u) {
                    const uint64_t w = wb + 16ull * kAppTeam * u;
                    const uint64_t sa = (w - delta) & ~(uint64_t)15;
                    U4a va{0u, 0u, 0u, 0u};
                    if (sa < send) va = *LNL_G(const U4a, sa);
                    d[u][0] = va.x;
                    d[u][1] = va.y;
                    d[u][2] = va.z;
                    d[u][3] = va.w;
                    d[u][4] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)va.x, 0x130, 0xf, 0xf, false);  // wave_shl:1
                    d[u][5] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)va.y, 0x130, 0xf, 0xf, false);
                    d[u][6] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)va.z, 0x130, 0xf, 0xf, false);
                    d[u][7] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)va.w, 0x130, 0xf, 0xf, false);
                    if (q == kAppTeam - 1u && w < c1 && off != 0u) {  // the team's last lane: its own next chunk
                        const U4a vb = *LNL_G(const U4a, sa + 16u);
                        d[u][4] = vb.x;
                        d[u][5] = vb.y;
                        d[u][6] = vb.z;
                        d[u][7] = vb.w;
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < kCopyU; ++u) {
                    const uint64_t w = wb + 16ull * kAppTeam * u;
                    if (w < c1) {
                        uint32_t m[5];
#pragma unroll
                        for (int j = 0; j < 5; ++j) {
                            const uint32_t a0 = d[u][j], a1 = d[u][j + 1], a2 = d[u][j + 2], a3 = d[u][(j + 3) & 7];
                            m[j] = kd == 0u ? a0 : (kd == 1u ? a1 : (kd == 2u ? a2 : a3));
                        }
                        store16(w, __builtin_amdgcn_alignbyte(m[1], m[0], cb), __builtin_amdgcn_alignbyte(m[2], m[1], cb),
                                __builtin_amdgcn_alignbyte(m[3], m[2], cb), __builtin_amdgcn_alignbyte(m[4], m[3], cb));
                    }
                }
            }
        }
        if (b0) *LNL_G(uint8_t, x0) = v0;
        if (b1) *LNL_G(uint8_t, x1) = v1;
        continue;
#endif
        const uint32_t c = (uint32_t)((c0 - delta) & 3u);  // (the same for every chunk)
        for (uint64_t wb = c0 + 16ull * q; wb < c1; wb += 16ull * kAppTeam * kCopyU) {
            U4a v[kCopyU];
            uint32_t v4[kCopyU];
#pragma unroll
            for (uint32_t u = 0; u < kCopyU; ++u) {
                const uint64_t w = wb + 16ull * kAppTeam * u;
                if (w < c1) {
                    const uint64_t sw = (w - delta) & ~(uint64_t)3;
                    v[u] = *LNL_G(const U4a, sw);
                    v4[u] = c ? *LNL_G(const uint32_t, sw + 16) : 0u;  // (byte w - delta + 15: inside the payload)
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < kCopyU; ++u) {
                const uint64_t w = wb + 16ull * kAppTeam * u;
                if (w < c1)
                    store16(w, __builtin_amdgcn_alignbyte(v[u].y, v[u].x, c), __builtin_amdgcn_alignbyte(v[u].z, v[u].y, c),
                            __builtin_amdgcn_alignbyte(v[u].w, v[u].z, c), __builtin_amdgcn_alignbyte(v4[u], v[u].w, c));
            }
        }
        if (b0) *LNL_G(uint8_t, x0) = v0;
        if (b1) *LNL_G(uint8_t, x1) = v1;
    }
}
#endif

}  // namespace

bool append_two_pass() { return LNL_APPEND_MODE != 1; }

#ifndef LNL_APPEND_WGS
#define LNL_APPEND_WGS 16u  // copy kernel: workgroups per CU (teams stride over the datagrams)
#endif
hipError_t launch_append(const AppendArgs& a, int cus, hipStream_t stream) {
#if LNL_APPEND_MODE == 0
    const uint32_t per = kCopyThreads / kAppTeam;
    const uint32_t want = (a.n + per - 1) / per, cap = (uint32_t)cus * LNL_APPEND_WGS;
    hipLaunchKernelGGL(append_copy_kernel, dim3(want < cap ? (want ? want : 1) : cap), dim3(kCopyThreads), 0, stream, a);
#elif LNL_APPEND_MODE == 1
    // persistent: one workgroup per CU (LDS), teams striding over the datagrams
    const uint32_t per = kThreads / kAppTeam;
    const uint32_t want = (a.n + per - 1) / per;
    const uint32_t grid = want < (uint32_t)cus ? want : (uint32_t)cus;
    hipLaunchKernelGGL((append_team_kernel<true, kThreads>), dim3(grid ? grid : 1), dim3(kThreads), 0, stream, a);
#else  // 2
    // persistent: LNL_APPEND_COPY_WGS workgroups per CU, teams striding over the datagrams
    const uint32_t per = kCopyTeamThreads / kAppTeam;
    const uint32_t want = (a.n + per - 1) / per, cap = (uint32_t)cus * LNL_APPEND_COPY_WGS;
    hipLaunchKernelGGL((append_team_kernel<false, kCopyTeamThreads>), dim3(want < cap ? (want ? want : 1) : cap),
                       dim3(kCopyTeamThreads), 0, stream, a);
#endif
    return hipGetLastError();
}

}  // namespace lnl
