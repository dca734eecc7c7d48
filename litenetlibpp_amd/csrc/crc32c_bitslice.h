// crc32c_bitslice.h -- the per-lane algebra of the batched CRC-32C kernels.
//
// One lane owns one datagram.  The datagram is read as 128-byte ROWS that are
// the 128-byte-aligned memory lines it touches (a row straddling two lines
// would make the LDS-DMA fetch both).  A row is 32 little-endian words
// w_0..w_31.  STREAM j of a row is bit j of every word -- so the 32 streams
// are already BIT-SLICED in the words as loaded: register k holds coordinate k
// of all 32 streams, stream j in bit j.  No transpose.
//
// Algebra (register model: step(c) = (c >> 1) ^ (POLY & -(c & 1)), one bit).
// A 1 at row bit 32k + j contributes step^(1023-32k-j)(POLY) to the register
// after the row, so stream j contributes L_j(W_j) = step^(31-j) L(W_j) with
// L(e_k) = step^(992-32k)(POLY).  L is invertible (x^32 generates GF(2^32)),
// and in the basis V = L^-1(.) one row is the constant Horner step
//
//     V <- A V ^ X,   A = L^-1 step^1024 L        (X = the row's 32 words)
//
// (generated XOR network lnl_net_row_x, ~150 VALU ops per 128 bytes).  After
// the last row the register is L( sum_j B^(31-j) V_j ) with B = L^-1 step L:
// a 5-level bit-sliced fold (level l combines streams 2^l apart with
// B^(2^(l-1))) and a 32-bit gather of bit 0 of every register (lnl_fold_tree).
//
// Framing.  Rows spell 0^pad || M || 0^e: the pad bytes of the first line
// before the datagram and the e bytes of the last line after it are zero
// (whole 16-byte pieces come from a zero line, the one partial piece at each
// end is masked: lnl_piece_masks; the kernel applies the masks to the piece
// in LDS before the lane reads its row).  Leading zeros leave a raw
// CRC unchanged; trailing ones multiply it by step^(8e), undone in the final
// map.  CRC-32C's init 0xFFFFFFFF enters at the datagram's first row: a
// register value c at the start of that row equals step^(8 pad)(c) at the
// datagram start, and a register value at the start of a message is the same
// as XORing it into the message's first 32 bits -- here word 0 of the row, so
// the lane XORs c0 = step^(-8 pad)(0xFFFFFFFF) into x[0] (table C[pad]).
// Then
//
//     CRC(M) = step^(-8e)( L( fold(V) ) ) ^ 0xFFFFFFFF      (len >= 1; 0 for len 0)
//
// with step^(-8e) o L applied by two nibble-table matrix products
// (e = 16a + b: step^(-128a) o (step^(-8b) o L)), tables from
// lnl_build_tables.
//
// This file is compiled twice: by hipcc into the gfx950 kernels (LNL_XOR3 is
// then v_bitop3_b32 0x96) and by g++ into the host-side unit test that checks
// the algebra against the oracle without a GPU (tests/emu).  It has no host
// fallback role: the product's batch entry points only ever launch kernels.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define LNL_HD __host__ __device__
#else
#define LNL_HD
#endif
#define LNL_INLINE inline __attribute__((always_inline))

#if defined(__HIP_DEVICE_COMPILE__)
#define LNL_XOR3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
#else
#define LNL_XOR3(a, b, c) ((a) ^ (b) ^ (c))
#endif
#define LNL_XOR2(a, b) ((a) ^ (b))

#include "crc32c_networks.inc"

#define LNL_CRC32C_POLY 0x82F63B78u
#define LNL_ROW_BYTES 128u

// ---- tables -----------------------------------------------------------------
// Matrices are stored as 8 nibble tables of 16 words (128 words): table k,
// entry v = N(v << 4k), so N(x) = XOR_k table_k[nibble_k(x)].
//   [  0 .. 16)  TB[b] = step^(-8b) o L        (b = e & 15)
//   [ 16 .. 24)  TA[a] = step^(-128a)          (a = e >> 4)
//   then 128 words C[pad] = step^(-8 pad)(0xFFFFFFFF)
#define LNL_TABLE_MATS 24
#define LNL_TABLE_C_OFF (LNL_TABLE_MATS * 128)
#define LNL_TABLE_WORDS (LNL_TABLE_C_OFF + 128)

// n reflected CRC steps forward (n > 0) or backward (n < 0) on one register.
LNL_HD LNL_INLINE uint32_t lnl_step_bits(uint32_t c, int32_t n) {
    for (; n > 0; --n) c = (c >> 1) ^ (LNL_CRC32C_POLY & (0u - (c & 1u)));
    for (; n < 0; ++n) {  // POLY has bit 31 set: the top bit says whether it was xored
        const uint32_t top = c >> 31;
        c = ((c ^ (LNL_CRC32C_POLY & (0u - top))) << 1) | top;
    }
    return c;
}

// Matrix given by columns applied to a vector.
LNL_HD LNL_INLINE uint32_t lnl_cols_apply(const uint32_t* cols, uint32_t v) {
    uint32_t r = 0;
    for (int k = 0; k < 32; ++k)
        if ((v >> k) & 1u) r ^= cols[k];
    return r;
}

// Host-side table construction (also used by the CPU emulation test).
LNL_HD inline void lnl_build_tables(uint32_t* t) {
    uint32_t L[32];
    for (int k = 0; k < 32; ++k) L[k] = lnl_step_bits(LNL_CRC32C_POLY, 992 - 32 * k);
    for (int m = 0; m < LNL_TABLE_MATS; ++m)
        for (int k = 0; k < 8; ++k)
            for (uint32_t v = 0; v < 16; ++v) {
                const uint32_t x = v << (4 * k);
                t[m * 128 + k * 16 + v] =
                    m < 16 ? lnl_step_bits(lnl_cols_apply(L, x), -8 * m) : lnl_step_bits(x, -128 * (m - 16));
            }
    for (int pad = 0; pad < 128; ++pad) t[LNL_TABLE_C_OFF + pad] = lnl_step_bits(0xFFFFFFFFu, -8 * pad);
}

// Inverse of a 32x32 GF(2) matrix given by its columns (Gauss-Jordan).
LNL_HD inline void lnl_cols_inverse(const uint32_t* cols, uint32_t* inv) {
    uint32_t row[32], aug[32];
    for (int i = 0; i < 32; ++i) {
        uint32_t r = 0;
        for (int k = 0; k < 32; ++k) r |= ((cols[k] >> i) & 1u) << k;
        row[i] = r;
        aug[i] = 1u << i;
    }
    for (int c = 0; c < 32; ++c) {
        int p = c;
        while (!((row[p] >> c) & 1u)) ++p;
        const uint32_t tr = row[p], ta = aug[p];
        row[p] = row[c];
        aug[p] = aug[c];
        row[c] = tr;
        aug[c] = ta;
        for (int i = 0; i < 32; ++i)
            if (i != c && ((row[i] >> c) & 1u)) {
                row[i] ^= row[c];
                aug[i] ^= aug[c];
            }
    }
    for (int k = 0; k < 32; ++k) {
        uint32_t v = 0;
        for (int i = 0; i < 32; ++i) v |= ((aug[i] >> k) & 1u) << i;
        inv[k] = v;
    }
}

LNL_HD LNL_INLINE uint32_t lnl_table_b(uint32_t e) { return e & 15u; }
LNL_HD LNL_INLINE uint32_t lnl_table_a(uint32_t e) { return 16u + (e >> 4); }

// Host/emulation form of one matrix product (the kernel does the same 8
// lookups from LDS in inline asm).
LNL_HD LNL_INLINE uint32_t lnl_table_apply(const uint32_t* mat, uint32_t v) {
    uint32_t r = 0;
    for (int k = 0; k < 8; ++k) r ^= mat[k * 16 + ((v >> (4 * k)) & 15u)];
    return r;
}

// ---- framing masks --------------------------------------------------------
// Bytes b (0..3) of a word kept when d <= b (from) or b < d (below).
LNL_HD LNL_INLINE uint32_t lnl_keep_from(int32_t d) {
    return d <= 0 ? 0xFFFFFFFFu : (d >= 4 ? 0u : (0xFFFFFFFFu << (8 * d)));
}
LNL_HD LNL_INLINE uint32_t lnl_keep_below(int32_t d) {
    return d <= 0 ? 0u : (d >= 4 ? 0xFFFFFFFFu : ((1u << (8 * d)) - 1u));
}

// Word masks of the partial pieces of a datagram's first / last row.  hp: the
// piece holding the first byte (8: no head on this row), hm[w] keeps its
// bytes >= pad; tp: the piece holding the last byte (8: no tail), tm[w] keeps
// its bytes <= 127 - e.  Whole pieces outside the datagram are zero already
// (the kernel fetches the zero line for them).
LNL_HD LNL_INLINE void lnl_piece_masks(bool head, bool tail, uint32_t pad, uint32_t e, uint32_t& hp,
                                       uint32_t& tp, uint32_t* hm, uint32_t* tm) {
    hp = head ? (pad >> 4) : 8u;
    tp = tail ? ((127u - e) >> 4) : 8u;
    const int32_t hlo = (int32_t)(pad & 15u);
    const int32_t thi = (int32_t)((127u - e) & 15u) + 1;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        hm[w] = lnl_keep_from(hlo - 4 * w);
        tm[w] = lnl_keep_below(thi - 4 * w);
    }
}

LNL_HD LNL_INLINE void lnl_mask_row(uint32_t* x, uint32_t hp, uint32_t tp, const uint32_t* hm,
                                    const uint32_t* tm) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t piece = (uint32_t)k >> 2;
        const uint32_t a = piece == hp ? hm[k & 3] : 0xFFFFFFFFu;
        const uint32_t b = piece == tp ? tm[k & 3] : 0xFFFFFFFFu;
        x[k] &= a & b;
    }
}

// Word w of a row (bytes 4w .. 4w+3): keep the bytes at row offsets <= be /
// >= bs.  (The lane-run kernel's datagram end / start masks; be, bs are
// wave-uniform there, so these fold to scalar code.)
// (Written as a clamped 64-bit shift: a handful of scalar ops per word.)
LNL_HD LNL_INLINE uint32_t lnl_low_bits(int32_t n) {  // n clamped to [0, 32] low bits set
    const int32_t c = n < 0 ? 0 : (n > 32 ? 32 : n);
    return (uint32_t)((1ull << c) - 1ull);
}
LNL_HD LNL_INLINE uint32_t lnl_word_keep_le(int32_t w, uint32_t be) {
    return lnl_low_bits(8 * (int32_t)be + 8 - 32 * w);
}
LNL_HD LNL_INLINE uint32_t lnl_word_keep_ge(int32_t w, uint32_t bs) {
    return ~lnl_low_bits(8 * (int32_t)bs - 32 * w);
}

// ---- fold ---------------------------------------------------------------
// sum_j B^(31-j) V_j gathered into one word (bit k = coordinate k).  s is
// destroyed.
LNL_HD LNL_INLINE uint32_t lnl_fold_tree(uint32_t* s) {
    uint32_t z[32];
    lnl_net_fold1(s, z);  // bit 2i: B V_2i ^ V_2i+1
    lnl_net_fold2(z, s);  // bit 4i
    lnl_net_fold4(s, z);  // bit 8i
    lnl_net_fold8(z, s);  // bit 16i
    lnl_net_fold16(s, z);  // bit 0: sum_j B^(31-j) V_j
    uint32_t r = 0;
#pragma unroll
    for (int k = 31; k >= 0; --k) r = (r << 1) | (z[k] & 1u);
    return r;
}

// The fold split for PAIRS of datagrams (lane-run kernel): level 1 per
// datagram, then the two level-1 results -- meaningful at even bits only --
// are interleaved (a at bits 2i, b at bits 2i+1) and levels 2..5 run once for
// both: every level is the same shift-and-network on all bit positions, so a's
// streams end at bit 0 and b's at bit 1.  ra / rb equal lnl_fold_tree of each.
LNL_HD LNL_INLINE void lnl_fold_level1(const uint32_t* s, uint32_t* f) {
    lnl_net_fold1(s, f);
}

LNL_HD LNL_INLINE void lnl_fold_pair(const uint32_t* a, const uint32_t* b, uint32_t& ra, uint32_t& rb) {
    uint32_t s[32], z[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) s[k] = (a[k] & 0x55555555u) | ((b[k] << 1) & 0xAAAAAAAAu);
    lnl_net_fold2(s, z);
    lnl_net_fold4(z, s);
    lnl_net_fold8(s, z);
    lnl_net_fold16(z, s);
    uint32_t x = 0, y = 0;
#pragma unroll
    for (int k = 31; k >= 0; --k) {
        x = (x << 1) | (s[k] & 1u);
        y = (y << 1) | ((s[k] >> 1) & 1u);
    }
    ra = x;
    rb = y;
}

// A level-1 fold result is meaningful at even bits only, so two of its words
// fit in one: p[m] = f[2m] (even bits) | f[2m+1] (moved to the odd bits).
// The pair kernel keeps the first datagram's result like this (16 registers,
// not 32) until its partner's is ready.
LNL_HD LNL_INLINE void lnl_pack_level1(const uint32_t* f, uint32_t* p) {
#pragma unroll
    for (int m = 0; m < 16; ++m) p[m] = (f[2 * m] & 0x55555555u) | ((f[2 * m + 1] << 1) & 0xAAAAAAAAu);
}

LNL_HD LNL_INLINE void lnl_fold_pair_packed(const uint32_t* p, const uint32_t* b, uint32_t& ra, uint32_t& rb) {
    uint32_t a[32];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        a[2 * m] = p[m] & 0x55555555u;
        a[2 * m + 1] = (p[m] >> 1) & 0x55555555u;
    }
    lnl_fold_pair(a, b, ra, rb);
}
