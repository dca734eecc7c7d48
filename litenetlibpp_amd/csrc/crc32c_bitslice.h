// crc32c_bitslice.h -- the per-lane algebra of the batched CRC-32C kernels.
//
// One lane owns one datagram.  The datagram is read as 128-byte ROWS that are
// the 128-byte-aligned memory lines it touches (line alignment is what the
// HBM path wants: a row that straddles two lines costs a second line fetch).
// Word j (bytes 4j..4j+3) of every row belongs to STREAM j, j = 0..31.  The
// 32 streams are processed together BIT-SLICED: register S[i] holds bit i of
// the CRC register of all 32 streams, stream j in bit j.  Per row:
//
//     X = transpose32(row words)            X[k] bit j = word j bit k
//     X &= keep, X ^= inv                   (first / last rows only)
//     S = M_128(S) ^ X                      (generated XOR network)
//
// where M_n is the CRC-32C "advance over n zero bytes" operator (linear over
// GF(2); the networks are in crc32c_networks.inc).  The masks zero the `pad`
// bytes of the first line that precede the datagram and the `e` bytes of the
// last line that follow it, so the rows spell 0^pad || M || 0^e.  Leading
// zeros do not change a raw (init 0) CRC; trailing ones multiply it by
// M_e.  After the last row, with T rows, stream s holds
// Q_s = sum_t M_128^(T-1-t) w_{s,t} and
//
//     raw(M) = M_e^-1( M_4( sum_s M_{4(31-s)} Q_s ) ) = M_{4-e}( tree(Q) )
//
// tree(Q) is a 5-level bit-sliced fold (level l combines streams 2^l apart
// with M_{4*2^(l-1)}) followed by a 32-bit gather of bit 0 of every register;
// M_{4-e} is applied with two nibble tables (e = 16a + b:
// M_{4-e} = M_{4-b} o M_{-16a}; 24 matrices, lnl_build_fold_tables).
// CRC-32C's init 0xFFFFFFFF is applied by XORing 0xFF into the first 4 real
// bytes (valid for L >= 4; shorter datagrams use a constant), and xorout by a
// final XOR, so no per-length table is needed.
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
#define LNL_STREAMS 32

// CRC-32C of L zero bytes (init/xorout 0xFFFFFFFF) for L < 4: the final XOR
// used when the init cannot be folded into the first 4 data bytes.
LNL_HD LNL_INLINE uint32_t lnl_final_xor(uint32_t len) {
    // crc32c(0x00 * L) for L = 0..3; L >= 4 folds the init into the data.
    return len == 0 ? 0x00000000u
         : len == 1 ? 0x527D5351u
         : len == 2 ? 0xF16177D2u
         : len == 3 ? 0x6064A37Au
                    : 0xFFFFFFFFu;
}

// v_perm_b32: byte i of the result is byte sel.byte[i] of the 8-byte value
// {hi, lo} (selectors 0-3 pick bytes of lo, 4-7 bytes of hi).  Only selectors
// 0-7 are used here.
LNL_HD LNL_INLINE uint32_t lnl_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) r |= (uint32_t)((v >> (8 * ((sel >> (8 * i)) & 7u))) & 0xFFu) << (8 * i);
    return r;
#endif
}

// 32x32 bit transpose in registers: on exit a[k] bit j = (entry) a[j] bit k.
// Stages of 16 and 8 bits are byte moves (one v_perm_b32 per output word), the
// rest are shift + bit-field-insert pairs.
LNL_HD LNL_INLINE void lnl_transpose32(uint32_t* a) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {  // swap 16-bit halves: a' = [x0 x1 y0 y1], b' = [x2 x3 y2 y3]
        const uint32_t x = a[j], y = a[j + 16];
        a[j] = lnl_perm(x, y, 0x01000504u);
        a[j + 16] = lnl_perm(x, y, 0x03020706u);
    }
#pragma unroll
    for (int j0 = 0; j0 < 32; j0 += 16) {  // swap bytes: a' = [x0 y0 x2 y2], b' = [x1 y1 x3 y3]
#pragma unroll
        for (int j = j0; j < j0 + 8; ++j) {
            const uint32_t x = a[j], y = a[j + 8];
            a[j] = lnl_perm(x, y, 0x02060004u);
            a[j + 8] = lnl_perm(x, y, 0x03070105u);
        }
    }
#define LNL_TSTAGE(S, M)                                                   \
    _Pragma("unroll") for (int j0 = 0; j0 < 32; j0 += 2 * (S)) {           \
        _Pragma("unroll") for (int j = j0; j < j0 + (S); ++j) {            \
            const uint32_t x = a[j], y = a[j + (S)];                       \
            a[j] = (x & (M)) | ((y << (S)) & ~(M));                        \
            a[j + (S)] = ((x >> (S)) & (M)) | (y & ~(M));                  \
        }                                                                  \
    }
    LNL_TSTAGE(4, 0x0F0F0F0Fu)
    LNL_TSTAGE(2, 0x33333333u)
    LNL_TSTAGE(1, 0x55555555u)
#undef LNL_TSTAGE
}

// Masks for row `rel` of a datagram (rel = row index within the datagram,
// negative for the virtual rows of a lane whose datagram spans fewer lines
// than the wave's longest).  In bit-sliced form byte b of a row is stream
// b>>2, bit range 8*(b&3) .. +7, so the masks depend only on q = k>>3.
//   keep: zero the `pad` bytes before the datagram (rel == 0) and the `e`
//         bytes after it (rel == T-1); everything on virtual rows.
//   inv:  XOR the init 0xFFFFFFFF into the first four real bytes (len >= 4);
//         they spill into row 1 when pad > 124.
LNL_HD LNL_INLINE void lnl_row_masks(int32_t rel, uint32_t T, uint32_t pad, uint32_t e,
                                     uint32_t len, uint32_t* keep, uint32_t* inv) {
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        uint32_t k = 0xFFFFFFFFu, v = 0u;
        if (rel < 0) {
            k = 0u;
        } else {
            const uint32_t h = (pad + 3u - q) >> 2;  // first stream whose byte 4h+q >= pad
            if (rel == 0) {
                k = h >= 32u ? 0u : (0xFFFFFFFFu << h);
                v = (h >= 32u || len < 4u) ? 0u : (1u << h);
            } else if (rel == 1) {
                v = (h == 32u && len >= 4u) ? 1u : 0u;  // byte 128+q of the padded datagram
            }
            if ((uint32_t)rel == T - 1u) {
                // keep streams j with 4j + q <= 127 - e
                const int32_t lim = 127 - (int32_t)e - (int32_t)q;
                const uint32_t cnt = lim < 0 ? 0u : (uint32_t)(lim >> 2) + 1u;
                k &= cnt >= 32u ? 0xFFFFFFFFu : ((1u << cnt) - 1u);
            }
        }
        keep[q] = k;
        inv[q] = v;
    }
}

LNL_HD LNL_INLINE void lnl_apply_masks(uint32_t* x, const uint32_t* keep, const uint32_t* inv) {
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = (x[k] & keep[k >> 3]) ^ inv[k >> 3];
}


// ---- fold tables: R = M_{4-e}(tree) for e = 16a + b ----------------------
// 24 matrices stored as 8 nibble tables of 16 words each (128 words):
// matrix m, table k, entry v = N_m(v << 4k).  m = 0..15: M_{4-b}; m = 16..23:
// M_{-16a}.  Built on the host (lnl_build_fold_tables), staged into LDS by the
// kernel, applied with 8 lookups per matrix.
#define LNL_FOLD_TABLE_WORDS (24 * 128)

// n reflected CRC steps forward (n > 0) or backward (n < 0) on one register.
LNL_HD LNL_INLINE uint32_t lnl_step_bits(uint32_t c, int32_t n) {
    for (; n > 0; --n) c = (c >> 1) ^ (LNL_CRC32C_POLY & (0u - (c & 1u)));
    for (; n < 0; ++n) {  // POLY has bit 31 set: the top bit says whether it was xored
        const uint32_t top = c >> 31;
        c = ((c ^ (LNL_CRC32C_POLY & (0u - top))) << 1) | top;
    }
    return c;
}

LNL_HD LNL_INLINE void lnl_build_fold_tables(uint32_t* t) {
    for (int m = 0; m < 24; ++m) {
        const int32_t nbits = m < 16 ? 8 * (4 - m) : -128 * (m - 16);
        for (int k = 0; k < 8; ++k)
            for (uint32_t v = 0; v < 16; ++v) t[m * 128 + k * 16 + v] = lnl_step_bits(v << (4 * k), nbits);
    }
}

// Table index of the two matrices for tail padding e (0..127).
LNL_HD LNL_INLINE uint32_t lnl_fold_a(uint32_t e) { return 16u + (e >> 4); }
LNL_HD LNL_INLINE uint32_t lnl_fold_b(uint32_t e) { return e & 15u; }

// Host/emulation form of one matrix application (the kernel does the same 8
// lookups from LDS in inline asm).
LNL_HD LNL_INLINE uint32_t lnl_fold_apply(const uint32_t* mat, uint32_t v) {
    uint32_t r = 0;
    for (int k = 0; k < 8; ++k) r ^= mat[k * 16 + ((v >> (4 * k)) & 15u)];
    return r;
}

// Combine the 32 stream states into tree(Q) = M_4^-1(raw CRC of the padded
// rows) (see header).  s is destroyed.
LNL_HD LNL_INLINE uint32_t lnl_fold_tree(uint32_t* s) {
    uint32_t t[32], z[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) t[k] = s[k] >> 1;
    lnl_net_adv4_x(s, t, z);  // bit 2i: M_4 Q_2i ^ Q_2i+1
#pragma unroll
    for (int k = 0; k < 32; ++k) t[k] = z[k] >> 2;
    lnl_net_adv8_x(z, t, s);  // bit 4i
#pragma unroll
    for (int k = 0; k < 32; ++k) t[k] = s[k] >> 4;
    lnl_net_adv16_x(s, t, z);  // bit 8i
#pragma unroll
    for (int k = 0; k < 32; ++k) t[k] = z[k] >> 8;
    lnl_net_adv32_x(z, t, s);  // bit 16i
#pragma unroll
    for (int k = 0; k < 32; ++k) t[k] = s[k] >> 16;
    lnl_net_adv64_x(s, t, z);  // bit 0: sum_s M_{4(31-s)} Q_s
    uint32_t r = 0;
#pragma unroll
    for (int k = 31; k >= 0; --k) r = (r << 1) | (z[k] & 1u);
    return r;
}
