// crc32c_append.h -- the one-pass outbound layer (lnl_append.hip): algebra,
// table layout and the chunk-ownership rule, shared by the gfx950 kernel and
// the CPU emulation test (tests/emu/emu_append.cpp).
//
// The wire burst of a CSR payload burst: datagram i goes to
//   P0 = dst + (off[i] - off[0]) + 4 i,   payload [P0, P1), LE32(CRC) [P1, P2)
// (P1 = P0 + L, P2 = P1 + 4 = the next datagram's P0), the bytes
// net_manager::send_raw puts on the socket with the layer on
// (/root/reference/src/lnl/net_manager.cpp:515-521).  A team of 32 lanes takes
// one datagram, reads its payload ONCE -- 16 destination-aligned bytes per lane
// per step -- and from the same registers both stores the copy and computes
// the CRC:
//
//  * Pieces.  Piece v covers destination [V0 + 16 v, V0 + 16 v + 16), V0 =
//    P0 & ~15, v < nv = ceil((P1 - V0) / 16); lane q takes v = q, q + 32, ...
//    A piece's bytes outside the payload are zeroed and the CRC init enters as
//    C[pad] = step^(-8 pad)(0xFFFFFFFF) XORed into word 0 of piece 0 (pad =
//    P0 - V0): the register is then 0xFFFFFFFF at P0, as the span kernel's
//    rows do it.
//  * Lane CRC.  The raw CRC (register from 0) of a piece: eight slicing-by-2
//    steps r <- (r >> 16) ^ T2a[b0(r ^ h)] ^ T2b[b1(r ^ h)], h the next 16
//    bits (T2 = step^16 of a byte at either position); or (LNL_APP_SLICE16)
//    slicing-by-16, XOR_j T16_j[b_j], T16_j = step^(8 (16 - j)): one round of
//    16 independent lookups instead of a chain of eight.  A lane's pieces are
//    512 bytes apart: acc <- S512(acc) ^ raw (S512 = step^4096, nibble
//    tables).
//  * Team combine.  Lane q's acc is the register over its pieces up to its
//    last one, v_last; it still needs the 16 (nv - 1 - v_last) bytes after it:
//    M_s = step^(128 s), s = nv - 1 - v_last < 32, one nibble-table product
//    with the lane's own table.  XOR over the 32 lanes gives the register
//    over [V0, V0 + 16 nv); the Z = V0 + 16 nv - P1 zero bytes after the
//    payload come off with TB_Z = step^(-8 Z).  CRC = ~that (0 for L = 0).
//  * LDS.  Every lane-indexed table is laid out so that lane q of a 32-lane
//    group reads bank q: T2 and S512 are replicated kAppRepl times (copy
//    q % kAppRepl), the 32 M_s tables interleaved (word (k 16 + v) 32 + s).
//    TB is read by a whole team at one address (a broadcast).
//
// Ownership (every destination byte written exactly once, 16-byte stores
// wherever possible).  The 16-byte destination chunk c belongs to the
// datagram whose wire range [P0, P2) holds c's first byte.  Its owner stores
// it whole when it knows all 16 bytes: c + 16 <= P2 (its own payload and
// CRC), or c + 16 <= P1 of the next datagram (the rest is the next payload,
// read from the same contiguous source at shift delta + 4).  Otherwise every
// datagram with bytes in c stores them one by one.  A datagram whose P0 is
// not 16-byte aligned finds out the same way whether its head chunk was
// stored whole: full_head() below.  So a burst of datagrams >= 12 bytes has
// no byte stores except at its two ends.
#pragma once
#include <stdint.h>

#include "crc32c_bitslice.h"

namespace lnl {

#ifndef LNL_APP_REPL
#define LNL_APP_REPL 32  // copies of the lane-indexed tables (32: every lane of a 32-lane group its own bank)
#endif
#ifndef LNL_APP_SLICE16
#define LNL_APP_SLICE16 0  // 1: a piece's raw CRC by slicing-by-16 (16 independent lookups, one 16 KiB table set)
#endif
constexpr uint32_t kAppRepl = LNL_APP_REPL;
constexpr uint32_t kAppTeam = 32;

// table block (words)
constexpr uint32_t kAppT2 = 0;  // [t][v][copy], t = 0 (low byte), 1 (high byte); or (SLICE16) [j][v] = step^(8 (16 - j))(v)
constexpr uint32_t kAppPieceWords = LNL_APP_SLICE16 ? 16 * 256 : 2 * 256 * kAppRepl;
constexpr uint32_t kAppS512 = kAppT2 + kAppPieceWords;         // [k][v][copy]: nibble tables of step^4096
constexpr uint32_t kAppM = kAppS512 + 128 * kAppRepl;          // [k][v][s]: nibble tables of step^(128 s), s < 32
constexpr uint32_t kAppTB = kAppM + 128 * 32;                  // [Z][k][v]: step^(-8 Z), Z < 16
constexpr uint32_t kAppC = kAppTB + 16 * 128;                  // [pad] = step^(-8 pad)(0xFFFFFFFF), pad < 16
constexpr uint32_t kAppTabWords = kAppC + 16;
static_assert(kAppTabWords % 4 == 0, "the tables are copied to LDS as 16-byte pieces");

LNL_HD inline void lnl_build_append_tables(uint32_t* t) {
    for (uint32_t v = 0; v < 256; ++v) {
#if LNL_APP_SLICE16
        for (uint32_t j = 0; j < 16; ++j) t[kAppT2 + j * 256 + v] = lnl_step_bits(v, 8 * (16 - (int32_t)j));
#else
        const uint32_t lo = lnl_step_bits(v, 16), hi = lnl_step_bits(v << 8, 16);
        for (uint32_t c = 0; c < kAppRepl; ++c) {
            t[kAppT2 + (0 * 256 + v) * kAppRepl + c] = lo;
            t[kAppT2 + (1 * 256 + v) * kAppRepl + c] = hi;
        }
#endif
    }
    for (uint32_t k = 0; k < 8; ++k)
        for (uint32_t v = 0; v < 16; ++v) {
            const uint32_t x = v << (4 * k);
            const uint32_t s512 = lnl_step_bits(x, 8 * 512);
            for (uint32_t c = 0; c < kAppRepl; ++c) t[kAppS512 + (k * 16 + v) * kAppRepl + c] = s512;
            for (uint32_t s = 0; s < 32; ++s) t[kAppM + (k * 16 + v) * 32 + s] = lnl_step_bits(x, 128 * (int32_t)s);
            for (uint32_t z = 0; z < 16; ++z) t[kAppTB + z * 128 + k * 16 + v] = lnl_step_bits(x, -8 * (int32_t)z);
        }
    for (uint32_t pad = 0; pad < 16; ++pad) t[kAppC + pad] = lnl_step_bits(0xFFFFFFFFu, -8 * (int32_t)pad);
}

// ---- host / emulation forms of the lane algebra (the kernel reads the same
// tables from LDS) --------------------------------------------------------------
LNL_HD LNL_INLINE uint32_t lnl_app_t2(const uint32_t* t, uint32_t copy, uint32_t r, uint32_t h) {
    const uint32_t x = r ^ h;
    return (r >> 16) ^ t[kAppT2 + (x & 255u) * kAppRepl + copy] ^ t[kAppT2 + (256u + ((x >> 8) & 255u)) * kAppRepl + copy];
}
// raw CRC (register from 0) of a 16-byte piece w[0..3] (little-endian words)
LNL_HD LNL_INLINE uint32_t lnl_app_piece(const uint32_t* t, uint32_t copy, const uint32_t* w) {
    uint32_t r = 0;
#if LNL_APP_SLICE16
    (void)copy;
    for (uint32_t j = 0; j < 16; ++j) r ^= t[kAppT2 + j * 256 + ((w[j >> 2] >> (8 * (j & 3))) & 255u)];
#else
    for (int k = 0; k < 4; ++k) {
        r = lnl_app_t2(t, copy, r, w[k] & 0xFFFFu);
        r = lnl_app_t2(t, copy, r, w[k] >> 16);
    }
#endif
    return r;
}
LNL_HD LNL_INLINE uint32_t lnl_app_nibbles(const uint32_t* t, uint32_t base, uint32_t stride, uint32_t col, uint32_t v) {
    uint32_t r = 0;
    for (uint32_t k = 0; k < 8; ++k) r ^= t[base + (k * 16 + ((v >> (4 * k)) & 15u)) * stride + col];
    return r;
}
LNL_HD LNL_INLINE uint32_t lnl_app_s512(const uint32_t* t, uint32_t copy, uint32_t v) {
    return lnl_app_nibbles(t, kAppS512, kAppRepl, copy, v);
}
LNL_HD LNL_INLINE uint32_t lnl_app_m(const uint32_t* t, uint32_t s, uint32_t v) { return lnl_app_nibbles(t, kAppM, 32, s, v); }
LNL_HD LNL_INLINE uint32_t lnl_app_tb(const uint32_t* t, uint32_t z, uint32_t v) {
    return lnl_app_nibbles(t, kAppTB + z * 128u, 1, 0, v);
}

// ---- geometry and ownership ----------------------------------------------------
// One datagram's wire geometry (destination addresses, or offsets from any
// 16-byte-aligned origin: only their residues mod 16 and differences matter).
struct AppGeo {
    uint64_t P0, P1, P2;  // payload start, CRC start, end
    uint64_t V0;          // P0 & ~15
    uint64_t nv;          // pieces
    uint32_t pad;         // P0 - V0
    uint32_t Z;           // zero bytes after the payload in the last piece
};

LNL_HD LNL_INLINE AppGeo lnl_app_geo(uint64_t P0, uint64_t L) {
    AppGeo g;
    g.P0 = P0;
    g.P1 = P0 + L;
    g.P2 = g.P1 + 4u;
    g.V0 = P0 & ~(uint64_t)15;
    g.pad = (uint32_t)(P0 - g.V0);
    g.nv = (g.P1 - g.V0 + 15u) >> 4;
    g.Z = (uint32_t)(g.V0 + 16u * g.nv - g.P1);
    return g;
}

// The owner's test for a chunk c >= P0 it owns (c < P2): stored whole?
// (has_next / P1n: the next datagram and its payload end)
LNL_HD LNL_INLINE bool lnl_app_full_own(uint64_t c, uint64_t P2, bool has_next, uint64_t P1n) {
    return c + 16u <= P2 || (has_next && c + 16u <= P1n);
}
// The test of a datagram whose P0 is not 16-byte aligned for its head chunk
// hc = P0 & ~15 (owned by an earlier datagram): stored whole by its owner?
// Only the previous datagram can have stored it whole, and only when it owns
// hc (P0p <= hc) and this payload covers the rest of the chunk.
LNL_HD LNL_INLINE bool lnl_app_full_head(uint64_t hc, bool has_prev, uint64_t P0p, uint64_t P1) {
    return has_prev && P0p <= hc && hc + 16u <= P1;
}
// Is destination byte x of this datagram's wire range written by a whole-chunk
// store (its own or its owner's)?
LNL_HD LNL_INLINE bool lnl_app_byte_in_full_chunk(uint64_t x, uint64_t P0, uint64_t P1, uint64_t P2, bool has_prev,
                                                  uint64_t P0p, bool has_next, uint64_t P1n) {
    const uint64_t c = x & ~(uint64_t)15;
    return c >= P0 ? lnl_app_full_own(c, P2, has_next, P1n) : lnl_app_full_head(c, has_prev, P0p, P1);
}

// One 32-bit word of a tail chunk: bytes [cw, cw + 4) of the wire burst, from
// the 20 source bytes A[0..4] (dwords) at source address (cw - delta - 4) --
// so the payload byte at wire x is A byte x - cw + 4 and the next datagram's
// byte at wire x is A byte x - cw -- and the CRC at [P1, P2).
LNL_HD LNL_INLINE uint32_t lnl_app_tail_word(const uint32_t* A, uint32_t m, int64_t t1, int64_t t2, uint32_t crc) {
    // t1 = P1 - (chunk start + 4 m), t2 = P2 - (chunk start + 4 m)
    const uint32_t ma = t1 >= 4 ? 0xFFFFFFFFu : (t1 <= 0 ? 0u : (1u << (8 * t1)) - 1u);
    const uint32_t mb = t2 >= 4 ? 0u : (t2 <= 0 ? 0xFFFFFFFFu : ~((1u << (8 * t2)) - 1u));
    const uint32_t mc = ~(ma | mb);
    uint32_t cr = 0;
    if (t1 >= 0 && t1 < 4) cr = crc << (8 * t1);
    else if (t1 < 0 && t1 > -4) cr = crc >> (8 * -t1);
    return (A[m + 1] & ma) | (cr & mc) | (A[m] & mb);
}

}  // namespace lnl
