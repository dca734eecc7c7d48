// crc32c_span.h -- geometry of the CSR span kernel (crc32c_span.hip), shared by
// its pre-pass, the kernel, the fix-up and the host planner.
//
// A CSR batch's bytes are one contiguous stream: datagram i is
// base[off[i] - off0 .. off[i+1] - off0).  From the 128-byte line holding the
// first byte (S0) to the last byte (S0 + Pn) the stream is cut into SEGMENTS
// of R lines (Sb = 128 R bytes).  Lane l of wave-batch w owns segment
// g = 64 w + l.  R is chosen so that one round of every resident wave covers
// the batch (R = ceil(lines / 64 W)), clamped to [kSpanRmin, kSpanRmax];
// larger batches take several wave-batches per wave, up to kSpanMaxRounds
// rounds (beyond that the whole batch goes to the any-layout batch kernel).
#pragma once
#include <stdint.h>

#include "crc32c_bitslice.h"
#include "lnl_packet.h"

namespace lnl {

constexpr uint32_t kSpanRmin = 16;
constexpr uint32_t kSpanRmax = 127;      // boundaries fit 16 bits (2 Sb < 65535); row powers m < 128
constexpr uint32_t kSpanMaxRounds = 8;   // wave-batches per resident wave
// Control block (words): [1] overflow count, [2] segments, [3] R.  A stream's
// span scratch holds two, used by alternate calls: a call's batch kernel zeroes
// the other block's count, so every call starts from 0 with no memset launch.
constexpr uint32_t kSpanCtlWords = 8;

struct SpanGeo {
    uint64_t S0;   // address of the stream's first line
    uint64_t Pn;   // bytes from S0 to the end of the last datagram
    uint32_t R;    // lines per segment
    uint32_t NS;   // segments (0: nothing to do)
    uint32_t nwb;  // wave-batches (ceil(NS / 64))
};

LNL_HD LNL_INLINE uint32_t span_max_segments(uint32_t waves) { return 64u * waves * kSpanMaxRounds; }

LNL_HD LNL_INLINE SpanGeo span_geometry(uint64_t first_byte, uint64_t end_byte, uint32_t waves) {
    SpanGeo G;
    G.S0 = first_byte & ~(uint64_t)127;
    G.Pn = end_byte - G.S0;
    const uint64_t lines = (G.Pn + 127u) >> 7;
    const uint64_t per = 64ull * waves;
    uint64_t R = (lines + per - 1u) / per;
    R = R < kSpanRmin ? kSpanRmin : (R > kSpanRmax ? kSpanRmax : R);
    G.R = (uint32_t)R;
    const uint64_t ns = (lines + R - 1u) / R;
    G.NS = ns > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)ns;
    G.nwb = (G.NS + 63u) >> 6;
    return G;
}

// The span kernel takes the batch when it has something to do and fits the
// rounds the scratch was sized for.
LNL_HD LNL_INLINE bool span_runs(const SpanGeo& G, uint32_t waves) {
    return G.NS != 0u && G.NS <= span_max_segments(waves);
}

// Datagram [Pi, Pj) (offsets from S0, Pj > Pi) is left to the batch kernel
// when it touches three or more segments (a lane combines a datagram with at
// most the previous lane's tail).
LNL_HD LNL_INLINE bool span_overflow(uint64_t Pi, uint64_t Pj, uint32_t R) {
    const uint64_t gs = (Pi >> 7) / R, ge = ((Pj - 1u) >> 7) / R;
    return ge > gs + 1u;
}

// A head (the datagram that entered a segment from the previous one) and a
// tail (the one still open at a segment's end) are folded to CRC register
// values (lnl_span_phi below) and combined:
//   head CRC = ~step^(-8e)(step^(1024 m)(tail) ^ head)
// (m = rows from the segment start through the head's last row, e = bytes of
// that row after the head's last byte).  Within a wave-batch the lanes combine
// them through a shuffle; across wave-batches through an exchange block per
// boundary in the stream's scratch (kSpanXch*).
// hinfo word: m | e << 8 | head tracked << 16
constexpr uint32_t kSpanHeadBit = 1u << 16;
// exchange block of wave-batch boundary w (words): the arrival word (u64,
// words 0-1), the tail side (lane 63 of w - 1: its register value, its
// datagram's start in the segment | header byte << 16) and the head side (lane
// 0 of w: register value, datagram index, hinfo).
// Arrival: each side stores its part, drains it (vmcnt(0)), then swaps
// span_arrival(epoch, side) into the arrival word.  The side whose swap
// returns span_arrival(epoch, other side) arrived second and combines.  The
// epoch is the call's (SpanArgs::epoch, one per call on a scratch buffer), so
// whatever an earlier call -- finished or aborted -- left in the word never
// pairs: no word has to be reset between calls.
constexpr uint32_t kSpanXchFlag = 0, kSpanXchTail = 2, kSpanXchTailInfo = 3, kSpanXchHead = 4,
                   kSpanXchHeadIdx = 5, kSpanXchHeadInfo = 6;
constexpr uint32_t kSpanXchWords = 8;  // one 32-byte sector per boundary
constexpr uint32_t kSpanSideHead = 1, kSpanSideTail = 2;
LNL_HD LNL_INLINE uint64_t span_arrival(uint64_t epoch, uint32_t side) { return (epoch << 2) | side; }

// ---- verify modes ---------------------------------------------------------------
// The span kernel checks a wire datagram (payload || LE32(CRC)) without
// locating its CRC field: CRC-32C over the WHOLE datagram is the residue
// 0x48674BC7 exactly when the trailing four bytes are the CRC of the rest (the
// CRC of m || t is a bijection of t, and t = CRC(m) gives the residue).  So a
// verify call computes the same whole-datagram CRCs as a CSR call and compares.
enum : uint32_t { kSpanCrc = 0, kSpanVerify = 1, kSpanFilter = 2 };
constexpr uint32_t kCrc32cResidue = 0x48674BC7u;

// ---- the span kernel's fold -------------------------------------------------
// A state V (32 words) is folded to the CRC register directly: L(fold(V)) (the
// register lnl_fold_tree + L give, crc32c_bitslice.h) is the raw CRC -- zero
// init, no final XOR -- of the 128 bytes V itself, since both are the same
// linear map of the row bits (bit j of word k counts step^(1023-32k-j) POLY).
// So the fold is a table Horner over V's words: r <- T(r ^ V_k), T = step^32 as
// four byte tables, in four independent 8-word chains joined by step^256 --
// ~200 VALU ops and 128 LDS lookups instead of lnl_fold_tree's ~880 ops.  The
// final map is then step^(-8e) alone (no L).
//
// Table block (words); the first kSpanTabLds go to LDS:
//   T     [i * 256 + v] = step^32(v << 8 i), i = 0..3
//   S256  nibble tables of step^256
//   TB    [b] = step^(-8 b), b = 0..15 (nibble tables)
//   TA    [a] = step^(-128 a), a = 0..7
//   C     [pad] = step^(-8 pad)(0xFFFFFFFF)
//   ROWS  [m] = step^(1024 m), m = 0..127 (the head combine's row powers)
//   FIN   [e] = step^(-8 e), e = 0..127 (the final map in one product)
//   (ROWS and FIN: global memory only; one nibble-table product each, so a
//   head costs two dependent lookups rounds, not nine)
constexpr uint32_t kSpanTabT = 0;
constexpr uint32_t kSpanTabS = 1024;
constexpr uint32_t kSpanTabB = kSpanTabS + 128;
constexpr uint32_t kSpanTabA = kSpanTabB + 16 * 128;
constexpr uint32_t kSpanTabC = kSpanTabA + 8 * 128;
constexpr uint32_t kSpanTabLds = kSpanTabC + 128;
constexpr uint32_t kSpanTabRows = kSpanTabLds;
constexpr uint32_t kSpanTabFin = kSpanTabRows + 128 * 128;
constexpr uint32_t kSpanTabWords = kSpanTabFin + 128 * 128;

// nibble tables (128 words) of the matrix with columns cols
LNL_HD inline void lnl_nibble_tables(uint32_t* dst, const uint32_t* cols) {
    for (uint32_t k = 0; k < 8; ++k)
        for (uint32_t v = 0; v < 16; ++v) dst[16 * k + v] = lnl_cols_apply(cols, v << (4 * k));
}
// dst[m] = nibble tables of step^(n m), m = 0..127
LNL_HD inline void lnl_power_tables(uint32_t* dst, int32_t n) {
    uint32_t one[32], cur[32], nxt[32];
    for (int k = 0; k < 32; ++k) {
        one[k] = lnl_step_bits(1u << k, n);
        cur[k] = 1u << k;
    }
    for (uint32_t m = 0; m < 128; ++m) {
        lnl_nibble_tables(dst + 128 * m, cur);
        for (int k = 0; k < 32; ++k) nxt[k] = lnl_cols_apply(one, cur[k]);
        for (int k = 0; k < 32; ++k) cur[k] = nxt[k];
    }
}

LNL_HD inline void lnl_build_span_tables(uint32_t* t) {
    for (uint32_t i = 0; i < 4; ++i)
        for (uint32_t v = 0; v < 256; ++v) t[kSpanTabT + 256 * i + v] = lnl_step_bits(v << (8 * i), 32);
    for (uint32_t k = 0; k < 8; ++k)
        for (uint32_t v = 0; v < 16; ++v) {
            const uint32_t x = v << (4 * k);
            t[kSpanTabS + 16 * k + v] = lnl_step_bits(x, 256);
            for (int32_t b = 0; b < 16; ++b) t[kSpanTabB + 128 * b + 16 * k + v] = lnl_step_bits(x, -8 * b);
            for (int32_t a = 0; a < 8; ++a) t[kSpanTabA + 128 * a + 16 * k + v] = lnl_step_bits(x, -128 * a);
        }
    for (uint32_t pad = 0; pad < 128; ++pad) t[kSpanTabC + pad] = lnl_step_bits(0xFFFFFFFFu, -8 * (int32_t)pad);
    lnl_power_tables(t + kSpanTabRows, 1024);
    lnl_power_tables(t + kSpanTabFin, -8);
}

// Host / emulation form of the fold (the kernel reads the same tables from LDS).
LNL_HD LNL_INLINE uint32_t lnl_span_t4(const uint32_t* t, uint32_t x) {
    return t[x & 255u] ^ t[256u + ((x >> 8) & 255u)] ^ t[512u + ((x >> 16) & 255u)] ^ t[768u + (x >> 24)];
}
LNL_HD inline uint32_t lnl_span_phi(const uint32_t* t, const uint32_t* v) {
    uint32_t r[4] = {0u, 0u, 0u, 0u};
    for (int k = 0; k < 8; ++k)
        for (int c = 0; c < 4; ++c) r[c] = lnl_span_t4(t + kSpanTabT, r[c] ^ v[8 * c + k]);
    uint32_t p = r[0];
    for (int c = 1; c < 4; ++c) p = lnl_table_apply(t + kSpanTabS, p) ^ r[c];
    return p;
}
// CRC of a datagram from its register value r (lnl_span_phi of its ended
// state) and e < 128, the bytes of its last row after it: ~step^(-8e)(r) --
// as the kernel's LDS tables do it (TB, TA) and in one product (FIN)
LNL_HD LNL_INLINE uint32_t lnl_span_final2(const uint32_t* t, uint32_t e, uint32_t r) {
    r = lnl_table_apply(t + kSpanTabB + 128u * (e & 15u), r);
    r = lnl_table_apply(t + kSpanTabA + 128u * (e >> 4), r);
    return ~r;
}
LNL_HD LNL_INLINE uint32_t lnl_span_final(const uint32_t* t, uint32_t e, uint32_t r) {
    return ~lnl_table_apply(t + kSpanTabFin + 128u * e, r);
}
// step^(1024 m) r: m < 128 rows of zeros after a register value r
LNL_HD LNL_INLINE uint32_t lnl_span_rows(const uint32_t* t, uint32_t m, uint32_t r) {
    return lnl_table_apply(t + kSpanTabRows + 128u * m, r);
}

// LNL_INBOUND_* of a wire datagram from its whole-datagram CRC, its length and
// its first byte (verify: 1 / 0 only; filter: then net_packet::verify() of the
// stripped packet, lnl_packet.h)
LNL_HD LNL_INLINE uint32_t lnl_span_status(uint32_t mode, uint32_t crc, uint32_t len, uint32_t hdr) {
    if (len < 5u || crc != kCrc32cResidue) return 0u;
    if (mode != kSpanFilter) return 1u;
    return lnl_packet_verify_hdr((uint8_t)hdr, len - 4u) ? 1u : 2u;
}

}  // namespace lnl
