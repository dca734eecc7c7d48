// crc32c_seg.h -- geometry of the CSR segment kernel (crc32c_seg.hip), shared by
// its pre-pass, the kernel itself and the CPU emulation (tests/emu/emu_seg.cpp).
//
// The batch's bytes, from the 128-byte line holding its first byte (S0) to its
// last byte (S0 + Pn), are cut into SEGMENTS of R lines (Sb = 128 R bytes).
// Wave-batch w owns segments 64 w .. 64 w + 63, one per lane.  R is chosen so
// that the segments fill every resident wave once (R = ceil(lines / 64 W)),
// at least kSegRmin (a datagram of up to 2 KiB then touches at most two
// segments) and at most kSegRmax (the row-power tables and the 16-bit end
// offsets).  Longer batches take several wave-batches per wave, up to
// kSegBatchesPerWave; beyond that the whole batch goes to the batch kernel.
#pragma once
#include <stdint.h>

#include "crc32c_bitslice.h"

namespace lnl {

constexpr uint32_t kSegRmin = 16;
constexpr uint32_t kSegRmax = 127;
constexpr uint32_t kSegPowTables = 7;           // A^(2^b), b = 0..6: shifts by 1..127 rows
constexpr uint32_t kSegQueue = 16;              // datagram ends a lane queues (16-bit, two per register)
constexpr uint32_t kSegTrack = kSegQueue - 1;   // datagrams ending in one segment a lane checksums
constexpr uint32_t kSegBatchesPerWave = 4;

struct SegGeo {
    uint64_t S0;  // address of the batch's first line
    uint64_t Pn;  // bytes from S0 to the end of the last datagram
    uint32_t R;   // lines per segment
    uint32_t NS;  // segments (0: nothing to do)
};

LNL_HD LNL_INLINE uint32_t seg_max_segments(uint32_t waves) { return 64u * waves * kSegBatchesPerWave; }

LNL_HD LNL_INLINE SegGeo seg_geometry(uint64_t first_byte, uint64_t end_byte, uint32_t waves) {
    SegGeo G;
    G.S0 = first_byte & ~(uint64_t)127;
    G.Pn = end_byte - G.S0;
    const uint64_t lines = (G.Pn + 127u) >> 7;
    const uint64_t per = 64ull * waves;
    uint64_t R = (lines + per - 1u) / per;
    R = R < kSegRmin ? kSegRmin : (R > kSegRmax ? kSegRmax : R);
    G.R = (uint32_t)R;
    const uint64_t ns = (lines + R - 1u) / R;
    G.NS = ns > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)ns;
    return G;
}

// ceil(P / (128 R)) for a byte offset P from S0 (line indices fit 32 bits:
// batches below 512 GiB).
LNL_HD LNL_INLINE uint32_t seg_ceil(uint64_t P, uint32_t R) {
    const uint32_t lines = (uint32_t)((P + 127u) >> 7);
    return (lines + R - 1u) / R;
}

// Datagram [Pi, Pj) (offsets from S0, Pj > Pi) is left to the batch kernel
// when it touches three or more segments.
LNL_HD LNL_INLINE bool seg_overflow(uint64_t Pi, uint64_t Pj, uint32_t R) {
    const uint32_t gs = (uint32_t)(Pi >> 7) / R, ge = (uint32_t)((Pj - 1u) >> 7) / R;
    return ge > gs + 1u;
}

}  // namespace lnl
