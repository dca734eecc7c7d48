// Host-side check of the kernel's per-lane algebra (crc32c_bitslice.h) against
// the oracle, without a GPU.  Each datagram is processed exactly as one lane
// of the HIP kernel does: the 128-byte-aligned lines it touches are read from
// the shared buffer (so the first and last rows also contain bytes of the
// neighbouring datagrams, which the zero line and the masks must remove),
// preceded by virtual rows when the lane's wave needs more rows than the
// datagram has; init XOR, row network, fold tree, final tables.
//
// Build/run: driven by tests/test_algebra.py (g++ -O2).  Exit status 0 = all
// equal; mismatches are printed.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../litenetlibpp_amd/csrc/crc32c_bitslice.h"

extern "C" uint32_t oracle_crc32c_bitwise(const uint8_t* p, size_t n);
extern "C" uint32_t oracle_crc32c_hw(const uint8_t* p, size_t n);

static uint32_t g_tab[LNL_TABLE_WORDS];

// mem: the buffer; addresses are offsets into it and the buffer is treated as
// starting on a 128-byte line.  `extra_rows` leading virtual rows (as in a
// wave whose longest datagram spans more lines) read the zero line.
static uint32_t lane_crc(const uint8_t* mem, size_t mem_len, size_t start, uint32_t len,
                         uint32_t extra_rows) {
    if (len == 0) return 0;
    const uint64_t line0 = start >> 7, line1 = (start + len - 1) >> 7;
    const uint32_t T = (uint32_t)(line1 - line0 + 1);
    const uint32_t pad = (uint32_t)(start & 127), e = 127u - (uint32_t)((start + len - 1) & 127);
    const uint32_t rows = T + extra_rows, first = extra_rows;
    const uint32_t c0 = g_tab[LNL_TABLE_C_OFF + pad];
    uint32_t s[32] = {0};
    for (uint32_t t = 0; t < rows; ++t) {
        const int32_t rel = (int32_t)t - (int32_t)first;
        const bool head = rel == 0, tail = t + 1 == rows;
        uint32_t hp, tp, hm[4], tm[4];
        lnl_piece_masks(head, tail, pad, e, hp, tp, hm, tm);
        uint32_t x[32];
        for (int w = 0; w < 32; ++w) {
            const uint32_t piece = (uint32_t)w >> 2;
            // the kernel's glds lanes fetch the zero line for virtual rows and
            // for whole pieces outside the datagram
            const bool zero = rel < 0 || (head && piece < hp) || (tail && piece > tp);
            uint32_t v = 0;
            for (int b = 0; b < 4 && !zero; ++b) {
                const long long a = (long long)((line0 + rel) << 7) + 4 * w + b;
                const uint8_t byte = (a >= 0 && (size_t)a < mem_len) ? mem[a] : 0xA5;
                v |= (uint32_t)byte << (8 * b);
            }
            x[w] = v;
        }
        if (head || tail) lnl_mask_row(x, hp, tp, hm, tm);
        if (head) x[0] ^= c0;  // CRC init as the row's first word
        uint32_t o[32];
        lnl_net_row_x(s, x, o);
        memcpy(s, o, sizeof s);
    }
    uint32_t r = lnl_fold_tree(s);
    r = lnl_table_apply(g_tab + 128 * lnl_table_b(e), r);
    r = lnl_table_apply(g_tab + 128 * lnl_table_a(e), r);
    return r ^ 0xFFFFFFFFu;
}

int main(int argc, char** argv) {
    const int max_len = argc > 1 ? atoi(argv[1]) : 1500;
    lnl_build_tables(g_tab);
    std::mt19937_64 rng(7);
    std::vector<uint8_t> mem(1 << 20);
    for (auto& b : mem) b = (uint8_t)rng();
    int bad = 0, checked = 0;
    for (int len = 0; len <= max_len; ++len) {
        for (size_t start : {size_t(0), size_t(1), size_t(127), size_t(4099), size_t(65536 + 3 * len)}) {
            const uint32_t extra = (uint32_t)(len % 3);
            const uint32_t got = lane_crc(mem.data(), mem.size(), start, (uint32_t)len, extra);
            const uint32_t exp = oracle_crc32c_hw(mem.data() + start, len);
            ++checked;
            if (got != exp) {
                if (bad < 20)
                    printf("MISMATCH len=%d start=%zu got=%08x exp=%08x\n", len, start, got, exp);
                ++bad;
            }
        }
    }
    for (uint32_t len : {4096u, 9000u, 65507u, 100003u}) {
        const uint32_t got = lane_crc(mem.data(), mem.size(), 12345, len, 1);
        const uint32_t exp = oracle_crc32c_bitwise(mem.data() + 12345, len);
        ++checked;
        if (got != exp) {
            printf("MISMATCH len=%u got=%08x exp=%08x\n", len, got, exp);
            ++bad;
        }
    }
    printf("checked=%d bad=%d\n", checked, bad);
    return bad ? 1 : 0;
}
