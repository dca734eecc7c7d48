// Host-side check of the span kernel's fold tables (litenetlibpp_amd/csrc/crc32c_span.h):
// the table Horner (lnl_span_phi) followed by the register-basis final map
// (lnl_span_final, and the LDS form lnl_span_final2) equals the bit-sliced fold (lnl_fold_tree) followed by the
// batch kernels' final map, for random states and every e; the row powers
// equal step^(1024 m); and on real rows the Horner is the raw CRC of the row.
//
// Build/run: driven by tests/test_algebra.py (g++ -O2).  Exit status 0 = all equal.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../litenetlibpp_amd/csrc/crc32c_bitslice.h"
#include "../../litenetlibpp_amd/csrc/crc32c_span.h"

extern "C" uint32_t oracle_crc32c_hw(const uint8_t* p, size_t n);

using namespace lnl;

static uint32_t g_tab[LNL_TABLE_WORDS];
static uint32_t g_span[kSpanTabWords];

int main() {
    lnl_build_tables(g_tab);
    lnl_build_span_tables(g_span);
    std::mt19937_64 rng(7);
    int bad = 0, checked = 0;
    for (int it = 0; it < 4000; ++it) {
        uint32_t v[32], f[32];
        for (int k = 0; k < 32; ++k) v[k] = (uint32_t)rng();
        if (it % 5 == 0)  // sparse states too
            for (int k = 0; k < 32; ++k) v[k] &= (uint32_t)rng() & (uint32_t)rng();
        memcpy(f, v, sizeof f);
        const uint32_t r_old = lnl_fold_tree(f);
        const uint32_t r_new = lnl_span_phi(g_span, v);
        for (uint32_t e = 0; e < 128; e += (it < 8 ? 1u : 37u)) {
            uint32_t o = lnl_table_apply(g_tab + 128 * lnl_table_b(e), r_old);
            o = ~lnl_table_apply(g_tab + 128 * lnl_table_a(e), o);
            const uint32_t n = lnl_span_final(g_span, e, r_new);
            const uint32_t n2 = lnl_span_final2(g_span, e, r_new);
            ++checked;
            if (o != n || o != n2) {
                if (bad < 10) printf("state %d e %u: fold tree %08x, span %08x\n", it, e, o, n);
                ++bad;
            }
        }
        const uint32_t m = it < 128 ? (uint32_t)it : (uint32_t)(rng() % 128);
        ++checked;
        if (lnl_span_rows(g_span, m, r_new) != lnl_step_bits(r_new, 1024 * (int32_t)m)) {
            if (bad < 10) printf("row power m=%u wrong\n", m);
            ++bad;
        }
    }
    // a single datagram of 1..128 bytes at the start of a row: state = its row
    // (bytes after it zero) with C[0] in word 0; CRC = final(e = 128 - len, phi)
    for (uint32_t len = 1; len <= 128; ++len) {
        uint8_t row[128] = {0};
        for (uint32_t i = 0; i < len; ++i) row[i] = (uint8_t)rng();
        uint32_t v[32];
        memcpy(v, row, sizeof v);
        v[0] ^= g_span[kSpanTabC + 0];
        ++checked;
        const uint32_t got = lnl_span_final(g_span, 128 - len, lnl_span_phi(g_span, v));
        const uint32_t exp = oracle_crc32c_hw(row, len);
        if (got != exp) {
            if (bad < 10) printf("len %u: %08x vs oracle %08x\n", len, got, exp);
            ++bad;
        }
    }
    printf("checked=%d bad=%d\n", checked, bad);
    return bad ? 1 : 0;
}
