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

// One lane of the lane-run kernel (crc32c_run.hip): K datagrams of len bytes
// at stride S starting at mem offset A (len >= 129, S >= len, K even),
// processed as the 128-byte lines from A's line on, with the kernel's
// wave-uniform start / end events and the pairwise fold.
static int run_lane(const uint8_t* mem, size_t A, uint32_t S, uint32_t len, uint32_t K,
                    uint32_t* crc_out) {
    const uint32_t ph = (uint32_t)(A & 127);
    const size_t line0 = A - ph;
    const uint32_t R = (ph + (K - 1) * S + len + 127) >> 7;
    uint32_t s[32] = {0}, P[32] = {0};
    uint32_t ks = 0, ke = 0, sb = ph, eb = ph + len - 1, eprev = 0;
    for (uint32_t t = 0; t < R; ++t) {
        uint32_t x[32];
        memcpy(x, mem + line0 + 128 * (size_t)t, 128);
        const bool st = ks < K && (sb >> 7) == t;
        const bool en = ke < K && (eb >> 7) == t;
        uint32_t o[32];
        if (!st && !en) {
            lnl_net_row_x(s, x, o);
            memcpy(s, o, sizeof s);
            continue;
        }
        uint32_t xe[32];
        const uint32_t be = eb & 127u, bs = sb & 127u;
        if (en) {
            for (int w = 0; w < 32; ++w) xe[w] = x[w] & lnl_word_keep_le(w, be);
            lnl_net_row_x(s, xe, o);
        }
        if (st) {
            if (en && S == len)
                for (int w = 0; w < 32; ++w) s[w] = x[w] ^ xe[w];
            else
                for (int w = 0; w < 32; ++w) s[w] = x[w] & lnl_word_keep_ge(w, bs);
            s[0] ^= g_tab[LNL_TABLE_C_OFF + bs];
            ++ks;
            sb += S;
        }
        if (en) {
            uint32_t f[32];
            lnl_fold_level1(o, f);
            if ((ke & 1u) == 0) {
                memcpy(P, f, sizeof P);
                eprev = 127u - be;
            } else {
                uint32_t ra, rb;
                lnl_fold_pair(P, f, ra, rb);
                const uint32_t eb2 = 127u - be;
                ra = lnl_table_apply(g_tab + 128 * lnl_table_a(eprev), lnl_table_apply(g_tab + 128 * lnl_table_b(eprev), ra));
                rb = lnl_table_apply(g_tab + 128 * lnl_table_a(eb2), lnl_table_apply(g_tab + 128 * lnl_table_b(eb2), rb));
                crc_out[ke - 1] = ~ra;
                crc_out[ke] = ~rb;
            }
            ++ke;
            eb += S;
        }
    }
    return (int)ke;
}

static int check_runs(const std::vector<uint8_t>& mem, int& checked) {
    int bad = 0;
    const uint32_t lens[] = {129, 130, 200, 255, 256, 257, 511, 1000, 1399, 1400, 1401, 1432, 4000};
    const uint32_t gaps[] = {0, 1, 7, 100, 127, 128, 300};
    for (uint32_t len : lens)
        for (uint32_t gap : gaps)
            for (uint32_t K : {2u, 4u, 8u})
                for (uint32_t ph = 0; ph < 128; ph += 9) {
                    const uint32_t S = len + gap;
                    const size_t A = 4096 + ph;
                    uint32_t got[8];
                    const int nk = run_lane(mem.data(), A, S, len, K, got);
                    if (nk != (int)K) {
                        printf("RUN count len=%u S=%u K=%u ph=%u got %d\n", len, S, K, ph, nk);
                        ++bad;
                        continue;
                    }
                    for (uint32_t k = 0; k < K; ++k) {
                        const uint32_t exp = oracle_crc32c_hw(mem.data() + A + (size_t)k * S, len);
                        ++checked;
                        if (got[k] != exp) {
                            if (bad < 20)
                                printf("RUN MISMATCH len=%u S=%u K=%u ph=%u k=%u got=%08x exp=%08x\n", len, S,
                                       K, ph, k, got[k], exp);
                            ++bad;
                        }
                    }
                }
    return bad;
}

// One lane of the CSR pair kernel (crc32c_pair.hip): datagrams a = [sa, sa+la)
// and b = [sa+la, sa+la+lb) (CSR datagrams are contiguous) as Ta + Tb steps,
// step u reading line u (u < Ta) or u - shared (u >= Ta) of the run -- the
// line a and b share is read at two consecutive steps -- framed at read time
// to bytes lo..hi (a's / b's first byte on its first step, last byte on its
// last step); a fresh state V = X on a datagram's first step; pairwise fold.
static void pair_lane(const uint8_t* mem, size_t sa, uint32_t la, uint32_t lb, uint32_t* ca, uint32_t* cb) {
    const size_t sb = sa + la;
    const uint32_t Ta = la ? (uint32_t)(((sa + la - 1) >> 7) - (sa >> 7) + 1) : 0;
    const uint32_t Tb = lb ? (uint32_t)(((sb + lb - 1) >> 7) - (sb >> 7) + 1) : 0;
    const uint32_t shared = (la && lb && ((sa + la - 1) >> 7) == (sb >> 7)) ? 1u : 0u;
    const uint32_t steps = Ta + Tb;
    *ca = 0;
    *cb = 0;
    if (steps == 0) return;
    const size_t first = la ? sa : sb;
    const size_t line0 = first & ~(size_t)127;
    const uint32_t pad_a = (uint32_t)(sa & 127), be_a = (uint32_t)((sa + la - 1) & 127);
    const uint32_t pad_b = (uint32_t)(sb & 127), be_b = (uint32_t)((sb + lb - 1) & 127);
    uint32_t s[32] = {0}, P[16] = {0};
    for (uint32_t u = 0; u < steps; ++u) {
        const uint32_t line = u - (shared && u >= Ta ? 1u : 0u);
        uint32_t x[32];
        memcpy(x, mem + line0 + 128 * (size_t)line, 128);
        const bool inA = u < Ta;
        const bool start = u == 0 || u == Ta;
        const bool end = u + 1 == Ta || u + 1 == steps;
        const uint32_t lo = start ? (inA ? pad_a : pad_b) : 0u;
        const uint32_t hi = end ? (inA ? be_a : be_b) : 127u;
        for (int w = 0; w < 32; ++w) x[w] &= lnl_word_keep_ge(w, lo) & lnl_word_keep_le(w, hi);
        if (start) {
            x[0] ^= g_tab[LNL_TABLE_C_OFF + (inA ? pad_a : pad_b)];
            memcpy(s, x, sizeof s);
        } else {
            uint32_t o[32];
            lnl_net_row_x(s, x, o);
            memcpy(s, o, sizeof s);
        }
        if (end) {
            if (inA) {
                uint32_t fa[32];
                lnl_fold_level1(s, fa);
                lnl_pack_level1(fa, P);
            }
            if (!inA || !Tb) {
                uint32_t f[32] = {0}, ra, rb;
                if (!inA) lnl_fold_level1(s, f);
                lnl_fold_pair_packed(P, f, ra, rb);
                const uint32_t ea = 127u - be_a, eb = 127u - be_b;
                if (Ta) *ca = ~lnl_table_apply(g_tab + 128 * lnl_table_a(ea), lnl_table_apply(g_tab + 128 * lnl_table_b(ea), ra));
                if (Tb) *cb = ~lnl_table_apply(g_tab + 128 * lnl_table_a(eb), lnl_table_apply(g_tab + 128 * lnl_table_b(eb), rb));
            }
        }
    }
}

static int check_pairs(const std::vector<uint8_t>& mem, int& checked) {
    int bad = 0;
    std::mt19937_64 rng(99);
    const uint32_t lens[] = {0, 1, 2, 3, 4, 15, 16, 17, 100, 126, 127, 128, 129, 200, 255, 256, 257, 700, 1400, 1432, 3000};
    for (uint32_t la : lens)
        for (uint32_t lb : lens)
            for (int rep = 0; rep < 6; ++rep) {
                const size_t sa = 4096 + (rng() % 128) + (rep == 0 ? 0 : 128 * (rng() % 4));
                uint32_t ca, cb;
                pair_lane(mem.data(), sa, la, lb, &ca, &cb);
                const uint32_t ea = oracle_crc32c_hw(mem.data() + sa, la);
                const uint32_t eb = oracle_crc32c_hw(mem.data() + sa + la, lb);
                checked += 2;
                if (ca != ea || cb != eb) {
                    if (bad < 20)
                        printf("PAIR MISMATCH la=%u lb=%u sa=%zu got=%08x,%08x exp=%08x,%08x\n", la, lb, sa, ca, cb,
                               ea, eb);
                    ++bad;
                }
            }
    return bad;
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
    bad += check_runs(mem, checked);
    bad += check_pairs(mem, checked);
    printf("checked=%d bad=%d\n", checked, bad);
    return bad ? 1 : 0;
}
