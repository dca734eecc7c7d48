// Host-side check of the CSR segment kernel (litenetlibpp_amd/csrc/crc32c_seg.hip)
// against the oracle, without a GPU.  The whole launch is emulated with the
// kernel's own geometry and per-lane event logic: the pre-pass (first[], CRC 0
// for empty datagrams, overflow list), every lane of every wave-batch row by
// row (the datagram ends framed at the same row bytes, CRC init words, the
// fold at each end, the head/tail split), the lane-shuffle combine, the
// cross-wave fix-up, and the datagrams left to the batch kernel (checked
// with the oracle here; the batch kernel has its own emulation in
// emu_lane.cpp).  Every datagram must be written exactly once, with the
// oracle's CRC.
//
// Build/run: driven by tests/test_algebra.py (g++ -O2).  Exit status 0 = all
// equal.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../litenetlibpp_amd/csrc/crc32c_bitslice.h"
#include "../../litenetlibpp_amd/csrc/crc32c_seg.h"

extern "C" uint32_t oracle_crc32c_hw(const uint8_t* p, size_t n);

using namespace lnl;

static uint32_t g_tab[LNL_TABLE_WORDS];
static uint32_t g_pow[kSegPowTables * 128];

struct Case {
    uint64_t vbase;              // "device address" of mem[0] (128-byte aligned)
    std::vector<uint8_t> mem;    // the buffer, padded to whole lines with junk
    std::vector<uint64_t> off;   // n + 1 offsets, relative to base = vbase + base_shift
    uint64_t base_shift;         // d_base = vbase + base_shift
    uint64_t off0;
};

static uint32_t final_crc(uint32_t e, uint32_t r) {
    r = lnl_table_apply(g_tab + 128 * lnl_table_b(e), r);
    r = lnl_table_apply(g_tab + 128 * lnl_table_a(e), r);
    return ~r;
}

static uint32_t pow_apply(uint32_t m, uint32_t r) {
    for (uint32_t b = 0; b < kSegPowTables; ++b)
        if ((m >> b) & 1u) r = lnl_table_apply(g_pow + 128 * b, r);
    return r;
}

// run one case with `waves` resident waves; returns mismatches
static int run_case(const Case& C, uint32_t waves, const char* what, int& checked) {
    const uint32_t n = (uint32_t)C.off.size() - 1;
    const uint64_t base = C.vbase + C.base_shift;
    const uint64_t bsh = base - C.off0;
    const SegGeo G = seg_geometry(bsh + C.off[0], bsh + C.off[n], waves);
    std::vector<uint32_t> out(n, 0xDEADBEEFu);
    std::vector<int> writes(n, 0);
    std::vector<uint32_t> ovf;
    auto put = [&](uint32_t i, uint32_t v) {
        out[i] = v;
        ++writes[i];
    };
    auto mem_word = [&](uint64_t addr) -> uint32_t {
        uint32_t v;
        memcpy(&v, C.mem.data() + (addr - C.vbase), 4);
        return v;
    };
    const bool runs = G.NS != 0 && G.NS <= seg_max_segments(waves);
    // ---- pre-pass
    std::vector<uint32_t> first(runs ? G.NS + 1 : 0, 0xFFFFFFFFu);
    for (uint32_t i = 0; i < n; ++i) {
        if (!runs) {
            ovf.push_back(i);
            continue;
        }
        const uint64_t Pi = bsh + C.off[i] - G.S0, Pj = bsh + C.off[i + 1] - G.S0;
        if (Pi == Pj) put(i, 0u);
        if (Pj > Pi && seg_overflow(Pi, Pj, G.R)) ovf.push_back(i);
        const uint32_t lo = i == 0 ? 0u : seg_ceil(Pi, G.R), hi = seg_ceil(Pj, G.R);
        for (uint32_t g = lo; g < hi; ++g) first[g] = i;
        if (i + 1 == n) first[G.NS] = n;
    }
    if (runs) {
        for (uint32_t g = 0; g <= G.NS; ++g)
            if (first[g] == 0xFFFFFFFFu) {
                printf("%s: first[%u] unset\n", what, g);
                return 1;
            }
        const uint32_t R = G.R, NS = G.NS, Sb = R << 7;
        const uint32_t nwb = (NS + 63) >> 6;
        const uint64_t last_line = (G.S0 + G.Pn - 1) & ~(uint64_t)127;
        std::vector<uint32_t> carry(nwb, 0);
        struct Fix {
            uint32_t r, me, id, valid;
        };
        std::vector<Fix> fix(nwb, Fix{0, 0, 0, 0});
        for (uint32_t wb = 0; wb < nwb; ++wb) {
            uint32_t tails[64], heads_r[64], heads_m[64], heads_e[64], heads_id[64];
            bool has_head_v[64];
            for (uint32_t lane = 0; lane < 64; ++lane) {
                const uint32_t g = wb * 64 + lane;
                const bool live = g < NS;
                const uint64_t segbase = G.S0 + (uint64_t)g * Sb;
                uint32_t h0 = 0, h1 = 0, hp = 0;
                if (live) {
                    h0 = first[g];
                    h1 = first[g + 1];
                    hp = g ? first[g - 1] : h0;
                }
                const uint32_t cnt = h1 - h0;
                const bool excess = cnt > kSegTrack;
                const bool prev_excess = h0 - hp > kSegTrack;
                const uint32_t E = !live ? 0u : (excess ? kSegTrack : cnt + (h1 < n ? 1u : 0u));
                std::vector<uint32_t> Q;
                for (uint32_t k = 1; k <= E; ++k) {
                    const uint64_t p = bsh + C.off[h0 + k];
                    Q.push_back(p <= segbase ? 0u : (p - segbase >= 0xFFFF ? 0xFFFFu : (uint32_t)(p - segbase)));
                }
                size_t qi = 0;
                int32_t cs = 0;
                if (live) {
                    const int64_t d = (int64_t)(bsh + C.off[h0]) - (int64_t)segbase;
                    cs = d < -(int64_t)(2u * Sb) ? -(int32_t)(2u * Sb) : (int32_t)d;
                }
                if (live && excess) {
                    bool tail = false;
                    if (h1 < n) {
                        const uint64_t p0 = bsh + C.off[h1] - G.S0, p1 = bsh + C.off[h1 + 1] - G.S0;
                        tail = G.S0 + p0 < segbase + Sb && p1 > p0 && !seg_overflow(p0, p1, R);
                    }
                    for (uint32_t k = h0 + kSegTrack; k < h1 + (tail ? 1u : 0u); ++k) ovf.push_back(k);
                }
                uint32_t left = E, cid = h0, ce = 0, inj = 0;
                bool active = false, track = false, head = false;
                auto advance = [&]() {
                    do {
                        cs = (int32_t)ce;
                        ++cid;
                        head = false;
                        if (left == 0) {
                            active = false;
                            return;
                        }
                        ce = Q[qi++];
                        --left;
                        track = ce <= 2u * Sb;
                    } while (ce == (uint32_t)cs);
                };
                if (live && cs > 0) {
                    active = true;
                    ce = (uint32_t)cs;
                    cid = h0 - 1;
                } else if (live && left) {
                    active = true;
                    ce = Q[qi++];
                    --left;
                    head = cs < 0;
                    track = head ? (cs >= -(int32_t)Sb && ce <= Sb && !prev_excess) : ce <= 2u * Sb;
                    if (ce == (uint32_t)cs) advance();
                    if (active && !head && cs == 0 && track) inj = 0xFFFFFFFFu;
                }
                uint32_t s[32] = {0};
                uint32_t r_head = 0, m_head = 0, e_head = 0, id_head = 0;
                bool has_head = false;
                for (uint32_t t = 0; t < R; ++t) {
                    uint64_t line = segbase + ((uint64_t)t << 7);
                    if (line > last_line) line = last_line;
                    uint32_t x[32];
                    for (int w = 0; w < 32; ++w) x[w] = mem_word(line + 4 * w);
                    const uint32_t rowst = t << 7, rowend = rowst + 128u;
                    const bool ev0 = active && ce <= rowend;
                    uint32_t v[32] = {0};
                    uint32_t be = 0;
                    if (ev0) {
                        be = ce - 1u - rowst;
                        if (be > 127u) {
                            printf("%s: bad end byte g=%u t=%u ce=%u\n", what, g, t, ce);
                            return 1;
                        }
                        for (int w = 0; w < 32; ++w) {
                            const uint32_t xe = x[w] & lnl_word_keep_le(w, be);
                            v[w] = x[w] ^ xe;
                            x[w] = xe;
                        }
                    }
                    x[0] ^= inj;
                    inj = 0;
                    uint32_t o[32];
                    lnl_net_row_x(s, x, o);
                    if (!ev0) {
                        memcpy(s, o, sizeof s);
                        continue;
                    }
                    uint32_t ini = 0;
                    if (track) {
                        const uint32_t r = lnl_fold_tree(o);
                        if (head) {
                            r_head = r;
                            m_head = t + 1;
                            e_head = 127u - be;
                            id_head = cid;
                            has_head = true;
                        } else {
                            put(cid, final_crc(127u - be, r));
                        }
                    }
                    advance();
                    ini = active && track && cs < (int32_t)rowend ? g_tab[LNL_TABLE_C_OFF + (uint32_t)cs - rowst] : 0u;
                    while (active && ce <= rowend) {
                        const uint32_t be2 = ce - 1u - rowst;
                        uint32_t xe[32];
                        for (int w = 0; w < 32; ++w) {
                            const uint32_t m = lnl_word_keep_le(w, be2);
                            xe[w] = v[w] & m;
                            v[w] &= ~m;
                        }
                        xe[0] ^= ini;
                        if (track) put(cid, final_crc(127u - be2, lnl_fold_tree(xe)));
                        advance();
                        ini = active && track && cs < (int32_t)rowend ? g_tab[LNL_TABLE_C_OFF + (uint32_t)cs - rowst] : 0u;
                    }
                    if (active && cs < (int32_t)rowend) {
                        v[0] ^= ini;
                    } else {
                        memset(v, 0, sizeof v);
                        inj = active && track && cs == (int32_t)rowend ? 0xFFFFFFFFu : 0u;
                    }
                    memcpy(s, v, sizeof s);
                }
                uint32_t f[32];
                memcpy(f, s, sizeof f);
                tails[lane] = lnl_fold_tree(f);
                heads_r[lane] = r_head;
                heads_m[lane] = m_head;
                heads_e[lane] = e_head;
                heads_id[lane] = id_head;
                has_head_v[lane] = has_head;
            }
            for (uint32_t lane = 0; lane < 64; ++lane) {
                if (lane == 0) {
                    fix[wb] = Fix{heads_r[0], heads_m[0] | (heads_e[0] << 8), heads_id[0], has_head_v[0] ? 1u : 0u};
                } else if (has_head_v[lane]) {
                    put(heads_id[lane], final_crc(heads_e[lane], pow_apply(heads_m[lane], tails[lane - 1]) ^ heads_r[lane]));
                }
            }
            carry[wb] = tails[63];
        }
        for (uint32_t w = 1; w < nwb; ++w) {
            if (!fix[w].valid) continue;
            uint32_t r = pow_apply(fix[w].me & 0xFF, carry[w - 1]) ^ fix[w].r;
            put(fix[w].id, final_crc((fix[w].me >> 8) & 0xFF, r));
        }
    }
    // the batch kernel's share
    for (uint32_t i : ovf) put(i, oracle_crc32c_hw(C.mem.data() + (base + C.off[i] - C.off0 - C.vbase), C.off[i + 1] - C.off[i]));
    int bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t len = C.off[i + 1] - C.off[i];
        const uint32_t exp = oracle_crc32c_hw(C.mem.data() + (base + C.off[i] - C.off0 - C.vbase), len);
        ++checked;
        const bool once = writes[i] == 1 || (len == 0 && writes[i] >= 1);
        if (out[i] != exp || !once) {
            if (bad < 10)
                printf("%s: datagram %u len %llu writes %d got %08x exp %08x (R=%u NS=%u)\n", what, i,
                       (unsigned long long)len, writes[i], out[i], exp, G.R, G.NS);
            ++bad;
        }
    }
    return bad;
}

static Case make_case(std::mt19937_64& rng, const std::vector<uint64_t>& lens, uint32_t lead, uint64_t off0) {
    Case C;
    C.vbase = 0x100000;
    C.base_shift = lead % 128;
    C.off0 = off0;
    C.off.resize(lens.size() + 1);
    C.off[0] = off0 + (lead - C.base_shift);
    for (size_t i = 0; i < lens.size(); ++i) C.off[i + 1] = C.off[i] + lens[i];
    const uint64_t end = C.base_shift + (C.off.back() - off0);
    C.mem.resize(((end + 127) / 128 + 1) * 128);
    for (auto& b : C.mem) b = (uint8_t)rng();
    return C;
}

int main(int argc, char** argv) {
    const double scale = argc > 1 ? atof(argv[1]) : 1.0;  // fraction of each case's datagrams
    lnl_build_tables(g_tab);
    lnl_build_seg_tables(g_pow, (int)kSegPowTables);
    // the row-power tables against their definition: A^m r = L^-1 step^(1024 m) L r
    {
        uint32_t L[32], Li[32];
        for (int k = 0; k < 32; ++k) L[k] = lnl_step_bits(LNL_CRC32C_POLY, 992 - 32 * k);
        lnl_cols_inverse(L, Li);
        std::mt19937_64 r(3);
        for (uint32_t m = 1; m < 128; m += 7) {
            const uint32_t v = (uint32_t)r();
            const uint32_t exp = lnl_cols_apply(Li, lnl_step_bits(lnl_cols_apply(L, v), 1024 * (int32_t)m));
            if (pow_apply(m, v) != exp) {
                printf("pow table wrong at m=%u\n", m);
                return 1;
            }
        }
    }
    std::mt19937_64 rng(11);
    int bad = 0, checked = 0;
    auto uni = [&](uint64_t lo, uint64_t hi) { return lo + rng() % (hi - lo + 1); };
    struct Spec {
        const char* what;
        uint32_t n;
        int kind;
    };
    const Spec specs[] = {
        {"config3", 30000, 0}, {"tiny", 40000, 1}, {"long_mix", 8000, 2}, {"line_multiples", 12000, 3},
        {"segment_multiples", 3000, 4}, {"with_empties", 20000, 5}, {"one", 1, 0}, {"all_empty", 500, 6},
        {"one_long", 1, 7},
    };
    for (const Spec& sp : specs) {
        for (uint32_t waves : {1u, 2u, 5u, 16u}) {
            for (uint32_t lead : {0u, 1u, 77u, 127u, 128u, 300u}) {
                std::vector<uint64_t> lens(sp.n > 1 ? (size_t)(sp.n * scale) + 1 : sp.n);
                for (auto& L : lens) {
                    switch (sp.kind) {
                        case 0: L = uni(64, 1400); break;
                        case 1: L = uni(0, 40); break;
                        case 2: L = rng() % 10 == 0 ? uni(2000, 40000) : uni(0, 1432); break;
                        case 3: L = 128 * uni(0, 12) + (rng() % 4 == 0 ? uni(0, 2) : 0); break;
                        case 4: L = 2048 * uni(1, 3) - (rng() % 3 == 0 ? 1 : 0); break;
                        case 5: L = rng() % 3 == 0 ? 0 : uni(1, 1432); break;
                        case 6: L = 0; break;
                        default: L = 200000; break;
                    }
                }
                Case C = make_case(rng, lens, lead, lead % 3 == 0 ? 0 : 5000);
                char what[96];
                snprintf(what, sizeof what, "%s/W%u/lead%u", sp.what, waves, lead);
                bad += run_case(C, waves, what, checked);
            }
        }
    }
    printf("checked=%d bad=%d\n", checked, bad);
    return bad ? 1 : 0;
}
