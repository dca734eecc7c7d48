// Host-side check of the one-pass outbound layer (litenetlibpp_amd/csrc/crc32c_append.h,
// the kernel in lnl_append.hip): every 32-lane team's CRC algebra -- destination-
// aligned pieces, C[pad] init, slicing-by-2 lane CRCs, S512 Horner across a lane's
// pieces, per-lane M_s shifts, team XOR, TB_Z unshift -- and the chunk-ownership
// rule that decides which destination chunks are stored whole, by whom, and which
// bytes go one by one.  Bursts of many shapes (every destination alignment,
// empty and 1..40-byte datagrams, MTU sizes, 65,507-byte datagrams) are written
// into a poisoned buffer through exactly the stores the kernel makes; every wire
// byte must be written, and by one store, and the CRCs must equal the oracle's.
//
// Build/run: driven by tests/test_algebra.py (g++ -O2).  Prints bad=0 when all agree.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../litenetlibpp_amd/csrc/crc32c_append.h"

extern "C" uint32_t oracle_crc32c_hw(const uint8_t* p, size_t n);

using namespace lnl;

static std::vector<uint32_t> g_t(kAppTabWords);

struct Burst {
    std::vector<uint8_t> src;   // guard bytes around the payloads
    std::vector<uint64_t> off;  // into src
    uint32_t dalign;            // destination origin mod 16
};

static int g_bad = 0;
static long g_checked = 0;

static void fail(const char* what, uint32_t i, long x) {
    if (g_bad++ < 20) printf("FAIL %s datagram %u byte %ld\n", what, i, x);
}

static void run(const Burst& b) {
    const uint32_t n = (uint32_t)b.off.size() - 1;
    const uint64_t total = b.off[n] - b.off[0] + 4ull * n;
    const uint64_t D = b.dalign;  // wire byte k of the burst is destination D + k
    std::vector<uint8_t> wire(D + total + 64, 0xA5);
    std::vector<uint8_t> writes(wire.size(), 0);
    auto src_at = [&](uint32_t i, uint64_t P0, uint64_t x) -> uint8_t {  // source byte for wire x at datagram i's shift
        const int64_t s = (int64_t)b.off[i] + (int64_t)(x - P0);
        return (s >= 0 && s < (int64_t)b.src.size()) ? b.src[s] : 0xEE;
    };
    auto put = [&](uint64_t x, uint8_t v, uint32_t i) {
        if (x < D || x >= D + total) return fail("store outside the burst", i, (long)x);
        wire[x] = v;
        ++writes[x];
    };
    std::vector<uint32_t> crcs(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t L = b.off[i + 1] - b.off[i];
        const uint64_t P0 = D + (b.off[i] - b.off[0]) + 4ull * i;
        const AppGeo g = lnl_app_geo(P0, L);
        const bool has_prev = i > 0, has_next = i + 1 < n;
        const uint64_t P0p = has_prev ? P0 - 4 - (b.off[i] - b.off[i - 1]) : 0;
        const uint64_t P1n = has_next ? g.P2 + (b.off[i + 2] - b.off[i + 1]) : 0;
        // ---- pieces: lane q takes v = q, q + 32, ...
        uint32_t acc[kAppTeam] = {0}, vlast[kAppTeam];
        bool has[kAppTeam] = {false};
        for (uint64_t v = 0; v < g.nv; ++v) {
            const uint32_t q = (uint32_t)(v % kAppTeam);
            const uint64_t c = g.V0 + 16 * v;
            uint8_t win[16], pc[16];
            for (int j = 0; j < 16; ++j) {
                win[j] = src_at(i, P0, c + j);
                pc[j] = (c + j >= g.P0 && c + j < g.P1) ? win[j] : 0;
            }
            uint32_t w[4];
            memcpy(w, pc, 16);
            if (v == 0) w[0] ^= g_t[kAppC + g.pad];
            const uint32_t copy = q % kAppRepl;
            const uint32_t r = lnl_app_piece(g_t.data(), copy, w);
            acc[q] = has[q] ? lnl_app_s512(g_t.data(), copy, acc[q]) ^ r : r;
            has[q] = true;
            vlast[q] = (uint32_t)v;
            if (c >= g.P0 && c + 16 <= g.P1)  // a payload chunk it owns: stored whole in the main loop
                for (int j = 0; j < 16; ++j) put(c + j, win[j], i);
        }
        uint32_t x = 0;
        for (uint32_t q = 0; q < kAppTeam; ++q)
            if (has[q]) x ^= lnl_app_m(g_t.data(), (uint32_t)(g.nv - 1 - vlast[q]), acc[q]);
        const uint32_t crc = L ? ~lnl_app_tb(g_t.data(), g.Z, x) : 0u;
        crcs[i] = crc;
        ++g_checked;
        const uint32_t exp = oracle_crc32c_hw(b.src.data() + b.off[i], L);
        if (crc != exp) fail("crc", i, -1);
        // ---- tail chunks (lanes 0, 1)
        for (uint32_t q = 0; q < 2; ++q) {
            const uint64_t c = (g.P1 & ~(uint64_t)15) + 16 * q;
            if (c < g.P0 || c >= g.P2 || !lnl_app_full_own(c, g.P2, has_next, P1n)) continue;
            uint32_t A[5];
            uint8_t a8[20];
            for (int j = 0; j < 20; ++j) a8[j] = src_at(i, P0, c - 4 + j);
            memcpy(A, a8, 20);
            for (uint32_t m = 0; m < 4; ++m) {
                const uint32_t wv = lnl_app_tail_word(A, m, (int64_t)g.P1 - (int64_t)(c + 4 * m),
                                                      (int64_t)g.P2 - (int64_t)(c + 4 * m), crc);
                for (int k = 0; k < 4; ++k) put(c + 4 * m + k, (uint8_t)(wv >> (8 * k)), i);
            }
        }
        // ---- byte path: head chunk bytes, then tail bytes, of chunks not stored whole
        const uint64_t hc = g.P0 & ~(uint64_t)15, tb = (g.P1 & ~(uint64_t)15) > g.P0 ? (g.P1 & ~(uint64_t)15) : g.P0;
        std::vector<uint8_t> done(36, 0);
        for (uint32_t k = 0; k < 36; ++k) {
            const uint64_t xb = k < 16 ? g.P0 + k : tb + (k - 16);
            if (xb >= g.P2) continue;
            if (k < 16 && !(hc < g.P0 && xb < hc + 16)) continue;
            if (k >= 16 && xb < hc + 16 && hc < g.P0) continue;  // (the head candidates took it)
            if (lnl_app_byte_in_full_chunk(xb, g.P0, g.P1, g.P2, has_prev, P0p, has_next, P1n)) continue;
            put(xb, xb < g.P1 ? src_at(i, P0, xb) : (uint8_t)(crc >> (8 * (xb - g.P1))), i);
        }
    }
    // ---- the burst: payload || LE32(crc) per datagram, each byte written once
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t P0 = D + (b.off[i] - b.off[0]) + 4ull * i, L = b.off[i + 1] - b.off[i];
        for (uint64_t k = 0; k < L + 4; ++k) {
            const uint8_t e = k < L ? b.src[b.off[i] + k] : (uint8_t)(crcs[i] >> (8 * (k - L)));
            if (wire[P0 + k] != e) fail("wire byte", i, (long)k);
            if (writes[P0 + k] != 1) fail(writes[P0 + k] ? "byte written twice" : "byte never written", i, (long)k);
        }
    }
    for (uint64_t x = 0; x < D; ++x)
        if (writes[x]) fail("write before the burst", 0, (long)x);
}

int main() {
    lnl_build_append_tables(g_t.data());
    std::mt19937_64 rng(2026);
    auto burst = [&](const std::vector<uint64_t>& lens, uint32_t dalign, uint32_t lead) {
        Burst b;
        b.dalign = dalign;
        uint64_t total = 0;
        for (auto l : lens) total += l;
        b.src.resize(lead + total + 40);
        for (auto& v : b.src) v = (uint8_t)rng();
        b.off.push_back(lead);
        for (auto l : lens) b.off.push_back(b.off.back() + l);
        run(b);
    };
    // every length 0..80 and the MTU edges, alone and in pairs, at every alignment
    for (uint32_t da = 0; da < 16; ++da)
        for (uint64_t L = 0; L <= 80; ++L) {
            burst({L}, da, (uint32_t)(rng() % 7));
            burst({L, 1400 - L}, da, 3);
            burst({3, L, 5}, da, 1);
        }
    // random bursts: mixed short / config-3 / long, at every alignment
    for (int it = 0; it < 400; ++it) {
        std::vector<uint64_t> lens(1 + rng() % 60);
        for (auto& l : lens) {
            const uint32_t k = (uint32_t)(rng() % 10);
            l = k < 3 ? rng() % 24 : (k < 8 ? 64 + rng() % 1337 : (k < 9 ? 1400 + rng() % 40 : 1000 + rng() % 9000));
        }
        burst(lens, (uint32_t)(rng() % 16), (uint32_t)(rng() % 16));
    }
    for (uint32_t da : {0u, 7u, 15u}) burst({65507, 0, 1, 65535, 12, 11, 13}, da, 5);
    printf("checked=%ld bad=%d\n", g_checked, g_bad);
    return g_bad ? 1 : 0;
}
