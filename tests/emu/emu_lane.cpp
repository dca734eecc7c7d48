// Host-side check of the kernel's per-lane algebra (crc32c_bitslice.h) against
// the oracle, without a GPU.  Each datagram is processed exactly as one lane
// of the HIP kernel does: end-aligned 128-byte windows read from the shared
// buffer (so the first window also contains bytes of the previous datagram,
// which the masks must remove), transpose, M_128 network, finalize.
//
// Build/run: driven by tests/test_emulation.py (g++ -O2).  Exit status 0 = all
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

static uint32_t lane_crc(const uint8_t* mem, size_t mem_len, size_t start, uint32_t len) {
    const uint32_t T = (len + 127u) / 128u;
    const uint32_t pad = 128u * T - len;
    uint32_t s[32] = {0};
    for (uint32_t t = 0; t < T; ++t) {
        uint32_t x[32];
        // window bytes [start - pad + 128t, +128); bytes outside the buffer read 0xA5
        for (int w = 0; w < 32; ++w) {
            uint32_t v = 0;
            for (int b = 0; b < 4; ++b) {
                long long a = (long long)start - pad + 128ll * t + 4 * w + b;
                uint8_t byte = (a >= 0 && (size_t)a < mem_len) ? mem[a] : 0xA5;
                v |= (uint32_t)byte << (8 * b);
            }
            x[w] = v;
        }
        lnl_transpose32(x);
        uint32_t keep[4], inv0[4], inv1[4];
        lnl_first_row_masks(pad, len, keep, inv0, inv1);
        if (t == 0) lnl_apply_masks(x, keep, inv0);
        if (t == 1) lnl_apply_inv(x, inv1);
        uint32_t o[32];
        lnl_net_adv128_x(s, x, o);
        memcpy(s, o, sizeof s);
    }
    return lnl_finalize(s) ^ lnl_final_xor(len);
}

int main(int argc, char** argv) {
    const int max_len = argc > 1 ? atoi(argv[1]) : 1500;
    std::mt19937_64 rng(7);
    std::vector<uint8_t> mem(1 << 20);
    for (auto& b : mem) b = (uint8_t)rng();
    int bad = 0, checked = 0;
    // every length 0..max_len at a few offsets, incl. offset 0 (window starts before the buffer)
    for (int len = 0; len <= max_len; ++len) {
        for (size_t start : {size_t(0), size_t(1), size_t(4099), size_t(65536 + 3 * len)}) {
            uint32_t got = lane_crc(mem.data(), mem.size(), start, (uint32_t)len);
            uint32_t exp = oracle_crc32c_hw(mem.data() + start, len);
            ++checked;
            if (got != exp) {
                if (bad < 20) printf("MISMATCH len=%d start=%zu got=%08x exp=%08x\n", len, start, got, exp);
                ++bad;
            }
        }
    }
    // a few long ones, checked against the bitwise oracle
    for (uint32_t len : {4096u, 9000u, 65507u, 100003u}) {
        uint32_t got = lane_crc(mem.data(), mem.size(), 12345, len);
        uint32_t exp = oracle_crc32c_bitwise(mem.data() + 12345, len);
        ++checked;
        if (got != exp) {
            printf("MISMATCH len=%u got=%08x exp=%08x\n", len, got, exp);
            ++bad;
        }
    }
    printf("checked=%d bad=%d\n", checked, bad);
    return bad ? 1 : 0;
}
