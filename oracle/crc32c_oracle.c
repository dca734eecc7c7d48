/*
 * crc32c_oracle.c -- CPU restatement of CRC-32C, TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle for the batched CRC-32C path. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / reported CPU baseline. The product library
 * (litenetlibpp_amd/csrc) never links, loads or calls anything here.
 *
 * What it restates
 * ----------------
 * The reference (Revan600/LiteNetLibPP) has NO checksum code: its README lists
 * "Extra packet layers (and thus, no built-in crc32 and encryption)" as
 * unported (/root/reference/README.MD:35).  The path this oracle checks is the
 * packet-layer CRC that would sit at the reference's two datagram choke points:
 *   outbound  net_manager::send_raw, right before sendto
 *             (/root/reference/src/lnl/net_manager.cpp:515-523)
 *   inbound   net_manager::receive_logic, after recvfrom/resize and before
 *             on_message_received -> packet->verify()
 *             (/root/reference/src/lnl/net_manager.cpp:210-222, :342-343,
 *              /root/reference/include/lnl/net_packet.h:120-131)
 * over exactly the bytes net_packet::data()[0 .. size()) (header byte included,
 * /root/reference/include/lnl/net_packet.h:112-118).
 *
 * PARITY UNPINNED AGAINST THE REFERENCE: with no CRC in the reference there
 * is no reference output, test or golden vector for this path, and no
 * oracle/_ref build (nothing in /root/reference computes a checksum; upstream
 * C# LiteNetLib's CRC32C.cs is not available offline).
 * Parity is therefore defined by the CRC-32C standard (Castagnoli):
 *   polynomial 0x1EDC6F41, reflected 0x82F63B78, refin = refout = true,
 *   init 0xFFFFFFFF, xorout 0xFFFFFFFF, check("123456789") = 0xE3069283,
 * pinned by the RFC 3720 section B.4 (iSCSI) known-answer vectors, which the
 * tests check against three independent restatements below (bitwise,
 * slicing-by-8 tables, and the x86 SSE4.2 crc32 instruction).
 *
 * Build: oracle/Makefile -> oracle/build/libcrc32c_oracle.so
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

#define ORACLE_POLY_REFLECTED 0x82F63B78u

/* ---- 1. bitwise restatement: one reflected LFSR step per input bit ------ */
uint32_t oracle_crc32c_bitwise_extend(uint32_t crc, const uint8_t *p, size_t n)
{
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) {
        crc ^= p[i];
        for (int b = 0; b < 8; ++b)
            crc = (crc >> 1) ^ (ORACLE_POLY_REFLECTED & (0u - (crc & 1u)));
    }
    return ~crc;
}

uint32_t oracle_crc32c_bitwise(const uint8_t *p, size_t n)
{
    return oracle_crc32c_bitwise_extend(0u, p, n);
}

/* ---- 2. slicing-by-8 tables (Kounavis & Berry) -------------------------- */
static uint32_t g_tab[8][256];
static int g_tab_ready = 0;

static void oracle_init_tables(void)
{
    if (g_tab_ready) return;
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int b = 0; b < 8; ++b)
            c = (c >> 1) ^ (ORACLE_POLY_REFLECTED & (0u - (c & 1u)));
        g_tab[0][i] = c;
    }
    for (int t = 1; t < 8; ++t)
        for (uint32_t i = 0; i < 256; ++i)
            g_tab[t][i] = (g_tab[t - 1][i] >> 8) ^ g_tab[0][g_tab[t - 1][i] & 0xFFu];
    g_tab_ready = 1;
}

uint32_t oracle_crc32c_sliced_extend(uint32_t crc, const uint8_t *p, size_t n)
{
    oracle_init_tables();
    crc = ~crc;
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);      /* little-endian host (x86_64 / aarch64 LE) */
        memcpy(&hi, p + 4, 4);
        lo ^= crc;
        crc = g_tab[7][lo & 0xFF] ^ g_tab[6][(lo >> 8) & 0xFF] ^
              g_tab[5][(lo >> 16) & 0xFF] ^ g_tab[4][lo >> 24] ^
              g_tab[3][hi & 0xFF] ^ g_tab[2][(hi >> 8) & 0xFF] ^
              g_tab[1][(hi >> 16) & 0xFF] ^ g_tab[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) crc = (crc >> 8) ^ g_tab[0][(crc ^ *p++) & 0xFF];
    return ~crc;
}

uint32_t oracle_crc32c_sliced(const uint8_t *p, size_t n)
{
    return oracle_crc32c_sliced_extend(0u, p, n);
}

/* ---- 3. x86 SSE4.2 crc32 instruction (implements exactly CRC-32C) ------- */
int oracle_has_sse42(void)
{
#if defined(__x86_64__)
    unsigned a, b, c, d;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & bit_SSE4_2) != 0;
#else
    return 0;
#endif
}

#if defined(__x86_64__)
__attribute__((target("sse4.2")))
static uint32_t hw_extend(uint32_t crc, const uint8_t *p, size_t n)
{
    uint64_t c = ~crc;
    while (n >= 8) {
        uint64_t v;
        memcpy(&v, p, 8);
        c = _mm_crc32_u64(c, v);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = (uint32_t)c;
    while (n--) c32 = _mm_crc32_u8(c32, *p++);
    return ~c32;
}
#endif

/* Returns -1 in *used_hw when the host has no SSE4.2 (falls back to tables). */
uint32_t oracle_crc32c_hw_extend(uint32_t crc, const uint8_t *p, size_t n)
{
#if defined(__x86_64__)
    static int has = -1;
    if (has < 0) has = oracle_has_sse42();
    if (has) return hw_extend(crc, p, n);
#endif
    return oracle_crc32c_sliced_extend(crc, p, n);
}

uint32_t oracle_crc32c_hw(const uint8_t *p, size_t n)
{
    return oracle_crc32c_hw_extend(0u, p, n);
}

/* ---- batch drivers (the CPU baseline + full-size checker) --------------- *
 * Fixed stride: out[i] = CRC32C(base + i*stride, len)      (BASELINE configs 2/4)
 * CSR:          out[i] = CRC32C(base + off[i], off[i+1]-off[i])   (config 3)
 * nthreads <= 0 -> all OpenMP threads.  Returns the thread count used.
 */
int oracle_batch_fixed(const uint8_t *base, uint64_t stride, uint32_t len,
                       uint64_t n, uint32_t *out, int nthreads)
{
    oracle_init_tables();
    int used = 1;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    used = nthreads;
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i)
        out[i] = oracle_crc32c_hw_extend(0u, base + (uint64_t)i * stride, len);
    return used;
}

int oracle_batch_csr(const uint8_t *base, const uint64_t *off, uint64_t n,
                     uint32_t *out, int nthreads)
{
    oracle_init_tables();
    int used = 1;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    used = nthreads;
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i)
        out[i] = oracle_crc32c_hw_extend(0u, base + off[i], (size_t)(off[i + 1] - off[i]));
    return used;
}

/* Bitwise batch (slow, independent of the table/HW paths): used by tests on
 * small inputs so that a table bug cannot hide behind itself. */
void oracle_batch_csr_bitwise(const uint8_t *base, const uint64_t *off, uint64_t n,
                              uint32_t *out)
{
    for (uint64_t i = 0; i < n; ++i)
        out[i] = oracle_crc32c_bitwise(base + off[i], (size_t)(off[i + 1] - off[i]));
}

/* ---- SURVEY.md section 8(d) synthetic input --------------------------------
 * mt19937_64 (Matsumoto & Nishimura 2000; the standard C++ engine: n = 312,
 * m = 156, matrix 0xB5026F5AA96619E9, tempering u=29 d=0x5555555555555555
 * s=17 b=0x71D67FFFEDA60000 t=37 c=0xFFF7EEE000000000 l=43, seeding with
 * 6364136223846793005) outputs stored little-endian: the recipe SURVEY.md
 * pins with out[0] = CRC-32C(first 1400 bytes of seed 42) = 0xD26C5CFE. */
void oracle_fill_mt19937_64(uint64_t seed, uint64_t *out, size_t nwords)
{
    uint64_t mt[312];
    mt[0] = seed;
    for (int i = 1; i < 312; ++i)
        mt[i] = 6364136223846793005ull * (mt[i - 1] ^ (mt[i - 1] >> 62)) + (uint64_t)i;
    int idx = 312;
    for (size_t k = 0; k < nwords; ++k) {
        if (idx >= 312) {
            for (int i = 0; i < 312; ++i) {
                const uint64_t x = (mt[i] & 0xFFFFFFFF80000000ull) | (mt[(i + 1) % 312] & 0x7FFFFFFFull);
                uint64_t xa = x >> 1;
                if (x & 1u) xa ^= 0xB5026F5AA96619E9ull;
                mt[i] = mt[(i + 156) % 312] ^ xa;
            }
            idx = 0;
        }
        uint64_t y = mt[idx++];
        y ^= (y >> 29) & 0x5555555555555555ull;
        y ^= (y << 17) & 0x71D67FFFEDA60000ull;
        y ^= (y << 37) & 0xFFF7EEE000000000ull;
        y ^= y >> 43;
        out[k] = y; /* x86-64 / gfx950 hosts are little-endian */
    }
}
