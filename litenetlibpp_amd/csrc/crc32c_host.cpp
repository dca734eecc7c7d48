// crc32c_host.cpp -- the per-datagram CPU side of the C ABI (include/lnl_crc32c.h).
//
// This is PRODUCT code for the reference's one-datagram-per-syscall hook sites
// (net_manager::send_raw before sendto, /root/reference/src/lnl/net_manager.cpp:515-523;
// receive_logic after recvfrom, :210-222), where a GPU round trip per datagram
// would cost far more than the ~0.2 us a CPU CRC of <= 1432 bytes takes
// (SURVEY.md section 3d).  It is not a fallback for the batch entry points:
// those only ever launch gfx950 kernels.
//
// Stateless and reentrant: send_raw is called from the receive, logic and user
// threads (/root/reference/src/lnl/net_manager.cpp:106-107).  Uses the SSE4.2
// crc32 instruction (which computes exactly CRC-32C) when the CPU has it, else
// slicing-by-8 tables built at compile time.
#include <errno.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <array>

#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

#include "../../include/lnl_crc32c.h"
#include "lnl_packet.h"

namespace {

constexpr uint32_t kPoly = 0x82F63B78u;

struct Tables {
    uint32_t t[8][256];
};

constexpr Tables make_tables() {
    Tables T{};
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
        T.t[0][i] = c;
    }
    for (int k = 1; k < 8; ++k)
        for (uint32_t i = 0; i < 256; ++i)
            T.t[k][i] = (T.t[k - 1][i] >> 8) ^ T.t[0][T.t[k - 1][i] & 0xFFu];
    return T;
}

constexpr Tables kTab = make_tables();

uint32_t sw_update(uint32_t c, const uint8_t* p, size_t n) {
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = kTab.t[7][lo & 0xFF] ^ kTab.t[6][(lo >> 8) & 0xFF] ^ kTab.t[5][(lo >> 16) & 0xFF] ^
            kTab.t[4][lo >> 24] ^ kTab.t[3][hi & 0xFF] ^ kTab.t[2][(hi >> 8) & 0xFF] ^
            kTab.t[1][(hi >> 16) & 0xFF] ^ kTab.t[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = (c >> 8) ^ kTab.t[0][(c ^ *p++) & 0xFF];
    return c;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t hw_update(uint32_t c, const uint8_t* p, size_t n) {
    uint64_t c64 = c;
    // three interleaved streams hide the crc32 instruction's 3-cycle latency
    // for long inputs; datagrams (<= 1432 B) mostly take the simple loop
    while (n >= 8) {
        uint64_t v;
        memcpy(&v, p, 8);
        c64 = _mm_crc32_u64(c64, v);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = (uint32_t)c64;
    while (n--) c32 = _mm_crc32_u8(c32, *p++);
    return c32;
}

bool cpu_has_sse42() {
    unsigned a, b, c, d;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
    return (c & bit_SSE4_2) != 0;
}
#endif

uint32_t update(uint32_t c, const uint8_t* p, size_t n) {
#if defined(__x86_64__)
    static const bool hw = cpu_has_sse42();
    if (hw) return hw_update(c, p, n);
#endif
    return sw_update(c, p, n);
}

}  // namespace

extern "C" uint32_t lnl_crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
    if (n == 0) return crc;
    return ~update(~crc, p, n);
}

extern "C" uint32_t lnl_crc32c(const uint8_t* p, size_t n) { return lnl_crc32c_extend(0u, p, n); }

extern "C" int64_t lnl_crc32c_layer_outbound(const uint8_t* data, size_t offset, size_t length,
                                             uint8_t* dst, size_t dst_cap) {
    if ((!data && length) || !dst) return -22;
    if (dst_cap < length + LNL_CRC32C_LAYER_EXTRA) return -22;
    const uint8_t* src = data + offset;
    if (length) memcpy(dst, src, length);
    const uint32_t c = lnl_crc32c(src, length);
    dst[length + 0] = (uint8_t)(c);
    dst[length + 1] = (uint8_t)(c >> 8);
    dst[length + 2] = (uint8_t)(c >> 16);
    dst[length + 3] = (uint8_t)(c >> 24);
    return (int64_t)(length + LNL_CRC32C_LAYER_EXTRA);
}

extern "C" int64_t lnl_crc32c_layer_inbound(const uint8_t* data, size_t length) {
    // header byte + CRC is the minimum (upstream: length < HeaderSize + CRC32C.ChecksumSize)
    if (!data || length < 1 + LNL_CRC32C_LAYER_EXTRA) return -1;
    const size_t body = length - LNL_CRC32C_LAYER_EXTRA;
    const uint32_t stored = (uint32_t)data[body] | ((uint32_t)data[body + 1] << 8) |
                            ((uint32_t)data[body + 2] << 16) | ((uint32_t)data[body + 3] << 24);
    return lnl_crc32c(data, body) == stored ? (int64_t)body : -1;
}

extern "C" int lnl_packet_verify(const uint8_t* data, size_t size) {
    if (!data || size == 0) return 0;
    return lnl_packet_verify_hdr(data[0], size) ? 1 : 0;
}

extern "C" int lnl_inbound_status(const uint8_t* data, size_t length) {
    const int64_t body = lnl_crc32c_layer_inbound(data, length);
    if (body < 0) return LNL_INBOUND_DROP_CRC;
    return lnl_packet_verify(data, (size_t)body) ? LNL_INBOUND_ACCEPT : LNL_INBOUND_MALFORMED;
}

extern "C" int lnl_xor_layer(uint8_t* data, size_t length, const uint8_t* key, size_t key_len) {
    if (!key || key_len == 0 || key_len > LNL_XOR_MAX_KEY) return -EINVAL;
    if (length && !data) return -EINVAL;
    for (size_t i = 0, k = 0; i < length; ++i) {
        data[i] ^= key[k];
        if (++k == key_len) k = 0;
    }
    return 0;
}
