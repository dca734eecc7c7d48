// C++ client of the boundary: include/lnl_crc32c_layer.hpp over
// liblnl_crc32c.so, exercised the way a net_manager would use it (outbound
// from a const shared buffer, inbound accept / drop, MTU arithmetic).  CPU
// only.  Built and run by tests/test_cpp_layer.py.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/lnl_crc32c_layer.hpp"

#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
            return 1;                                                   \
        }                                                               \
    } while (0)

int main() {
    lnl::crc32c_layer layer;
    static_assert(lnl::crc32c_layer::extra_packet_size_for_layer == 4, "extra size");
    CHECK(lnl::crc32c_layer::layer_mtu(1432) == 1428);
    CHECK(lnl_crc32c((const uint8_t*)"123456789", 9) == 0xE3069283u);

    // a MERGED datagram (property 11) in a shared, const send buffer
    std::vector<uint8_t> shared(300);
    for (size_t i = 0; i < shared.size(); ++i) shared[i] = (uint8_t)(i * 7 + 1);
    shared[0] = 11;
    const std::vector<uint8_t> before = shared;
    std::vector<uint8_t> wire(shared.size() + lnl::crc32c_layer::extra_packet_size_for_layer);
    const size_t n = layer.process_outbound_packet(shared.data(), shared.size(), wire.data(), wire.size());
    CHECK(n == shared.size() + 4);
    CHECK(shared == before);
    const uint32_t c = lnl_crc32c(shared.data(), shared.size());
    CHECK(wire[n - 4] == (uint8_t)c && wire[n - 1] == (uint8_t)(c >> 24));

    size_t len = n;
    CHECK(layer.process_inbound_packet(wire.data(), len) && len == shared.size());
    CHECK(std::memcmp(wire.data(), shared.data(), len) == 0);

    wire[5] ^= 0x10;
    len = n;
    CHECK(!layer.process_inbound_packet(wire.data(), len) && len == n);
    len = 4;
    CHECK(!layer.process_inbound_packet(wire.data(), len));
    CHECK(layer.dropped() == 2);

    bool threw = false;
    try {
        uint8_t small[8];
        layer.process_outbound_packet(shared.data(), 100, small, sizeof small);
    } catch (const std::length_error&) {
        threw = true;
    }
    CHECK(threw);

    // incremental form used for merge_data[offset..] without a copy
    const uint32_t a = lnl_crc32c(shared.data(), 100);
    CHECK(lnl_crc32c_extend(a, shared.data() + 100, 200) == c);
    std::printf("ok\n");
    return 0;
}
