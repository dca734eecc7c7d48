// ref_packet_verify.cpp -- a C-ABI shim over the REFERENCE's own
// lnl::net_packet (/root/reference/include/lnl/net_packet.h, header-only, with
// net_constants.h and net_enums.h), compiled where it lies by oracle/Makefile
// (target `ref`, output oracle/_ref/libref_packet.so).  Test infrastructure:
// it pins the packet acceptance test restated in
// litenetlibpp_amd/csrc/lnl_packet.h and tests/oracle.py (via the committed
// fixture tests/golden/packet_verify.bin, made by
// tests/golden/make_packet_golden.py).  No reference source is copied here.
#include <lnl/net_packet.h>

#include <cstddef>
#include <cstdint>

// net_packet::verify() on a packet holding data[0..size), exactly as
// net_manager::receive_logic leaves it before on_message_received
// (/root/reference/src/lnl/net_manager.cpp:205-222, :343): a pooled packet
// resized to the received length.
extern "C" int ref_packet_verify(const uint8_t* data, size_t size) {
    lnl::net_packet p;
    p.resize(size);
    p.copy_from(data, 0, 0, size);
    return p.verify() ? 1 : 0;
}

// net_packet::get_header_size() for property byte b (b & 0x1F < COUNT)
extern "C" int ref_packet_header_size(uint8_t b) {
    lnl::net_packet p;
    p.resize(1);
    p.copy_from(&b, 0, 0, 1);
    return (int)p.get_header_size();
}
