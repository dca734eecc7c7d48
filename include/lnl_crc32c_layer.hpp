// lnl_crc32c_layer.hpp -- C++ packet layer over the C ABI (lnl_crc32c.h).
//
// Mirrors upstream LiteNetLib's PacketLayerBase / Crc32cLayer, which
// LiteNetLibPP lists as unported ("Extra packet layers (and thus, no built-in
// crc32 and encryption)", /root/reference/README.MD:35), in the reference's
// naming style (snake_case, lnl:: namespace, net_address endpoints).  A
// net_manager holds one of these and calls it at its two datagram choke points:
//
//   outbound: net_manager::send_raw (/root/reference/src/lnl/net_manager.cpp:515)
//             -> process_outbound_packet(data + offset, length, scratch)
//             and sendto(scratch, new_length) instead of data (send_raw's buffer
//             is const and may be a shared per-peer buffer: net_peer.cpp:482,
//             :575, :534 -- never append in place)
//   inbound:  net_manager::receive_logic after packet->resize(size)
//             (/root/reference/src/lnl/net_manager.cpp:220)
//             -> if (!process_inbound_packet(data, size)) { pool_recycle; continue; }
//             then on_message_received (:222) sees the datagram without its CRC.
//   MTU:      every POSSIBLE_MTU entry (net_constants.h:29-39) minus
//             extra_packet_size_for_layer, so the 1432-byte MTU probe still fits
//             recvfrom's MAX_PACKET_SIZE buffer (net_manager.cpp:208-211).
//
// Batched inbound verification (a recvmmsg-style burst of datagrams already in
// device memory) goes through verify_batch_device().
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "lnl_crc32c.h"

namespace lnl {

class crc32c_layer {
public:
    // upstream ExtraPacketSizeForLayer
    static constexpr size_t extra_packet_size_for_layer = LNL_CRC32C_LAYER_EXTRA;

    // Effective MTU when the layer is on.
    static constexpr int32_t layer_mtu(int32_t mtu) { return mtu - (int32_t)extra_packet_size_for_layer; }

    // Outbound (upstream ProcessOutBoundPacket): writes data[0..length) and its
    // LE32 CRC-32C into `out` (capacity out_cap).  Returns the new length.
    size_t process_outbound_packet(const uint8_t* data, size_t length, uint8_t* out, size_t out_cap) const {
        const int64_t r = lnl_crc32c_layer_outbound(data, 0, length, out, out_cap);
        if (r < 0) throw std::length_error("crc32c_layer: output buffer too small");
        return (size_t)r;
    }

    // Inbound (upstream ProcessInboundPacket): true and length reduced by 4 if
    // the datagram carries a valid CRC; false (drop silently, counted) if it is
    // shorter than header + CRC or the CRC does not match.
    bool process_inbound_packet(const uint8_t* data, size_t& length) {
        const int64_t r = lnl_crc32c_layer_inbound(data, length);
        if (r < 0) {
            ++m_dropped;
            return false;
        }
        length = (size_t)r;
        return true;
    }

    // Batched inbound check of n datagrams in device memory (CSR offsets,
    // trailing CRC included): d_ok[i] = 1 if datagram i passes.  Stream-ordered.
    static void verify_batch_device(const uint8_t* d_base, const uint64_t* d_off, uint32_t n, uint8_t* d_ok,
                                    void* hip_stream) {
        const int rc = lnl_crc32c_verify_csr_dev(d_base, d_off, n, d_ok, nullptr, hip_stream);
        if (rc != 0) throw std::runtime_error(std::string("crc32c_layer: ") + lnl_crc32c_last_error());
    }

    // "checksum: bad" counter (upstream logs each drop).
    uint64_t dropped() const { return m_dropped; }

private:
    uint64_t m_dropped = 0;
};

}  // namespace lnl
