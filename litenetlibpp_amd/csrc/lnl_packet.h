// lnl_packet.h -- LiteNetLibPP's packet acceptance test, for host and device.
//
// After the CRC layer has stripped its 4 bytes, net_manager::on_message_received
// drops the datagram unless net_packet::verify() passes
// (/root/reference/src/lnl/net_manager.cpp:342-349).  verify()
// (/root/reference/include/lnl/net_packet.h:120-131):
//
//   property = data[0] & 0x1F;  property >= PACKET_PROPERTY::COUNT (18) -> false
//   headerSize = HEADER_SIZES[property]
//   fragmented = data[0] & 0x80
//   return size >= headerSize && (!fragmented || size >= headerSize + FRAGMENT_HEADER_SIZE)
//
// HEADER_SIZES (net_packet.h:20-38) has 17 initialisers for 18 properties
// (net_enums.h:47-68), so the last entry (EMPTY) is 0, and the sizes are
// indexed by the property value as listed, not by the comments beside them.
// Values from net_constants.h:16-20: HEADER_SIZE 1, CHANNELED_HEADER_SIZE 4,
// CONNECT_REQUEST_HEADER_SIZE 18, CONNECT_ACCEPT_HEADER_SIZE 15,
// FRAGMENT_HEADER_SIZE 6.
//
// Pinned against the reference's own header compiled by oracle/Makefile
// (oracle/_ref) through tests/golden/packet_verify.bin.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define LNL_PKT_HD __host__ __device__
#else
#define LNL_PKT_HD
#endif

#define LNL_PACKET_PROPERTY_COUNT 18u
#define LNL_FRAGMENT_HEADER_SIZE 6u

// HEADER_SIZES[p] as 5-bit fields: p = 0..11 in the first word, 12..17 in the second.
#define LNL_HS5(p, v) ((uint64_t)(v) << (5 * (p)))
#define LNL_HEADER_SIZES_LO                                                                                  \
    (LNL_HS5(0, 1) | LNL_HS5(1, 4) | LNL_HS5(2, 4) | LNL_HS5(3, 3) | LNL_HS5(4, 11) | LNL_HS5(5, 18) |      \
     LNL_HS5(6, 15) | LNL_HS5(7, 9) | LNL_HS5(8, 1) | LNL_HS5(9, 1) | LNL_HS5(10, 1) | LNL_HS5(11, 1))
#define LNL_HEADER_SIZES_HI \
    (LNL_HS5(0, 1) | LNL_HS5(1, 1) | LNL_HS5(2, 1) | LNL_HS5(3, 1) | LNL_HS5(4, 1) | LNL_HS5(5, 0))

// net_packet::get_header_size() for property p < 18 (branch-free, no table load)
LNL_PKT_HD inline uint32_t lnl_packet_header_size(uint32_t p) {
    const uint64_t w = p < 12u ? (uint64_t)LNL_HEADER_SIZES_LO : (uint64_t)LNL_HEADER_SIZES_HI;
    return (uint32_t)(w >> (5u * (p < 12u ? p : p - 12u))) & 31u;
}

// net_packet::verify() of a packet whose first byte is b0 and whose size is `size`
LNL_PKT_HD inline bool lnl_packet_verify_hdr(uint8_t b0, uint64_t size) {
    const uint32_t p = b0 & 0x1Fu;
    if (p >= LNL_PACKET_PROPERTY_COUNT) return false;
    const uint64_t hs = lnl_packet_header_size(p);
    const bool fragmented = (b0 & 0x80u) != 0;
    return size >= hs && (!fragmented || size >= hs + LNL_FRAGMENT_HEADER_SIZE);
}
