// lnl_dispatch.hip -- the packets a filtered burst delivers (SURVEY.md 8(f)
// item 3): every accepted datagram is one packet (its CRC stripped), except a
// MERGED container, which is cut into the packets it carries.
//
// The container walk restates net_peer::process_packet's MERGED case
// (/root/reference/src/lnl/net_peer.cpp:164-187), the sender side being
// net_peer::send_user_data / send_merged (:446-486): after the 1-byte header,
// [u16 LE size][packet of `size` bytes] repeated; each packet must pass
// net_packet::verify() (lnl_packet.h) or the walk stops there.
//
//   pos = HEADER_SIZE (1)
//   while pos < size:
//       if pos + 2 > size: stop                       (*)
//       L = u16 at pos; pos += 2
//       if L > size - pos: stop                       (*)
//       if !verify(packet[pos .. pos+L)): stop         (L = 0 fails: no header byte)
//       emit [pos, pos+L); pos += L
//
// (*) The reference bounds both reads by its pooled buffer's capacity
// (buffer_size(), 2048 for received packets), not by the datagram, and reads
// stale pool bytes past the datagram's end; a container that runs past its
// datagram stops here instead.  Well-formed containers -- all send_merged
// produces -- split identically.
//
// A nested container is delivered as one packet (the reference's
// process_packet would cut it again); send_merged never nests.
//
// Two launches around a device-wide exclusive scan (hipCUB): count the packets
// of every datagram, then emit them in datagram order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "crc32c_kernels.h"
#include "lnl_packet.h"

namespace lnl {

namespace {

constexpr uint32_t kMergedProperty = 12;  // PACKET_PROPERTY::MERGED, net_enums.h:60

// Walk datagram i; for each delivered packet call emit(start, len) (start
// relative to base).  Returns the number of packets.
template <typename F>
__device__ inline uint32_t walk(const DispatchArgs& a, uint32_t i, F&& emit) {
    if (a.status[i] != 1u) return 0;  // LNL_INBOUND_ACCEPT only
    const uint64_t s = a.off[i] - a.off0;
    const uint32_t size = (uint32_t)(a.off[i + 1] - a.off[i]) - 4u;  // CRC stripped
    const uint8_t* p = a.base + s;
    if ((p[0] & 0x1Fu) != kMergedProperty) {
        emit(s, size);
        return 1;
    }
    uint32_t pos = 1, c = 0;
    while (pos < size) {
        if (pos + 2u > size) break;
        const uint32_t L = (uint32_t)p[pos] | ((uint32_t)p[pos + 1] << 8);
        pos += 2;
        if (L > size - pos) break;
        if (L == 0u || !lnl_packet_verify_hdr(p[pos], L)) break;
        emit(s + pos, L);
        pos += L;
        ++c;
    }
    return c;
}

__global__ __launch_bounds__(256) void dispatch_count_kernel(DispatchArgs a) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= a.n) return;
    a.counts[i] = walk(a, i, [](uint64_t, uint32_t) {});
}

__global__ __launch_bounds__(256) void dispatch_emit_kernel(DispatchArgs a) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= a.n) return;
    uint32_t k = a.first[i];
    const uint32_t c = walk(a, i, [&](uint64_t start, uint32_t len) {
        if (k < a.cap) {
            a.pkt_start[k] = start;
            a.pkt_len[k] = len;
            a.pkt_parent[k] = i;
        }
        ++k;
    });
    if (i + 1u == a.n) *a.total = a.first[i] + c;
}

}  // namespace

size_t dispatch_scan_bytes(uint32_t n) {
    size_t bytes = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n) !=
        hipSuccess)
        return 0;
    return bytes;
}

hipError_t launch_dispatch(const DispatchArgs& a, void* scan_tmp, size_t scan_bytes, hipStream_t stream) {
    const dim3 grid((a.n + 255u) / 256u);
    hipLaunchKernelGGL(dispatch_count_kernel, grid, dim3(256), 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, a.counts, a.first, (int)a.n, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(dispatch_emit_kernel, grid, dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
