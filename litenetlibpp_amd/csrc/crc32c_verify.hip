// crc32c_verify.hip -- batched inbound check from whole-datagram CRCs.
//
// The large-batch verify path (lnl_crc32c_verify_csr_dev) runs the CSR pair
// kernel over the WIRE datagrams (body || LE32 CRC, contiguous, so the pair
// kernel's shared-line reuse applies) and finishes here, per datagram:
//
//   ok  = len >= 5 && CRC(wire) == 0x48674BC7
//         (CRC-32C residue: CRC(M || LE32(CRC(M))) is that constant for every
//          M, and X -> CRC(M || X) is a bijection, so the test is exactly
//          "stored CRC == CRC(body)")
//   crc = CRC(body) = step^-32(CRC(wire) ^ ~0) ^ X ^ ~0, X = the stored LE32
//         (register model: reg(M || X) = step^32(reg(M) ^ X) for 4 bytes X)
//
// matching the batch kernel's verify mode (crc 0 and ok 0 for len < 5; with
// `filter`, ok 2 for a matching CRC whose packet fails net_packet::verify).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_bitslice.h"
#include "crc32c_kernels.h"
#include "lnl_packet.h"

namespace lnl {

namespace {

constexpr uint32_t kResidue = 0x48674BC7u;

__global__ __launch_bounds__(256) void verify_from_wire_kernel(VerifyArgs a) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= a.n) return;
    const uint64_t s = a.off[i], e = a.off[i + 1];
    const uint64_t total = e - s;
    const uint32_t wire = a.wire[i];
    const bool big = total >= 5u;
    uint32_t ok = big && wire == kResidue ? 1u : 0u;
    if (ok && a.filter) ok = lnl_packet_verify_hdr(a.base[s - a.off0], total - 4u) ? 1u : 2u;
    a.ok[i] = (uint8_t)ok;
    if (a.crc) {
        uint32_t c = 0;
        if (big) {
            const uint8_t* t = a.base + (e - a.off0) - 4;
            const uint32_t x = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) |
                               ((uint32_t)t[3] << 24);
            c = lnl_step_bits(wire ^ 0xFFFFFFFFu, -32) ^ x ^ 0xFFFFFFFFu;
        }
        a.crc[i] = c;
    }
}

}  // namespace

hipError_t launch_verify_from_wire(const VerifyArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(verify_from_wire_kernel, dim3((a.n + 255u) / 256u), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
