// crc32c_device.h -- device helpers shared by the gfx950 CRC-32C kernels
// (crc32c_kernels.hip: any-layout batch kernel; crc32c_run.hip: fixed-stride
// lane-run kernel).  Internal.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_bitslice.h"

namespace lnl {
namespace dev {

constexpr int kRowU4 = 8;                   // one 128-byte row = 8 x uint4
constexpr int kBufU4 = 64 * kRowU4;         // one row buffer = 64 rows = 8 KiB
constexpr uint32_t kBufBytes = kBufU4 * 16;
constexpr int kFoldU4 = LNL_TABLE_WORDS / 4;  // 12.5 KiB of tables (crc32c_bitslice.h)

// LDS slot swizzle of a row's 16-byte pieces (bank-conflict-free row reads).
__device__ LNL_INLINE uint32_t swz(uint32_t row) { return (row >> 1) & 7u; }

__device__ LNL_INLINE uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// A global-address-space view of an integer address: a plain pointer made from
// an integer would compile to flat instructions.  (The host pass only parses
// device code.)
#if defined(__HIP_DEVICE_COMPILE__)
#define LNL_GLOBAL(T, a) reinterpret_cast<__attribute__((address_space(1))) T*>(a)
#else
#define LNL_GLOBAL(T, a) reinterpret_cast<T*>(a)
#endif

// One LDS word read in inline asm (see read_row for why asm).
__device__ LNL_INLINE uint32_t lds_read_u32(uint32_t addr) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

// 8 x ds_read_b128 of the lane's row + lgkmcnt(0), as ONE asm statement so that
// no consumer can be scheduled before the wait.  ad[k]: LDS byte address of
// piece k of the row in buffer 0; OFF selects the buffer.
template <uint32_t OFF>
__device__ LNL_INLINE void read_row(const uint32_t* ad, uint32_t* x) {
    uint4 v0, v1, v2, v3, v4, v5, v6, v7;
    asm volatile(
        "ds_read_b128 %0, %8 offset:%16\n\t"
        "ds_read_b128 %1, %9 offset:%16\n\t"
        "ds_read_b128 %2, %10 offset:%16\n\t"
        "ds_read_b128 %3, %11 offset:%16\n\t"
        "ds_read_b128 %4, %12 offset:%16\n\t"
        "ds_read_b128 %5, %13 offset:%16\n\t"
        "ds_read_b128 %6, %14 offset:%16\n\t"
        "ds_read_b128 %7, %15 offset:%16\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(v4), "=&v"(v5), "=&v"(v6), "=&v"(v7)
        : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]),
          "v"(ad[7]), "i"(OFF)
        : "memory");
    const uint4 v[8] = {v0, v1, v2, v3, v4, v5, v6, v7};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        x[4 * k + 0] = v[k].x;
        x[4 * k + 1] = v[k].y;
        x[4 * k + 2] = v[k].z;
        x[4 * k + 3] = v[k].w;
    }
}

// AND-mask one 16-byte piece of the lane's row in LDS (read, mask, write back;
// the row read that follows sees the masked bytes: LDS ops of a wave execute
// in order).  Asm for the same reason as read_row.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <uint32_t OFF>
__device__ LNL_INLINE void patch_piece(uint32_t addr, const uint32_t* m) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr), "i"(OFF)
                 : "memory");
    v.x &= m[0];
    v.y &= m[1];
    v.z &= m[2];
    v.w &= m[3];
    asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(OFF) : "memory");
}

// One 16-byte LDS piece read / written (asm, see read_row).
__device__ LNL_INLINE u32x4 lds_read_piece(uint32_t addr) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}
__device__ LNL_INLINE void lds_write_piece(uint32_t addr, u32x4 v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// One fold matrix applied to v: 8 nibble lookups in the LDS copy of the fold
// tables (inline asm for the same reason as read_row).
__device__ LNL_INLINE uint32_t fold_apply_lds(uint32_t mat_base, uint32_t v) {
    uint32_t ad[8], r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) ad[k] = mat_base + 4u * (16u * k + ((v >> (4 * k)) & 15u));
    asm volatile(
        "ds_read_b32 %0, %8\n\t"
        "ds_read_b32 %1, %9\n\t"
        "ds_read_b32 %2, %10\n\t"
        "ds_read_b32 %3, %11\n\t"
        "ds_read_b32 %4, %12\n\t"
        "ds_read_b32 %5, %13\n\t"
        "ds_read_b32 %6, %14\n\t"
        "ds_read_b32 %7, %15\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]),
          "=&v"(r[7])
        : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7])
        : "memory");
    return LNL_XOR3(LNL_XOR3(r[0], r[1], r[2]), LNL_XOR3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

}  // namespace dev
}  // namespace lnl
