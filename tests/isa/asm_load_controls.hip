// Controls for tests/isa_scan.py (CPU test; compiled for gfx950 into a code
// object and disassembled, never run): kernels that touch an inline-asm load's
// destination register before the wait that covers it -- the pattern behind
// the round-4 three-row span fault -- and the same kernels with
// the wait in place.  The asm loads are invisible to the compiler, which is
// exactly why nothing but such a scan can see these hazards.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ inline void asm_load(uint32_t& v, const uint32_t* p) {
    asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
}

// the value is read before the wait: stale data
extern "C" __global__ void bad_read_before_wait(const uint32_t* p, uint32_t* o) {
    uint32_t v;
    asm_load(v, p + threadIdx.x);
    o[threadIdx.x] = v + 1u;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// the value is copied to an accumulation register before the wait (what the
// compiler does when it runs out of VGPRs); the load lands afterwards in a
// register that may already hold something else
extern "C" __global__ void bad_agpr_copy_before_wait(const uint32_t* p, uint32_t* o) {
    uint32_t v, w;
    asm_load(v, p + threadIdx.x);
    asm volatile("v_accvgpr_write_b32 a0, %0" ::"v"(v));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("v_accvgpr_read_b32 %0, a0" : "=v"(w));
    o[threadIdx.x] = w;
}

// counted wait one short: two loads in flight, vmcnt(1) covers the first only,
// and the second is read
extern "C" __global__ void bad_count_short(const uint32_t* p, uint32_t* o) {
    uint32_t a, b;
    asm_load(a, p + threadIdx.x);
    asm_load(b, p + 64 + threadIdx.x);
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    o[threadIdx.x] = a + b;
}

// a loop whose next load goes out at the bottom and is waited for at the top
// only on some iterations
extern "C" __global__ void bad_loop_skipped_wait(const uint32_t* p, uint32_t* o, int n) {
    uint32_t v, acc = 0;
    asm_load(v, p + threadIdx.x);
    for (int i = 0; i < n; ++i) {
        if (i & 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc += v;
        asm_load(v, p + threadIdx.x + 64 * i);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    o[threadIdx.x] = acc + v;
}

extern "C" __global__ void good_wait_then_read(const uint32_t* p, uint32_t* o) {
    uint32_t v;
    asm_load(v, p + threadIdx.x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    o[threadIdx.x] = v + 1u;
}

// a two-deep counted pipeline, every value pinned behind its wait (the wait
// names it as an operand: a use may otherwise be scheduled above an asm
// statement that does not name its register)
extern "C" __global__ void good_counted_pipeline(const uint32_t* p, uint32_t* o, int n) {
    uint32_t a, b, acc = 0;
    asm_load(a, p + threadIdx.x);
    asm_load(b, p + 64 + threadIdx.x);
    for (int i = 0; i < n; ++i) {
        asm volatile("s_waitcnt vmcnt(1)" : "+v"(a), "+v"(b)::"memory");   // a landed
        acc += a;
        asm_load(a, p + threadIdx.x + 128 * i);
        asm volatile("s_waitcnt vmcnt(1)" : "+v"(a), "+v"(b)::"memory");   // b landed
        acc ^= b;
        asm_load(b, p + 64 + threadIdx.x + 128 * i);
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b)::"memory");
    o[threadIdx.x] = acc + a + b;
}

// the uniform flag pattern the structurizer emits for if (c) wait(N) else
// wait(0) after if (c) issue(N loads): correlated branches on one SGPR mask
extern "C" __global__ void good_flagged_waits(const uint32_t* p, uint32_t* o, int c) {
    uint32_t t = 0, v0 = 0, v1 = 0;
    asm_load(t, p + threadIdx.x);
    const bool on = c > 3;
    if (on) {
        asm_load(v0, p + 64 + threadIdx.x);
        asm_load(v1, p + 128 + threadIdx.x);
    }
    if (on)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    o[threadIdx.x] = t;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    o[64 + threadIdx.x] = v0 + v1;
}
