// broken_ring.hip -- deliberately WRONG asm load rings, kept to prove that tests/isa_check.py
// (tests/test_isa_guard.py) catches the round-1 failure class.  Never linked into the product.
//   copy_before_wait: the value of an asm load is copied (the compiler materialises `w = v`
//                     while the load is in flight) and the copy is what the wait names -- the
//                     shape of the phi copy seen in crc_regular_kernel<copy> before the fix.
//   two_branch_waits: the ring's wait is chosen on a run-time condition with TWO asm waits on
//                     two branches (the pre-fix form of LAMPI_WAIT_SEL_ASM): the compiler merges
//                     the ring registers through a phi and copies in-flight registers.
//   refill_skipped:   round 4's ring drain in crc_regular_kernel: no refill past the
//                     last task -- the slot's reload skipped under a branch -- and the wait then
//                     drains (vmcnt(0)) or not on two branches.  Its GPU run failed parity
//                     (test_regular_batches_every_schedule[32768-sum]); rebuilt on the CPU in round 5,
//                     the regular kernel in this form shows 603 touches of in-flight registers
//                     (v_mov copies right after the loads) in all five instantiations.
// Build (device assembly only): hipcc --offload-arch=gfx950 --cuda-device-only -S -O3 broken_ring.hip
#include <hip/hip_runtime.h>

#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const uint8_t gbyte;

__device__ __forceinline__ u32x4 issue(gbyte *p) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(v) : "v"(p) : "memory");
    return v;
}

__global__ void copy_before_wait(const uint8_t *src, u32x4 *out, int n) {
    gbyte *p = (gbyte *)(src + 16 * threadIdx.x);
    u32x4 v = issue(p);
    u32x4 w = v;  // still in flight: the copy reads garbage
    asm volatile("s_waitcnt vmcnt(0) ; lampi-wait %0" : "+v"(w) : : "memory");
    out[threadIdx.x] = w + v;
}

__global__ void two_branch_waits(const uint8_t *src, u32x4 *out, int n, int first) {
    gbyte *p = (gbyte *)(src + 16 * threadIdx.x);
    u32x4 a = issue(p), b = issue(p + 4096);
    u32x4 acc = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        u32x4 c = issue(p + 8192 * (i + 2));
        if (i == 0 && first)
            asm volatile("s_waitcnt vmcnt(1) ; lampi-wait %0" : "+v"(a) : : "memory");
        else
            asm volatile("s_waitcnt vmcnt(2) ; lampi-wait %0" : "+v"(a) : : "memory");
        acc += a;
        a = b;
        b = c;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[threadIdx.x] = acc + a + b;
}

__global__ void refill_skipped(const uint8_t *src, u32x4 *out, int n) {
    gbyte *p = (gbyte *)(src + 16 * threadIdx.x);
    u32x4 r0 = issue(p), r1 = issue(p + 4096), r2 = issue(p + 8192);
    u32x4 acc = {0, 0, 0, 0};
    bool drain = false;
    for (int i = 0; i < n; i += 3) {
#define STEP(R, K)                                                                       \
        if (drain)                                                                       \
            asm volatile("s_waitcnt vmcnt(0) ; lampi-wait %0" : "+v"(R) : : "memory");   \
        else                                                                             \
            asm volatile("s_waitcnt vmcnt(2) ; lampi-wait %0" : "+v"(R) : : "memory");   \
        acc += R;                                                                        \
        if (i + (K) + 3 < n)                                                             \
            R = issue(p + 4096 * (i + (K) + 3));                                         \
        else                                                                             \
            drain = true;
        STEP(r0, 0)
        STEP(r1, 1)
        STEP(r2, 2)
#undef STEP
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[threadIdx.x] = acc;
}
