// broken_ring.hip -- deliberately WRONG asm load rings, kept to prove that tests/isa_check.py
// (tests/test_isa_guard.py) catches the round-1 failure class.  Never linked into the product.
//   copy_before_wait: the value of an asm load is copied (the compiler materialises `w = v`
//                     while the load is in flight) and the copy is what the wait names -- the
//                     shape of the phi copy seen in crc_regular_kernel<copy> before the fix.
//   two_branch_waits: the ring's wait is chosen on a run-time condition with TWO asm waits on
//                     two branches (the pre-fix form of LAMPI_WAIT_SEL_ASM): the compiler merges
//                     the ring registers through a phi and copies in-flight registers.
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
