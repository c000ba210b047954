// ring_nt.hip -- config B's load schedule without the checksum (round 6): crc_regular_kernel's ring (asm-issued
// global_load_dwordx4, three slots, two chains per wave, 12 items of two 4 KiB rows per wave, 256-thread workgroups
// holding 66 KB of LDS: two per CU) over 16 GiB and 1 GiB, the rows XOR-folded into one word per wave, in four
// layouts: lane-contiguous 64-byte pieces (the product) or coalesced rows (lane l the 16-byte chunks at 16 l + 1024 q:
// 1 KiB per instruction), each with and without the non-temporal bit.  Plain reads measured 86.9% coalesced + nt in
// 128-thread workgroups, 50.6% lane-contiguous + nt (launch_size.hip).  Three interleaved rounds, 20 launches each.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 ring_nt.hip -o ring_nt
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                       \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) {                                     \
            std::printf("HIP %d at %d\n", (int)e_, __LINE__);       \
            std::exit(1);                                           \
        }                                                           \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const uint8_t gbyte;
struct Row {
    u32x4 q[4];
};

template <int kS, bool kNt>
__device__ __forceinline__ void issue_row(gbyte *p, Row &r) {
    if constexpr (kNt)
        asm volatile(
            "global_load_dwordx4 %0, %4, off nt\n\t"
            "global_load_dwordx4 %1, %4, off offset:%5 nt\n\t"
            "global_load_dwordx4 %2, %4, off offset:%6 nt\n\t"
            "global_load_dwordx4 %3, %4, off offset:%7 nt"
            : "=&v"(r.q[0]), "=&v"(r.q[1]), "=&v"(r.q[2]), "=&v"(r.q[3])
            : "v"(p), "n"(kS), "n"(2 * kS), "n"(3 * kS)
            : "memory");
    else
        asm volatile(
            "global_load_dwordx4 %0, %4, off\n\t"
            "global_load_dwordx4 %1, %4, off offset:%5\n\t"
            "global_load_dwordx4 %2, %4, off offset:%6\n\t"
            "global_load_dwordx4 %3, %4, off offset:%7"
            : "=&v"(r.q[0]), "=&v"(r.q[1]), "=&v"(r.q[2]), "=&v"(r.q[3])
            : "v"(p), "n"(kS), "n"(2 * kS), "n"(3 * kS)
            : "memory");
}

struct Slot {
    Row x[2];
};

template <int N>
__device__ __forceinline__ void wait_slot(Slot &b) {
    asm volatile("s_waitcnt vmcnt(%8) ; lampi-wait %0 %1 %2 %3 %4 %5 %6 %7"
                 : "+v"(b.x[0].q[0]), "+v"(b.x[0].q[1]), "+v"(b.x[0].q[2]), "+v"(b.x[0].q[3]), "+v"(b.x[1].q[0]),
                   "+v"(b.x[1].q[1]), "+v"(b.x[1].q[2]), "+v"(b.x[1].q[3])
                 : "n"(N)
                 : "memory");
}

// items of two 4 KiB rows (a pair of fragments); item i of wave w of workgroup b: b * 4 * fpw + w + 4 j
template <bool kCoal, bool kNt>
__global__ void __launch_bounds__(256) ring(const uint8_t *__restrict__ base, unsigned nitems, unsigned fpw,
                                            unsigned *out) {
    __shared__ uint32_t lds[66048 / 4];
    constexpr int kS = kCoal ? 1024 : 16;
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned f0 = blockIdx.x * 4 * fpw + wave;
    const unsigned nfr = f0 < nitems ? min(fpw, (nitems - f0 + 3) / 4) : 0u;
    const unsigned lane_off = kCoal ? lane * 16 : lane * 64;
    // steps: (group g of two items, row r): chain c reads item 2g + c, row r
    const unsigned ngrp = (nfr + 1) / 2, nsteps = 2 * ngrp;
    auto ptr = [&](unsigned step, int c) -> gbyte * {
        const unsigned s = min(step, nsteps ? nsteps - 1 : 0u);
        const unsigned g = s / 2, r = s % 2, j = min(2 * g + c, nfr ? nfr - 1 : 0u);
        return (gbyte *)(base + ((size_t)(f0 + 4 * j) * 2 + r) * 4096 + lane_off);
    };
    Slot ring[3];
    unsigned acc = 0;
    if (nfr == 0) return;
    for (int q = 0; q < 3; ++q)
        for (int c = 0; c < 2; ++c) issue_row<kS, kNt>(ptr(q, c), ring[q].x[c]);
    lds[threadIdx.x] = 0;  // (the LDS stays allocated: two workgroups per CU, as the product)
    unsigned step = 0;
#define STEP(S)                                                              \
    {                                                                        \
        wait_slot<16>(ring[S]);                                              \
        for (int c = 0; c < 2; ++c)                                          \
            for (int k = 0; k < 4; ++k) {                                    \
                const u32x4 v = ring[S].x[c].q[k];                           \
                acc ^= v.x ^ v.y ^ v.z ^ v.w;                                \
            }                                                                \
        if (step + 1 >= nsteps) break;                                       \
        for (int c = 0; c < 2; ++c) issue_row<kS, kNt>(ptr(step + 3, c), ring[S].x[c]); \
        ++step;                                                              \
    }
    for (;;) {
        STEP(0)
        STEP(1)
        STEP(2)
    }
#undef STEP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc ^= lds[(threadIdx.x + 1) & 255];
    for (int o = 32; o >= 1; o >>= 1) acc ^= __shfl_xor(acc, o);
    if (lane == 0) out[blockIdx.x * 4 + wave] = acc;
}

int main() {
    const size_t max_bytes = 16ull << 30;
    uint8_t *buf;
    unsigned *out;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMemset(buf, 0x5A, max_bytes));
    CK(hipMalloc(&out, (max_bytes / 4096) * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[4] = {"pieces", "pieces_nt", "coal", "coal_nt"};
    const unsigned gib[2] = {1, 16};
    for (int round = 0; round < 3; ++round) {
        for (int k = 0; k < 4; ++k) {
            for (int s = 0; s < 2; ++s) {
                const size_t bytes = (size_t)gib[s] << 30;
                const unsigned nitems = (unsigned)(bytes / 8192), fpw = 12;
                const dim3 g((nitems + 4 * fpw - 1) / (4 * fpw));
                auto launch = [&] {
                    if (k == 0) hipLaunchKernelGGL((ring<false, false>), g, dim3(256), 0, 0, buf, nitems, fpw, out);
                    if (k == 1) hipLaunchKernelGGL((ring<false, true>), g, dim3(256), 0, 0, buf, nitems, fpw, out);
                    if (k == 2) hipLaunchKernelGGL((ring<true, false>), g, dim3(256), 0, 0, buf, nitems, fpw, out);
                    if (k == 3) hipLaunchKernelGGL((ring<true, true>), g, dim3(256), 0, 0, buf, nitems, fpw, out);
                };
                for (int i = 0; i < 5; ++i) launch();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < 20; ++i) launch();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double t = ms * 1e3 / 20;
                std::printf("round %d %-10s %2u GiB %9.1f us  %5.1f%%\n", round, names[k], gib[s], t,
                            bytes / (t * 1e-6) / 8e12 * 100);
                std::fflush(stdout);
            }
        }
    }
    return 0;
}
