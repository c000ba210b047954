// copybw.hip -- device copy patterns on MI355X (read + write bandwidth, bytes counted both ways).
//   GS  : grid-stride float4 copy, fully coalesced, unroll U, persistent grid (CUs x 2..8 WGs)
//   ROW : one 4 KiB block per wave, lane-contiguous 64 B (4 x dwordx4), 256-thread WGs, fpw blocks
//         per wave interleaved across the 4 waves (the checksum kernels' shape)
//   COA : as ROW but coalesced inside the block: lane l moves 16 B at l*16 + 1024k
//   *nt : the same with non-temporal stores
// Build: hipcc --offload-arch=gfx950 -O3 copybw.hip -o copybw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                                \
        }                                                                                           \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool kNt>
__global__ void __launch_bounds__(256) cp_gs(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (kNt)
                __builtin_nontemporal_store(v[u], d + i + u * stride);
            else
                d[i + u * stride] = v[u];
        }
    }
    for (; i < n16; i += stride) d[i] = s[i];
}

// block b (4 KiB) of wave w in WG g: b = g*4*fpw + w + 4j, j < fpw; two blocks in flight per step
template <bool kCoalesced, bool kNt>
__global__ void __launch_bounds__(256) cp_row(const unsigned char *__restrict__ s, unsigned char *__restrict__ d,
                                              unsigned nblk, unsigned fpw) {
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned b0 = blockIdx.x * 4 * fpw + w;
    for (unsigned j = 0; j < fpw; j += 2) {
        unsigned ba = b0 + 4 * j, bb = b0 + 4 * (j + 1);
        if (ba >= nblk) break;
        const bool hb = (j + 1 < fpw) && bb < nblk;
        if (!hb) bb = ba;
        u32x4 va[4], vb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const size_t oa = (size_t)ba * 4096 + (kCoalesced ? lane * 16 + 1024 * k : lane * 64 + 16 * k);
            const size_t ob = (size_t)bb * 4096 + (kCoalesced ? lane * 16 + 1024 * k : lane * 64 + 16 * k);
            va[k] = *(const u32x4 *)(s + oa);
            vb[k] = *(const u32x4 *)(s + ob);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const size_t oa = (size_t)ba * 4096 + (kCoalesced ? lane * 16 + 1024 * k : lane * 64 + 16 * k);
            const size_t ob = (size_t)bb * 4096 + (kCoalesced ? lane * 16 + 1024 * k : lane * 64 + 16 * k);
            if (kNt) {
                __builtin_nontemporal_store(va[k], (u32x4 *)(d + oa));
                if (hb) __builtin_nontemporal_store(vb[k], (u32x4 *)(d + ob));
            } else {
                *(u32x4 *)(d + oa) = va[k];
                if (hb) *(u32x4 *)(d + ob) = vb[k];
            }
        }
    }
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
    unsigned char *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 0x5A, bytes));
    CK(hipMemset(d, 0, bytes));
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n16 = bytes / 16;
    const unsigned nblk = (unsigned)(bytes / 4096);
    auto run = [&](const char *name, auto launch) {
        launch();
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        const int reps = 6;
        float tot = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        const double sec = tot / 1e3 / reps;
        printf("%-28s %7.3f ms  %7.1f GB/s r+w (%5.1f%% of 8 TB/s)\n", name, sec * 1e3, 2.0 * bytes / sec / 1e9,
               2.0 * bytes / sec / 8e10);
        fflush(stdout);
    };
    char nm[64];
    for (int wpc : {2, 4, 8}) {
        snprintf(nm, sizeof nm, "GS u4 wg/cu=%d", wpc);
        run(nm, [&] { hipLaunchKernelGGL((cp_gs<4, false>), dim3(cus * wpc), dim3(256), 0, 0, (const u32x4 *)s, (u32x4 *)d, n16); });
        snprintf(nm, sizeof nm, "GS u4 nt wg/cu=%d", wpc);
        run(nm, [&] { hipLaunchKernelGGL((cp_gs<4, true>), dim3(cus * wpc), dim3(256), 0, 0, (const u32x4 *)s, (u32x4 *)d, n16); });
    }
    snprintf(nm, sizeof nm, "GS u8 wg/cu=4");
    run(nm, [&] { hipLaunchKernelGGL((cp_gs<8, false>), dim3(cus * 4), dim3(256), 0, 0, (const u32x4 *)s, (u32x4 *)d, n16); });
    for (unsigned fpw : {2u, 8u, 32u}) {
        const unsigned grid = (nblk + 4 * fpw - 1) / (4 * fpw);
        snprintf(nm, sizeof nm, "ROW fpw=%u", fpw);
        run(nm, [&] { hipLaunchKernelGGL((cp_row<false, false>), dim3(grid), dim3(256), 0, 0, s, d, nblk, fpw); });
        snprintf(nm, sizeof nm, "ROW nt fpw=%u", fpw);
        run(nm, [&] { hipLaunchKernelGGL((cp_row<false, true>), dim3(grid), dim3(256), 0, 0, s, d, nblk, fpw); });
        snprintf(nm, sizeof nm, "COA fpw=%u", fpw);
        run(nm, [&] { hipLaunchKernelGGL((cp_row<true, false>), dim3(grid), dim3(256), 0, 0, s, d, nblk, fpw); });
        snprintf(nm, sizeof nm, "COA nt fpw=%u", fpw);
        run(nm, [&] { hipLaunchKernelGGL((cp_row<true, true>), dim3(grid), dim3(256), 0, 0, s, d, nblk, fpw); });
    }
    run("hipMemcpyDtoD", [&] { CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); });
    return 0;
}
