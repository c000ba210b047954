// readocc.hip -- raw 4 KiB-per-wave read bandwidth vs occupancy shape.
// One wave reads `fpw` consecutive 4 KiB fragments (lane-contiguous 64 B, 4 x dwordx4),
// non-persistent grid; `lds` bytes of dynamic LDS per block cap workgroups per CU.
// Build: hipcc --offload-arch=gfx950 -O3 readocc.hip -o readocc
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

// interleaved: the block owns wpb*fpw consecutive fragments; wave w takes w, w+wpb, ...
template <int kDepth, bool kNT = false>
__global__ void rd_il(const u32x4 *__restrict__ p, unsigned nfrag, unsigned fpw, unsigned *out) {
    extern __shared__ unsigned lds[];
    const unsigned lane = threadIdx.x & 63;
    const unsigned wpb = blockDim.x >> 6, wib = threadIdx.x >> 6;
    if (threadIdx.x == 0) lds[0] = blockIdx.x;
    unsigned acc = 0;
    const unsigned b0 = blockIdx.x * wpb * fpw + wib;
    if (b0 >= nfrag) return;
    for (unsigned i = 0; i < fpw; i += kDepth) {
        u32x4 v[kDepth][4];
#pragma unroll
        for (int d = 0; d < kDepth; ++d) {
            unsigned f = b0 + (i + d) * wpb;
            if (f >= nfrag || i + d >= fpw) f = b0;
            const u32x4 *q = p + (size_t)f * 256 + lane * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[d][k] = kNT ? __builtin_nontemporal_load(q + k) : q[k];
        }
#pragma unroll
        for (int d = 0; d < kDepth; ++d)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc ^= v[d][k].x ^ v[d][k].y ^ v[d][k].z ^ v[d][k].w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc + lds[0];
}

// XCD-grouped: workgroups 8g..8g+7 (one per XCD under round-robin dispatch) read adjacent
// 16 KiB blocks at every step; step i of workgroup b reads block (b>>3)*8*fpw + 8i + (b&7)
template <int kDepth>
__global__ void rd_xg(const u32x4 *__restrict__ p, unsigned nfrag, unsigned fpw, unsigned *out) {
    extern __shared__ unsigned lds[];
    const unsigned lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    if (threadIdx.x == 0) lds[0] = blockIdx.x;
    unsigned acc = 0;
    const unsigned b = blockIdx.x;
    const unsigned blk0 = (b >> 3) * 8 * fpw + (b & 7);
    for (unsigned i = 0; i < fpw; i += kDepth) {
        u32x4 v[kDepth][4];
#pragma unroll
        for (int d = 0; d < kDepth; ++d) {
            unsigned f = (blk0 + 8 * (i + d)) * 4 + wib;
            if (f >= nfrag || i + d >= fpw) f = 0;
            const u32x4 *q = p + (size_t)f * 256 + lane * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[d][k] = q[k];
        }
#pragma unroll
        for (int d = 0; d < kDepth; ++d)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc ^= v[d][k].x ^ v[d][k].y ^ v[d][k].z ^ v[d][k].w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc + lds[0];
}

// grid-stride non-persistent: step i of workgroup b reads 16 KiB chunk b + i*gridDim.x
template <int kDepth>
__global__ void rd_gs(const u32x4 *__restrict__ p, unsigned nfrag, unsigned fpw, unsigned *out) {
    extern __shared__ unsigned lds[];
    const unsigned lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    if (threadIdx.x == 0) lds[0] = blockIdx.x;
    unsigned acc = 0;
    const unsigned wpb = blockDim.x >> 6;
    for (unsigned i = 0; i < fpw; i += kDepth) {
        u32x4 v[kDepth][4];
#pragma unroll
        for (int d = 0; d < kDepth; ++d) {
            unsigned f = (blockIdx.x + (i + d) * gridDim.x) * wpb + wib;
            if (f >= nfrag || i + d >= fpw) f = 0;
            const u32x4 *q = p + (size_t)f * 256 + lane * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[d][k] = q[k];
        }
#pragma unroll
        for (int d = 0; d < kDepth; ++d)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc ^= v[d][k].x ^ v[d][k].y ^ v[d][k].z ^ v[d][k].w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc + lds[0];
}

template <int kDepth>
__global__ void rd(const u32x4 *__restrict__ p, unsigned nfrag, unsigned fpw, unsigned *out) {
    extern __shared__ unsigned lds[];
    const unsigned lane = threadIdx.x & 63;
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (threadIdx.x == 0) lds[0] = w;
    unsigned acc = 0;
    const unsigned f0 = w * fpw;
    if (f0 >= nfrag) return;  // whole wave past the end (grid rounding)
    for (unsigned i = 0; i < fpw; i += kDepth) {
        u32x4 v[kDepth][4];
#pragma unroll
        for (int d = 0; d < kDepth; ++d) {
            unsigned f = f0 + i + d;
            if (f >= nfrag || i + d >= fpw) f = f0;
            const u32x4 *q = p + (size_t)f * 256 + lane * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[d][k] = q[k];
        }
#pragma unroll
        for (int d = 0; d < kDepth; ++d)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc ^= v[d][k].x ^ v[d][k].y ^ v[d][k].z ^ v[d][k].w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc + lds[0];
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 30);
    const unsigned nfrag = (unsigned)(bytes / 4096);
    void *buf;
    unsigned *out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 0x5A, bytes));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Cfg {
        int block;
        unsigned fpw;
        int lds;
        int depth;
        bool il;
        bool nt;
        bool xg;
    };
    const Cfg cfgs[] = {
        {256, 1, 0, 1, false, false, false},      {256, 1, 65536, 1, false, false, false},
        {256, 16, 65536, 4, true, false, false},  {256, 32, 65536, 4, true, false, false},
        {256, 8, 65536, 4, false, true, false},   {256, 16, 65536, 4, false, true, false},
        {256, 32, 65536, 4, false, true, false},  {256, 64, 65536, 4, false, true, false},
        {256, 32, 65536, 2, false, true, false},  {256, 16, 0, 4, false, true, false},
    };
    for (const Cfg &c : cfgs) {
        const unsigned wpb = c.block / 64;
        const unsigned grid = (nfrag + wpb * c.fpw - 1) / (wpb * c.fpw);
        auto launch = [&] {
            if (!c.il && c.nt) {
                if (c.depth == 2)
                    hipLaunchKernelGGL(rd_gs<2>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                else
                    hipLaunchKernelGGL(rd_gs<4>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                return;
            }
            if (c.xg) {
                if (c.depth == 2)
                    hipLaunchKernelGGL(rd_xg<2>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                else if (c.depth == 3)
                    hipLaunchKernelGGL(rd_xg<3>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                else
                    hipLaunchKernelGGL(rd_xg<4>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                return;
            }
            if (c.il && c.nt) {
                if (c.depth == 1)
                    hipLaunchKernelGGL((rd_il<1, true>), dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                else if (c.depth == 2)
                    hipLaunchKernelGGL((rd_il<2, true>), dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                else if (c.depth == 3)
                    hipLaunchKernelGGL((rd_il<3, true>), dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                else
                    hipLaunchKernelGGL((rd_il<4, true>), dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                return;
            }
            if (c.il) {
                if (c.depth == 1)
                    hipLaunchKernelGGL(rd_il<1>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                else if (c.depth == 2)
                    hipLaunchKernelGGL(rd_il<2>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                else if (c.depth == 3)
                    hipLaunchKernelGGL(rd_il<3>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                else
                    hipLaunchKernelGGL(rd_il<4>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
                return;
            }
            if (c.depth == 1)
                hipLaunchKernelGGL(rd<1>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
            else if (c.depth == 2)
                hipLaunchKernelGGL(rd<2>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
            else
                hipLaunchKernelGGL(rd<3>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.fpw, out);
        };
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 8;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double s = ms / 1e3 / reps;
        printf("%s%s block=%4d fpw=%3u lds=%6d depth=%d grid=%7u  %7.3f ms  %7.1f GB/s (%5.1f%%)\n", c.xg ? "XG " : c.il ? "IL " : (c.nt ? "GS " : "SEQ"), (c.il && c.nt) ? "nt" : "  ",
               c.block, c.fpw, c.lds, c.depth, grid, s * 1e3, bytes / s / 1e9, bytes / s / 8e10);
        fflush(stdout);
    }
    return 0;
}
