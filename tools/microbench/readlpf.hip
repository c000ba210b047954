// readlpf.hip -- raw read bandwidth of the "lane per fragment" shape against the "wave per
// fragment" one.  Lane l of wave W streams fragment 64W + l from start to end, kB bytes per
// step (kB/16 dwordx4 loads at consecutive 16-byte offsets), kD steps in flight; a workgroup
// of 4 waves covers 256 consecutive fragments.  `lds` bytes of dynamic LDS cap workgroups/CU.
// Build: hipcc --offload-arch=gfx950 -O3 readlpf.hip -o readlpf
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                                \
        }                                                                                           \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int kB, int kD>
__global__ void __launch_bounds__(256) lpf(const u32x4 *__restrict__ p, unsigned nfrag, unsigned L, unsigned *out) {
    extern __shared__ unsigned lds[];
    constexpr int kQ = kB / 16;
    const unsigned lane = threadIdx.x & 63;
    if (threadIdx.x == 0) lds[0] = blockIdx.x;
    const unsigned F = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 + lane;
    if ((F & ~63u) >= nfrag) return;
    const unsigned f = F < nfrag ? F : (F & ~63u);
    const u32x4 *q = p + (size_t)f * (L / 16);
    const unsigned steps = L / kB;
    unsigned acc = 0;
    for (unsigned s = 0; s < steps; s += kD) {
        u32x4 v[kD][kQ];
#pragma unroll
        for (int d = 0; d < kD; ++d) {
            const unsigned ss = (s + d < steps) ? s + d : s;
#pragma unroll
            for (int k = 0; k < kQ; ++k) v[d][k] = q[ss * kQ + k];
        }
#pragma unroll
        for (int d = 0; d < kD; ++d)
#pragma unroll
            for (int k = 0; k < kQ; ++k) acc ^= v[d][k].x ^ v[d][k].y ^ v[d][k].z ^ v[d][k].w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc + lds[0];
}

// reference shape: one wave per fragment, lane-contiguous 64 B per 4 KiB row, 4 waves/WG
__global__ void __launch_bounds__(256) wpf(const u32x4 *__restrict__ p, unsigned nfrag, unsigned L, unsigned *out) {
    extern __shared__ unsigned lds[];
    const unsigned lane = threadIdx.x & 63;
    if (threadIdx.x == 0) lds[0] = blockIdx.x;
    const unsigned f = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (f >= nfrag) return;
    const u32x4 *q = p + (size_t)f * (L / 16) + lane * 4;
    unsigned acc = 0;
    for (unsigned r = 0; r < L / 4096; ++r) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = q[r * 256 + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc + lds[0];
}

__global__ void fill_rand(unsigned long long *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned long long z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

// wave per fragment plus one 4-byte result store per wave (the checksum kernels' output)
__global__ void __launch_bounds__(256) wpf_out(const u32x4 *__restrict__ p, unsigned nfrag, unsigned L, unsigned *out) {
    const unsigned lane = threadIdx.x & 63;
    const unsigned f = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (f >= nfrag) return;
    const u32x4 *q = p + (size_t)f * (L / 16) + lane * 4;
    unsigned acc = 0;
    for (unsigned r = 0; r < L / 4096; ++r) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = q[r * 256 + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    acc ^= __shfl_xor(acc, 1);
    if (lane == 0) out[f] = acc;
}

// kOut: 1 = 4-B store per wave (lane 0), 2 = nontemporal 4-B store, 3 = store into a 256 KiB
// ring (L2-resident), 4 = results gathered in LDS, one 16-B store per workgroup
template <int kOut>
__global__ void __launch_bounds__(256) wpf_o(const u32x4 *__restrict__ p, unsigned nfrag, unsigned L, unsigned *out) {
    __shared__ unsigned res[4];
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned f = blockIdx.x * 4 + w;
    if (f >= nfrag) return;
    const u32x4 *q = p + (size_t)f * (L / 16) + lane * 4;
    unsigned acc = 0;
    for (unsigned r = 0; r < L / 4096; ++r) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = q[r * 256 + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    acc ^= __shfl_xor(acc, 1);
    if (kOut == 1 && lane == 0) out[f] = acc;
    if (kOut == 2 && lane == 0) __builtin_nontemporal_store(acc, out + f);
    if (kOut == 3 && lane == 0) out[f & 65535] = acc;
    if (kOut == 4) {
        if (lane == 0) res[w] = acc;
        __syncthreads();
        if (threadIdx.x == 0) *(u32x4 *)(out + blockIdx.x * 4) = u32x4{res[0], res[1], res[2], res[3]};
    }
}

// interleaved fpw fragments per wave (the product's shape, 2 in flight); kOut 1 = 4-B store per
// fragment as it completes, 0 = none, 4 = per-wave results in a lane register, one store at the end
template <int kOut>
__global__ void __launch_bounds__(256) il_o(const u32x4 *__restrict__ p, unsigned nfrag, unsigned fpw, unsigned *out) {
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned b0 = blockIdx.x * 4 * fpw + w;
    unsigned mine = 0, acc0 = 0;
    for (unsigned i = 0; i < fpw; i += 2) {
        const unsigned f0 = b0 + 4 * i, f1 = b0 + 4 * (i + 1);
        const u32x4 *q0 = p + (size_t)f0 * 256 + lane * 4;
        const u32x4 *q1 = p + (size_t)f1 * 256 + lane * 4;
        u32x4 v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = q0[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[4 + k] = q1[k];
        unsigned a0 = 0, a1 = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) a0 ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
#pragma unroll
        for (int k = 0; k < 4; ++k) a1 ^= v[4 + k].x ^ v[4 + k].y ^ v[4 + k].z ^ v[4 + k].w;
        a0 ^= __shfl_xor(a0, 1);
        a1 ^= __shfl_xor(a1, 1);
        if (kOut == 1 && lane == 0) { out[f0] = a0; out[f1] = a1; }
        if (kOut == 4) { if (lane == i) mine = a0; if (lane == i + 1) mine = a1; }
        acc0 ^= a0 ^ a1;
    }
    if (kOut == 4 && lane < fpw) out[b0 + 4 * lane] = mine;
    if (kOut == 0 && acc0 == 0x9E3779B9u) out[0] = acc0;
}

// interleaved, double-buffered: kD fragments per set, the next set in flight while one is
// folded (kD..2kD fragments in flight per wave); 4-B store per fragment
template <int kD>
__global__ void __launch_bounds__(256) il_d(const u32x4 *__restrict__ p, unsigned nfrag, unsigned fpw, unsigned *out) {
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned b0 = blockIdx.x * 4 * fpw + w;
    u32x4 A[kD][4], B[kD][4];
    auto ld = [&](u32x4 (&X)[kD][4], unsigned i) {
#pragma unroll
        for (int d = 0; d < kD; ++d) {
            const unsigned ii = i + d < fpw ? i + d : i;
            const u32x4 *q = p + (size_t)(b0 + 4 * ii) * 256 + lane * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) X[d][k] = q[k];
        }
    };
    auto fold = [&](u32x4 (&X)[kD][4], unsigned i) {
#pragma unroll
        for (int d = 0; d < kD; ++d) {
            unsigned a = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) a ^= X[d][k].x ^ X[d][k].y ^ X[d][k].z ^ X[d][k].w;
            a ^= __shfl_xor(a, 1);
            if (lane == 0 && i + d < fpw) out[b0 + 4 * (i + d)] = a;
        }
    };
    ld(A, 0);
    for (unsigned i = 0; i < fpw; i += 2 * kD) {
        ld(B, i + kD < fpw ? i + kD : i);
        fold(A, i);
        if (i + 2 * kD < fpw) ld(A, i + 2 * kD);
        if (i + kD < fpw) fold(B, i + kD);
    }
}

// superblock mapping: workgroups are grouped S at a time; workgroup p of superblock s reads,
// at step i (i < nsteps), block s*S*nsteps + p + i*S (a block = 8 consecutive 4 KiB fragments,
// wave w takes fragments w and w+4 of it).  The S workgroups of a superblock run together and
// sweep one compact window instead of S separate streams.  4-B store per fragment.
__global__ void __launch_bounds__(256) il_sb(const u32x4 *__restrict__ p, unsigned nfrag, unsigned nsteps,
                                             unsigned S, unsigned *out) {
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned s = blockIdx.x / S, pp = blockIdx.x % S;
    const unsigned nblk = nfrag / 8;
    for (unsigned i = 0; i < nsteps; ++i) {
        const unsigned B = s * S * nsteps + pp + i * S;
        if (B >= nblk) break;
        const unsigned f0 = B * 8 + w, f1 = f0 + 4;
        const u32x4 *q0 = p + (size_t)f0 * 256 + lane * 4;
        const u32x4 *q1 = p + (size_t)f1 * 256 + lane * 4;
        u32x4 v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = q0[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[4 + k] = q1[k];
        unsigned a0 = 0, a1 = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) a0 ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
#pragma unroll
        for (int k = 0; k < 4; ++k) a1 ^= v[4 + k].x ^ v[4 + k].y ^ v[4 + k].z ^ v[4 + k].w;
        a0 ^= __shfl_xor(a0, 1);
        a1 ^= __shfl_xor(a1, 1);
        if (lane == 0) { out[f0] = a0; out[f1] = a1; }
    }
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 30);
    void *buf;
    unsigned *out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, (bytes / 4096) * 4 + 64));
    for (int pass = 1; pass < 2; ++pass) {
    if (pass == 0) CK(hipMemset(buf, 0x5A, bytes));
    else hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, (unsigned long long *)buf, bytes / 8);
    printf("--- data: %s\n", pass == 0 ? "memset 0x5A" : "random (splitmix64)");
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Cfg {
        int kind;  // 0 = wave per fragment; else lane per fragment: kB*10 + kD
        unsigned L;
        int lds;
    };
    std::vector<Cfg> cfgs;
    for (int fpw : {8, 16, 32}) cfgs.push_back({100 + fpw, 4096, 65536});
    for (int S : {256, 512, 1024})
        for (int fpw : {16, 32, 64, 128}) cfgs.push_back({100000 + S * 1000 + fpw, 4096, 65536});
    for (int fpw : {8, 16, 32}) cfgs.push_back({100 + fpw, 4096, 65536});
    for (const Cfg &c : cfgs) {
        const unsigned nfrag = (unsigned)(bytes / c.L);
        const unsigned fpw = c.kind >= 100000 ? c.kind % 1000 : c.kind >= 1000 ? c.kind % 100 : c.kind >= 100 ? c.kind - 100 : c.kind >= 30 ? 32 : 16;
        const unsigned S = c.kind >= 100000 ? (c.kind - 100000) / 1000 : 0;
        const unsigned grid = c.kind >= 100000 ? (nfrag + 4 * fpw - 1) / (4 * fpw) : c.kind >= 20 ? (nfrag + 4 * fpw - 1) / (4 * fpw) : c.kind <= 14 ? (nfrag + 3) / 4 : (nfrag + 255) / 256;
        auto launch = [&] {
            const u32x4 *b = (const u32x4 *)buf;
            if (c.kind >= 100000) {
                hipLaunchKernelGGL(il_sb, dim3(grid), dim3(256), c.lds, 0, b, nfrag, fpw / 2, S, out);
                return;
            }
            switch (c.kind) {
                case 11: hipLaunchKernelGGL(wpf_o<1>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 12: hipLaunchKernelGGL(wpf_o<2>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 13: hipLaunchKernelGGL(wpf_o<3>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 14: hipLaunchKernelGGL(wpf_o<4>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 20: case 30: hipLaunchKernelGGL(il_o<0>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, fpw, out); break;
                case 21: case 31: hipLaunchKernelGGL(il_o<1>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, fpw, out); break;
                case 24: case 34: hipLaunchKernelGGL(il_o<4>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, fpw, out); break;
                case 102: case 104: case 108: case 116: case 132:
                    hipLaunchKernelGGL(il_o<1>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, fpw, out); break;
                case 1108: case 1116: case 1132: case 1164:
                    hipLaunchKernelGGL(il_d<1>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, fpw, out); break;
                case 1208: case 1216: case 1232: case 1264:
                    hipLaunchKernelGGL(il_d<2>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, fpw, out); break;
                case 1408: case 1416: case 1432: case 1464:
                    hipLaunchKernelGGL(il_d<4>, dim3(grid), dim3(256), c.lds, 0, b, nfrag, fpw, out); break;
                case 1: hipLaunchKernelGGL(wpf_out, dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 0: hipLaunchKernelGGL(wpf, dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 642: hipLaunchKernelGGL((lpf<64, 2>), dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 644: hipLaunchKernelGGL((lpf<64, 4>), dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 1282: hipLaunchKernelGGL((lpf<128, 2>), dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 1283: hipLaunchKernelGGL((lpf<128, 3>), dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                case 2562: hipLaunchKernelGGL((lpf<256, 2>), dim3(grid), dim3(256), c.lds, 0, b, nfrag, c.L, out); break;
                default: fprintf(stderr, "bad kind\n"); exit(2);
            }
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
        if (c.kind >= 10)
            printf("variant %6d (fpw %3u)     L=%5u lds=%6d grid=%7u  %7.3f ms  %7.1f GB/s (%5.1f%%)\n", c.kind, c.kind >= 20 ? fpw : 1, c.L, c.lds, grid, s * 1e3,
                   bytes / s / 1e9, bytes / s / 8e10);
        else if (c.kind <= 1)
            printf("wave-per-frag%s L=%5u lds=%6d grid=%7u  %7.3f ms  %7.1f GB/s (%5.1f%%)\n", c.kind ? "+out" : "    ", c.L, c.lds, grid, s * 1e3,
                   bytes / s / 1e9, bytes / s / 8e10);
        else
            printf("lane-per-frag B=%3d D=%d L=%5u lds=%6d grid=%7u  %7.3f ms  %7.1f GB/s (%5.1f%%)\n", c.kind / 10,
                   c.kind % 10, c.L, c.lds, grid, s * 1e3, bytes / s / 1e9, bytes / s / 8e10);
        fflush(stdout);
    }
    }
    return 0;
}
