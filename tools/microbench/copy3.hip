// copy3.hip -- copy shapes under the fused kernels' constraint: a workgroup holds tens of KiB of
// LDS tables, so it must be long-lived (the tables are staged once per workgroup) and few fit on
// a CU.  copy2.hip showed that a plain copy is fastest as the textbook one-float4-per-thread
// kernel (77.8% of 8 TB/s, short-lived 256-thread workgroups each copying a contiguous 4 KiB)
// and slows down as each wave copies more (4 KiB per wave 70%, 16 KiB 69%) or lives longer
// (persistent per-wave loops 64-70%).  Here:
//   WG<T, LDS, J, P> : T-thread workgroups with LDS bytes of static LDS; the workgroup walks
//                      `steps` consecutive super-rows of nw*J KiB (nw = T/64 waves); inside a
//                      super-row wave w moves KiB j*nw + w (j < J): at every step the workgroup's
//                      waves cover one contiguous range, 1 KiB per wave-instruction.  P: the next
//                      step's loads are issued before this step's stores.
// Payload random.  Three interleaved rounds x 4 launches per variant, 8 GiB (16 GiB moved).
// Build: hipcc --offload-arch=gfx950 -O3 copy3.hip -o copy3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
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

__global__ void fill(uint64_t *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = 0x1234567ull + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

template <int T, int LDSB, int J, bool P>
__global__ void __launch_bounds__(T) cp_wg(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n16,
                                           unsigned steps, unsigned *sink) {
    __shared__ unsigned lds[LDSB / 4 > 0 ? LDSB / 4 : 1];
    constexpr unsigned nw = T / 64;
    const unsigned w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (LDSB) {
        lds[threadIdx.x % (LDSB / 4 > 0 ? LDSB / 4 : 1)] = threadIdx.x;
        __syncthreads();
    }
    const size_t row = (size_t)nw * J * 64;  // u32x4 per step
    const size_t base = (size_t)blockIdx.x * steps * row;
    auto idx = [&](unsigned st, int j) { return base + st * row + (size_t)(j * nw + w) * 64 + lane; };
    u32x4 v[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const size_t i = idx(0, j);
        if (i < n16) v[j] = s[i];
    }
    for (unsigned st = 0; st < steps; ++st) {
        if (P) {
            u32x4 nv[J];
            const unsigned sn = st + 1 < steps ? st + 1 : st;
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const size_t i = idx(sn, j);
                if (i < n16) nv[j] = s[i];
            }
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const size_t i = idx(st, j);
                if (i < n16) d[i] = v[j];
            }
#pragma unroll
            for (int j = 0; j < J; ++j) v[j] = nv[j];
        } else {
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const size_t i = idx(st, j);
                if (i < n16) d[i] = v[j];
            }
            if (st + 1 < steps) {
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const size_t i = idx(st + 1, j);
                    if (i < n16) v[j] = s[i];
                }
            }
        }
    }
    if (LDSB && lds[(lane * 7) % (LDSB / 4 > 0 ? LDSB / 4 : 1)] == 0xFFFFFFFFu) sink[0] = 1;
}

// GM ring slots: block k's 4096 payload bytes live at slot k (stride 4176) + 72 -- 8 bytes past a
// 16-byte boundary.  G = gather (slots -> contiguous, the receive side), S = scatter (contiguous ->
// slots, the send side).  16-byte accesses at 8-byte-aligned addresses (aligned(8) vector type).
typedef u32x4 u32x4_a8 __attribute__((aligned(8)));
template <int T, int LDSB, int J, bool kGather>
__global__ void __launch_bounds__(T) cp_slot(const unsigned char *__restrict__ s, unsigned char *__restrict__ d,
                                             size_t nblk, unsigned steps, unsigned *sink) {
    __shared__ unsigned lds[LDSB / 4 > 0 ? LDSB / 4 : 1];
    constexpr unsigned nw = T / 64;
    const unsigned w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (LDSB) {
        lds[threadIdx.x % (LDSB / 4 > 0 ? LDSB / 4 : 1)] = threadIdx.x;
        __syncthreads();
    }
    // unit u = 1 KiB quarter of block u/4; the workgroup walks `steps` super-rows of nw*J units
    const size_t row = (size_t)nw * J;
    const size_t base = (size_t)blockIdx.x * steps * row;
    for (unsigned st = 0; st < steps; ++st) {
        u32x4 v[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const size_t u = base + st * row + (size_t)(j * nw + w);
            const size_t blk = u >> 2, q = u & 3;
            if (blk < nblk) {
                const size_t so = kGather ? blk * 4176 + 72 + q * 1024 + 16 * lane : u * 1024 + 16 * lane;
                v[j] = *(const u32x4_a8 *)(s + so);
            }
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const size_t u = base + st * row + (size_t)(j * nw + w);
            const size_t blk = u >> 2, q = u & 3;
            if (blk < nblk) {
                const size_t dof = kGather ? u * 1024 + 16 * lane : blk * 4176 + 72 + q * 1024 + 16 * lane;
                *(u32x4_a8 *)(d + dof) = v[j];
            }
        }
    }
    if (LDSB && lds[(lane * 7) % (LDSB / 4 > 0 ? LDSB / 4 : 1)] == 0xFFFFFFFFu) sink[0] = 1;
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
    unsigned char *s, *d;
    unsigned *sink;
    CK(hipMalloc(&s, bytes + bytes / 32));  // room for the slot layout (4176 / 4096 of the payload)
    CK(hipMalloc(&d, bytes + bytes / 32));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)s, (bytes + bytes / 32) / 8);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)d, (bytes + bytes / 32) / 8);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n16 = bytes / 16;
    const u32x4 *S = (const u32x4 *)s;
    u32x4 *D = (u32x4 *)d;
    struct V {
        std::string name;
        std::function<void()> f;
        float sum = 0;
    };
    std::vector<V> vs;
#define ADD(T, LDSB, J, P, STEPS)                                                                             \
    vs.push_back({"T=" #T " lds=" #LDSB " J=" #J " P=" #P " steps=" #STEPS, [=] {                             \
                      const size_t per = (size_t)(T / 64) * J * 64 * STEPS;                                   \
                      hipLaunchKernelGGL((cp_wg<T, LDSB, J, P>), dim3((unsigned)((n16 + per - 1) / per)),    \
                                         dim3(T), 0, 0, S, D, n16, STEPS, sink);                              \
                  }});
    // the textbook copy as a reference point (T=256 J=1 steps=1 lds=0) and its neighbours
    ADD(256, 0, 1, false, 1)
    ADD(256, 0, 1, false, 4)
    ADD(256, 0, 1, true, 4)
    ADD(256, 0, 1, true, 16)
    ADD(256, 0, 2, true, 8)
    // two 64 KiB-LDS workgroups per CU (the CRC kernels' budget)
    ADD(256, 65536, 1, true, 16)
    ADD(256, 65536, 1, true, 96)
    ADD(256, 65536, 2, true, 16)
    ADD(256, 65536, 2, true, 48)
    ADD(256, 65536, 4, true, 24)
    ADD(512, 65536, 1, true, 48)
    ADD(512, 65536, 2, true, 24)
    ADD(512, 65536, 2, true, 48)
    ADD(512, 65536, 4, true, 12)
    ADD(1024, 65536, 1, true, 24)
    ADD(1024, 65536, 2, true, 12)
    ADD(1024, 65536, 2, true, 48)
    ADD(1024, 65536, 1, false, 24)
    ADD(512, 65536, 1, false, 48)
    // ~77 KiB (the stream kernels)
    ADD(768, 79000, 1, true, 32)
    ADD(768, 79000, 2, true, 16)
    // one big workgroup per CU (LDS > 80 KiB)
    ADD(1024, 100000, 1, true, 48)
    ADD(1024, 100000, 2, true, 24)
    ADD(1024, 100000, 4, true, 12)
    const size_t nblk = bytes / 4096;
#define SLOT(T, LDSB, J, G, STEPS)                                                                              \
    vs.push_back({std::string(G ? "SLOT gather" : "SLOT scatter") + " T=" #T " lds=" #LDSB " J=" #J " steps=" #STEPS, \
                  [=] {                                                                                          \
                      const size_t per = (size_t)(T / 64) * J * STEPS;                                           \
                      hipLaunchKernelGGL((cp_slot<T, LDSB, J, G>), dim3((unsigned)((nblk * 4 + per - 1) / per)), \
                                         dim3(T), 0, 0, s, d, nblk, STEPS, sink);                                \
                  }});
    SLOT(256, 0, 1, true, 1)
    SLOT(256, 0, 1, false, 1)
    SLOT(256, 65536, 2, true, 16)
    SLOT(256, 65536, 2, false, 16)
    SLOT(512, 65536, 2, true, 24)
    SLOT(512, 65536, 2, false, 24)
    SLOT(1024, 100000, 4, true, 12)
    SLOT(1024, 100000, 4, false, 12)
    for (auto &v : vs) v.f();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const int rounds = 3, reps = 4;
    for (int r = 0; r < rounds; ++r)
        for (auto &v : vs)
            for (int k = 0; k < reps; ++k) {
                CK(hipEventRecord(e0));
                v.f();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.sum += ms;
            }
    for (auto &v : vs) {
        const double avg = v.sum / (rounds * reps) / 1e3;
        const double gb = 2.0 * bytes / avg / 1e9;
        printf("%-40s avg %7.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", v.name.c_str(), avg * 1e3, gb, gb / 80.0);
    }
    return 0;
}
