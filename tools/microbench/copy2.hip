// copy2.hip -- what a device copy can reach on MI355X (read + write bytes counted), to price the
// fused copy+checksum kernels against the chip and not against one microbenchmark shape.
//   RD   : read-only, one 4 KiB block per wave (the CRC kernels' best read shape), sink = xor
//   WR   : write-only, one 4 KiB block per wave, coalesced dwordx4 stores
//   S1   : the textbook float4 copy: one 16-byte element per thread, grid = n/256 workgroups
//   SU   : U elements per thread, workgroup-contiguous (thread t: i = blk*256*U + u*256 + t)
//   WC   : one C-KiB contiguous chunk per wave, all loads issued before the stores (coalesced,
//          1 KiB per instruction), non-persistent grid, WG threads T
//   WCnt : WC with non-temporal stores
// Payload is random (splitmix64), not a constant fill.  Three interleaved rounds per variant.
// Build: hipcc --offload-arch=gfx950 -O3 copy2.hip -o copy2
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

__global__ void __launch_bounds__(256) rd_block(const u32x4 *__restrict__ s, size_t n16, unsigned *sink) {
    const size_t blk = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & 63;
    if (blk * 256 >= n16) return;
    const u32x4 *p = s + blk * 256 + lane;
    u32x4 a = p[0], b = p[64], c = p[128], d = p[192];
    unsigned x = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    if (x == 0x9E3779B9u) sink[0] = x;
}

template <int T>
__global__ void __launch_bounds__(T) wr_block(u32x4 *__restrict__ d, size_t n16) {
    const size_t blk = (size_t)blockIdx.x * (T / 64) + (threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & 63;
    if (blk * 256 >= n16) return;
    u32x4 v = {lane, (unsigned)blk, 7u, 9u};
    u32x4 *p = d + blk * 256 + lane;
    p[0] = v;
    p[64] = v;
    p[128] = v;
    p[192] = v;
}

template <int U>
__global__ void __launch_bounds__(256) cp_su(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n16) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + u * 256 < n16) v[u] = s[base + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + u * 256 < n16) d[base + u * 256] = v[u];
}

// one C-KiB chunk per wave: C loads of 1 KiB per wave-instruction, then C stores
template <int C, int T, bool kNt>
__global__ void __launch_bounds__(T) cp_wc(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n16) {
    const size_t chunk = (size_t)blockIdx.x * (T / 64) + (threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & 63;
    const size_t b = chunk * 64 * C;
    if (b >= n16) return;
    u32x4 v[C];
#pragma unroll
    for (int k = 0; k < C; ++k) v[k] = s[b + 64 * k + lane];
#pragma unroll
    for (int k = 0; k < C; ++k) {
        if (kNt)
            __builtin_nontemporal_store(v[k], d + b + 64 * k + lane);
        else
            d[b + 64 * k + lane] = v[k];
    }
}

// persistent-per-wave pipeline: a wave walks W consecutive 4 KiB blocks (stride: waves of the
// grid), issuing block j+1's loads before block j's stores
template <int T>
__global__ void __launch_bounds__(T) cp_pipe(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n16,
                                             unsigned W) {
    const size_t w0 = ((size_t)blockIdx.x * (T / 64) + (threadIdx.x >> 6)) * W;
    const unsigned lane = threadIdx.x & 63;
    const size_t nblk = n16 / 256;
    if (w0 >= nblk) return;
    const size_t wend = w0 + W < nblk ? w0 + W : nblk;
    u32x4 a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = s[w0 * 256 + 64 * k + lane];
    for (size_t j = w0; j < wend; ++j) {
        u32x4 nb[4];
        const size_t jn = j + 1 < wend ? j + 1 : j;
#pragma unroll
        for (int k = 0; k < 4; ++k) nb[k] = s[jn * 256 + 64 * k + lane];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[j * 256 + 64 * k + lane] = a[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = nb[k];
    }
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (8ull << 30);
    unsigned char *s, *d;
    unsigned *sink;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)s, bytes / 8);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)d, bytes / 8);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n16 = bytes / 16;
    const u32x4 *S = (const u32x4 *)s;
    u32x4 *D = (u32x4 *)d;
    struct V {
        std::string name;
        double mult;  // bytes moved / `bytes`
        std::function<void()> f;
        float best = 1e30f, sum = 0;
    };
    std::vector<V> vs;
    auto add = [&](std::string n, double m, std::function<void()> f) { vs.push_back({n, m, f}); };
    const unsigned nblk = (unsigned)(n16 / 256);
    add("RD 4KiB/wave (read only)", 1.0, [=] { hipLaunchKernelGGL(rd_block, dim3((nblk + 3) / 4), dim3(256), 0, 0, S, n16, sink); });
    add("WR 4KiB/wave T256 (write only)", 1.0, [=] { hipLaunchKernelGGL(wr_block<256>, dim3((nblk + 3) / 4), dim3(256), 0, 0, D, n16); });
    add("WR 4KiB/wave T512 (write only)", 1.0, [=] { hipLaunchKernelGGL(wr_block<512>, dim3((nblk + 7) / 8), dim3(512), 0, 0, D, n16); });
    add("S1 float4/thread", 2.0, [=] { hipLaunchKernelGGL(cp_su<1>, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, 0, S, D, n16); });
    add("SU2", 2.0, [=] { hipLaunchKernelGGL(cp_su<2>, dim3((unsigned)((n16 + 511) / 512)), dim3(256), 0, 0, S, D, n16); });
    add("SU4", 2.0, [=] { hipLaunchKernelGGL(cp_su<4>, dim3((unsigned)((n16 + 1023) / 1024)), dim3(256), 0, 0, S, D, n16); });
    add("SU8", 2.0, [=] { hipLaunchKernelGGL(cp_su<8>, dim3((unsigned)((n16 + 2047) / 2048)), dim3(256), 0, 0, S, D, n16); });
#define WC(C, T)                                                                                                   \
    add("WC C=" #C "KiB T=" #T, 2.0, [=] {                                                                         \
        hipLaunchKernelGGL((cp_wc<C, T, false>), dim3((unsigned)((n16 / (64 * C) + T / 64 - 1) / (T / 64))),     \
                           dim3(T), 0, 0, S, D, n16);                                                              \
    });                                                                                                            \
    add("WCnt C=" #C "KiB T=" #T, 2.0, [=] {                                                                       \
        hipLaunchKernelGGL((cp_wc<C, T, true>), dim3((unsigned)((n16 / (64 * C) + T / 64 - 1) / (T / 64))),      \
                           dim3(T), 0, 0, S, D, n16);                                                              \
    });
    WC(4, 256) WC(8, 256) WC(16, 256) WC(4, 512) WC(8, 512) WC(4, 1024) WC(2, 256) WC(16, 512)
    for (unsigned W : {4u, 16u, 64u}) {
        add("PIPE T256 W=" + std::to_string(W), 2.0, [=] {
            const size_t waves = (nblk + W - 1) / W;
            hipLaunchKernelGGL(cp_pipe<256>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, 0, S, D, n16, W);
        });
    }
    add("hipMemcpyDtoD", 2.0, [=] { CK(hipMemcpyAsync(D, S, bytes, hipMemcpyDeviceToDevice, 0)); });
    for (auto &v : vs) {  // warm
        v.f();
        CK(hipGetLastError());
    }
    CK(hipDeviceSynchronize());
    const int rounds = 3, reps = 4;
    for (int r = 0; r < rounds; ++r) {
        for (auto &v : vs) {
            for (int k = 0; k < reps; ++k) {
                CK(hipEventRecord(e0));
                v.f();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.sum += ms;
                if (ms < v.best) v.best = ms;
            }
        }
    }
    for (auto &v : vs) {
        const double avg = v.sum / (rounds * reps) / 1e3;
        const double gb = v.mult * bytes / avg / 1e9;
        printf("%-34s avg %7.3f ms best %7.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", v.name.c_str(), avg * 1e3, v.best,
               gb, gb / 80.0);
    }
    return 0;
}
