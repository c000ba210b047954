// launch_size.hip -- the fixed cost of one launch on MI355X: plain read kernels (no checksum)
// at 1, 2, 4, 8 and 16 GiB per launch, so that the packed rows' and config B's 1 GiB numbers can be set against the
// read ceiling of the same launch size.
//   wave1 : non-persistent 256-thread workgroups, one 4 KiB block per wave (lane l: the 64 bytes at 64 l, four 16-byte
//           loads), XOR-folded, one 4-byte store per wave -- the shortest-lived read
//   wave1c: wave1 with lane l reading the 16-byte chunks at 16 l + 1024 q (1 KiB per load instruction)
//   wave1h: wave1 with lane l reading 32 bytes at 32 l and at 2048 + 32 l
//   wg128 : one 4 KiB block per 128-thread workgroup, thread t the chunks at 16 t and 2048 + 16 t (the SUM shape)
//   wg128nt, wave1nt: wg128 / wave1 with non-temporal loads (the SUM kernels' ld16u)
//   fpw12 : the same workgroups, each wave 12 blocks interleaved with the other waves of its workgroup, two blocks in
//           flight (config B's kernel's read shape without the tables)
// Time per launch by HIP events over 20 launches after 5 warm-ups, three interleaved rounds; a least-squares line
// t = t0 + bytes / B over the five sizes gives the fixed cost t0 and the asymptotic rate B.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 launch_size.hip -o launch_size
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

__global__ void __launch_bounds__(256) wave1(const u32x4 *__restrict__ p, unsigned nblk, unsigned *out) {
    const unsigned w = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    if (w >= nblk) return;
    const u32x4 *q = p + (size_t)w * 256 + l * 4;
    u32x4 a = q[0] ^ q[1] ^ q[2] ^ q[3];
    unsigned x = a.x ^ a.y ^ a.z ^ a.w;
    for (int o = 32; o >= 1; o >>= 1) x ^= __shfl_xor(x, o);
    if (l == 0) out[w] = x;
}

// wave1 with lane l reading the 16-byte chunks at 16 l + 1024 q (coalesced: 1 KiB per load instruction)
__global__ void __launch_bounds__(256) wave1c(const u32x4 *__restrict__ p, unsigned nblk, unsigned *out) {
    const unsigned w = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    if (w >= nblk) return;
    const u32x4 *q = p + (size_t)w * 256 + l;
    u32x4 a = q[0] ^ q[64] ^ q[128] ^ q[192];
    unsigned x = a.x ^ a.y ^ a.z ^ a.w;
    for (int o = 32; o >= 1; o >>= 1) x ^= __shfl_xor(x, o);
    if (l == 0) out[w] = x;
}

// wave1 with lane l reading the 32 bytes at 32 l and at 2048 + 32 l (2 KiB per load instruction pair)
__global__ void __launch_bounds__(256) wave1h(const u32x4 *__restrict__ p, unsigned nblk, unsigned *out) {
    const unsigned w = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    if (w >= nblk) return;
    const u32x4 *q = p + (size_t)w * 256 + 2 * l;
    u32x4 a = q[0] ^ q[1] ^ q[128] ^ q[129];
    unsigned x = a.x ^ a.y ^ a.z ^ a.w;
    for (int o = 32; o >= 1; o >>= 1) x ^= __shfl_xor(x, o);
    if (l == 0) out[w] = x;
}

// one 4 KiB block per 128-thread workgroup, thread t the 16-byte chunks at 16 t and 2048 + 16 t (the SUM kernel's shape)
__global__ void __launch_bounds__(128) wg128(const u32x4 *__restrict__ p, unsigned nblk, unsigned *out) {
    const unsigned w = blockIdx.x, t = threadIdx.x;
    const u32x4 *q = p + (size_t)w * 256 + t;
    u32x4 a = q[0] ^ q[128];
    unsigned x = a.x ^ a.y ^ a.z ^ a.w;
    for (int o = 32; o >= 1; o >>= 1) x ^= __shfl_xor(x, o);
    if ((t & 63) == 0) out[2 * w + (t >> 6)] = x;
}

// wg128 / wave1 with non-temporal loads (the SUM kernel's ld16u)
__global__ void __launch_bounds__(128) wg128nt(const u32x4 *__restrict__ p, unsigned nblk, unsigned *out) {
    const unsigned w = blockIdx.x, t = threadIdx.x;
    const u32x4 *q = p + (size_t)w * 256 + t;
    u32x4 a = __builtin_nontemporal_load(q) ^ __builtin_nontemporal_load(q + 128);
    unsigned x = a.x ^ a.y ^ a.z ^ a.w;
    for (int o = 32; o >= 1; o >>= 1) x ^= __shfl_xor(x, o);
    if ((t & 63) == 0) out[2 * w + (t >> 6)] = x;
}
__global__ void __launch_bounds__(256) wave1nt(const u32x4 *__restrict__ p, unsigned nblk, unsigned *out) {
    const unsigned w = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    if (w >= nblk) return;
    const u32x4 *q = p + (size_t)w * 256 + l * 4;
    u32x4 a = __builtin_nontemporal_load(q) ^ __builtin_nontemporal_load(q + 1) ^ __builtin_nontemporal_load(q + 2) ^
              __builtin_nontemporal_load(q + 3);
    unsigned x = a.x ^ a.y ^ a.z ^ a.w;
    for (int o = 32; o >= 1; o >>= 1) x ^= __shfl_xor(x, o);
    if (l == 0) out[w] = x;
}

__global__ void __launch_bounds__(256) fpw12(const u32x4 *__restrict__ p, unsigned nblk, unsigned *out) {
    const unsigned l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned b0 = blockIdx.x * 48 + wv;
    unsigned x = 0;
    u32x4 c0, c1, c2, c3;
    for (unsigned j = 0; j < 12; ++j) {
        const unsigned b = b0 + 4 * j;
        if (b >= nblk) break;
        const u32x4 *q = p + (size_t)b * 256 + l * 4;
        c0 = q[0];
        c1 = q[1];
        c2 = q[2];
        c3 = q[3];
        const u32x4 a = c0 ^ c1 ^ c2 ^ c3;
        x ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    for (int o = 32; o >= 1; o >>= 1) x ^= __shfl_xor(x, o);
    if (l == 0) out[blockIdx.x * 4 + wv] = x;
}

int main() {
    const size_t max_bytes = 16ull << 30;
    u32x4 *buf;
    unsigned *out;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMemset(buf, 0x5A, max_bytes));
    CK(hipMalloc(&out, (max_bytes / 4096) * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned gib[5] = {1, 2, 4, 8, 16};
    const char *names[7] = {"wave1", "fpw12", "wave1c", "wave1h", "wg128", "wg128nt", "wave1nt"};
    double us[7][5] = {};
    for (int round = 0; round < 3; ++round) {
        for (int k = 0; k < 7; ++k) {
            for (int s = 0; s < 5; ++s) {
                const size_t bytes = (size_t)gib[s] << 30;
                const unsigned nblk = (unsigned)(bytes / 4096);
                auto launch = [&] {
                    if (k == 0)
                        hipLaunchKernelGGL(wave1, dim3((nblk + 3) / 4), dim3(256), 0, 0, buf, nblk, out);
                    else if (k == 1)
                        hipLaunchKernelGGL(fpw12, dim3((nblk + 47) / 48), dim3(256), 0, 0, buf, nblk, out);
                    else if (k == 2)
                        hipLaunchKernelGGL(wave1c, dim3((nblk + 3) / 4), dim3(256), 0, 0, buf, nblk, out);
                    else if (k == 3)
                        hipLaunchKernelGGL(wave1h, dim3((nblk + 3) / 4), dim3(256), 0, 0, buf, nblk, out);
                    else if (k == 4)
                        hipLaunchKernelGGL(wg128, dim3(nblk), dim3(128), 0, 0, buf, nblk, out);
                    else if (k == 5)
                        hipLaunchKernelGGL(wg128nt, dim3(nblk), dim3(128), 0, 0, buf, nblk, out);
                    else
                        hipLaunchKernelGGL(wave1nt, dim3((nblk + 3) / 4), dim3(256), 0, 0, buf, nblk, out);
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
                if (round > 0) us[k][s] += t / 2;
                std::printf("round %d %-6s %2u GiB %9.1f us  %5.1f%%\n", round, names[k], gib[s], t,
                            bytes / (t * 1e-6) / 8e12 * 100);
                std::fflush(stdout);
            }
        }
    }
    for (int k = 0; k < 7; ++k) {  // least squares over rounds 1-2: t = t0 + bytes / B
        double sx = 0, sy = 0, sxx = 0, sxy = 0;
        for (int s = 0; s < 5; ++s) {
            const double x = (double)gib[s], y = us[k][s];
            sx += x;
            sy += y;
            sxx += x * x;
            sxy += x * y;
        }
        const double slope = (5 * sxy - sx * sy) / (5 * sxx - sx * sx), t0 = (sy - slope * sx) / 5;
        std::printf("%-6s fixed %.1f us per launch, asymptotic %.1f%% of 8 TB/s; 1 GiB %.1f%%, 16 GiB %.1f%%\n", names[k],
                    t0, (1ull << 30) / (slope * 1e-6) / 8e12 * 100, (1ull << 30) / (us[k][0] * 1e-6) / 8e12 * 100,
                    (16ull << 30) / (us[k][4] * 1e-6) / 8e12 * 100);
    }
    return 0;
}
