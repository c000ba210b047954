// launch_size.hip -- the fixed cost of one launch on MI355X: plain read kernels (no checksum)
// at 1, 2, 4, 8 and 16 GiB per launch, so that the packed rows' and config B's 1 GiB numbers can be set against the
// read ceiling of the same launch size.
//   wave1 : non-persistent 256-thread workgroups, one 4 KiB block per wave (lane l: the 64 bytes at 64 l, four 16-byte
//           loads), XOR-folded, one 4-byte store per wave -- the shortest-lived read
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
    CK(hipMalloc(&out, (max_bytes / 4096) * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned gib[5] = {1, 2, 4, 8, 16};
    const char *names[2] = {"wave1", "fpw12"};
    double us[2][5] = {};
    for (int round = 0; round < 3; ++round) {
        for (int k = 0; k < 2; ++k) {
            for (int s = 0; s < 5; ++s) {
                const size_t bytes = (size_t)gib[s] << 30;
                const unsigned nblk = (unsigned)(bytes / 4096);
                auto launch = [&] {
                    if (k == 0)
                        hipLaunchKernelGGL(wave1, dim3((nblk + 3) / 4), dim3(256), 0, 0, buf, nblk, out);
                    else
                        hipLaunchKernelGGL(fpw12, dim3((nblk + 47) / 48), dim3(256), 0, 0, buf, nblk, out);
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
    for (int k = 0; k < 2; ++k) {  // least squares over rounds 1-2: t = t0 + bytes / B
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
