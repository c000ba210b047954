// copy4.hip -- why do fused copies of 64 KiB fragments (the row kernels: one wave walks one
// fragment row by row) run ~10 points below the same kernels on 4 KiB fragments?  Hypothesis:
// a workgroup's eight waves stream eight fragments 64 KiB apart at once.  Plain copies (no
// checksum) in the row kernels' shape -- 512-thread workgroups holding 64 KiB of LDS, each wave
// F fragments of L bytes, one 4 KiB row (4 x 1 KiB wave-instructions) in flight, next row
// prefetched -- against the same bytes with the workgroup's waves interleaved on rows (wave w
// copies rows w, w + 8, ... of the workgroup's contiguous region).  16 GiB -> 16 GiB.
// Build: hipcc --offload-arch=gfx950 -O3 copy4.hip -o copy4
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

// kInter = false: wave w of workgroup b copies fragments (b * 8 + w) + 8 * j, j < F, each row by
// row; kInter = true: the workgroup's 8 * F fragments form one region whose rows the waves take
// in turn (row w, w + 8, ...).
template <bool kInter>
__global__ void __launch_bounds__(512) cp_rows(const unsigned char *__restrict__ s, unsigned char *__restrict__ d,
                                               size_t nfrag, uint32_t L, uint32_t F, unsigned *sink) {
    __shared__ unsigned lds[65536 / 4];
    const unsigned w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const uint32_t R = L / 4096;
    const size_t f0 = (size_t)blockIdx.x * 8 * F;
    const uint32_t nrows = kInter ? 8 * F * R : F * R;  // rows of this wave's walk (before the stride)
    auto row_off = [&](uint32_t i) -> size_t {          // i-th row of this wave
        if (kInter) {
            const size_t r = (size_t)i * 8 + w;  // region row
            return (f0 * L) + r * 4096;
        }
        const uint32_t j = i / R, r = i % R;
        return (f0 + w + 8 * (size_t)j) * L + (size_t)r * 4096;
    };
    const uint32_t n = kInter ? nrows / 8 : nrows;
    const size_t lim = nfrag * (size_t)L;
    u32x4 a[4], b[4];
    auto ld = [&](uint32_t i, u32x4 (&v)[4]) {
        const size_t o = row_off(i);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = o < lim ? *(const u32x4 *)(s + o + 1024 * k + 16 * lane) : u32x4{0, 0, 0, 0};
    };
    auto st = [&](uint32_t i, const u32x4 (&v)[4]) {
        const size_t o = row_off(i);
        if (o < lim) {
#pragma unroll
            for (int k = 0; k < 4; ++k) *(u32x4 *)(d + o + 1024 * k + 16 * lane) = v[k];
        }
    };
    if (n > 0) ld(0, a);
    for (uint32_t i = 0; i < n; i += 2) {
        if (i + 1 < n) ld(i + 1, b);
        st(i, a);
        if (i + 2 < n) ld(i + 2, a);
        if (i + 1 < n) st(i + 1, b);
    }
    if (lds[(lane * 7) & 16383] == 0xFFFFFFFFu) sink[0] = 1;
}

int main() {
    const size_t bytes = 16ull << 30;
    unsigned char *s, *d;
    unsigned *sink;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)s, bytes / 8);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V {
        std::string name;
        std::function<void()> f;
        float sum = 0;
    };
    std::vector<V> vs;
    for (uint32_t L : {4096u, 16384u, 65536u})
        for (uint32_t F : {1u, 6u})
            for (int inter = 0; inter < 2; ++inter) {
                if (L == 4096 && inter) continue;  // one row per fragment: the same walk
                const size_t nfrag = bytes / L;
                const unsigned g = (unsigned)((nfrag + 8 * F - 1) / (8 * F));
                vs.push_back({"L=" + std::to_string(L) + " F=" + std::to_string(F) + (inter ? " rows interleaved" : " fragment per wave"),
                              [=] {
                                  if (inter)
                                      hipLaunchKernelGGL(cp_rows<true>, dim3(g), dim3(512), 0, 0, s, d, nfrag, L, F, sink);
                                  else
                                      hipLaunchKernelGGL(cp_rows<false>, dim3(g), dim3(512), 0, 0, s, d, nfrag, L, F, sink);
                              }});
            }
    for (auto &v : vs) v.f();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const int rounds = 3, reps = 3;
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
