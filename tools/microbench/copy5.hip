// copy5.hip -- fused copy + 32-bit word sum (bcopy_uicsum's regular case: 4 KiB fragments,
// 16-byte-aligned source and destination) in the textbook copy shape against the product's
// one-fragment-per-wave shape.  The read + write bytes are counted.
//   PLAIN S1 : the textbook float4 copy (no sum): one 16-byte element per thread, 256-thread
//              workgroups (the copy ceiling, copy2.hip's S1)
//   WAVE4K   : the product's sum_regular_kernel<copy> shape: one 4 KiB fragment per wave, four
//              coalesced dwordx4 per lane, DPP sum, lane 0 stores
//   TB-LDS T : T/256 fragments per T-thread workgroup, one 16-byte element per thread, wave sums
//              combined through LDS after one barrier
//   TB-ATOM  : 256-thread workgroup per fragment, each wave atomically adds its 1 KiB sum into
//              out (zeroed by a memset inside the timed region)
//   TB2-LDS  : 128 threads per fragment, two elements per thread (coalesced 2 KiB runs)
// Every variant's sums are compared with WAVE4K's.  Build: hipcc --offload-arch=gfx950 -O3
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

__device__ __forceinline__ unsigned wsum(unsigned v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__global__ void __launch_bounds__(256) cp_s1(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n16) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) d[i] = s[i];
}

template <bool kNt>
__global__ void __launch_bounds__(256) sum_wave4k(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, unsigned n,
                                                  unsigned *out) {
    const unsigned f = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (f >= n) return;
    const u32x4 *p = s + (size_t)f * 256 + lane;
    u32x4 *q = d + (size_t)f * 256 + lane;
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = p[64 * k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (kNt)
            __builtin_nontemporal_store(v[k], q + 64 * k);
        else
            q[64 * k] = v[k];
    }
    unsigned a = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) a += v[k].x + v[k].y + v[k].z + v[k].w;
    a = wsum(a);
    if (lane == 0) out[f] = a;
}

// T threads, T/256 fragments per workgroup, one element per thread
template <int T, bool kNt>
__global__ void __launch_bounds__(T) sum_tb_lds(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, unsigned n,
                                                unsigned *out) {
    __shared__ unsigned part[T / 64];
    const size_t i = (size_t)blockIdx.x * T + threadIdx.x;
    const u32x4 v = s[i];
    if (kNt)
        __builtin_nontemporal_store(v, d + i);
    else
        d[i] = v;
    const unsigned a = wsum(v.x + v.y + v.z + v.w);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x < T / 256) {
        const unsigned *pp = part + 4 * threadIdx.x;
        out[(size_t)blockIdx.x * (T / 256) + threadIdx.x] = pp[0] + pp[1] + pp[2] + pp[3];
    }
}

__global__ void __launch_bounds__(256) sum_tb_atom(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, unsigned n,
                                                   unsigned *out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const u32x4 v = s[i];
    d[i] = v;
    const unsigned a = wsum(v.x + v.y + v.z + v.w);
    if ((threadIdx.x & 63) == 0) atomicAdd(out + blockIdx.x, a);
}

// 128 threads per fragment, elements t and t + 128
__global__ void __launch_bounds__(128) sum_tb2_lds(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, unsigned n,
                                                   unsigned *out) {
    __shared__ unsigned part[2];
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const u32x4 v = s[i], w = s[i + 128];
    d[i] = v;
    d[i + 128] = w;
    const unsigned a = wsum(v.x + v.y + v.z + v.w + w.x + w.y + w.z + w.w);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = part[0] + part[1];
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 30);
    const unsigned n = (unsigned)(bytes / 4096);
    unsigned char *s, *d;
    unsigned *ref, *out;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&ref, n * 4ull));
    CK(hipMalloc(&out, n * 4ull));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)s, bytes / 8);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)d, bytes / 8);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n16 = bytes / 16;
    const u32x4 *S = (const u32x4 *)s;
    u32x4 *D = (u32x4 *)d;
    hipLaunchKernelGGL(sum_wave4k<false>, dim3((n + 3) / 4), dim3(256), 0, 0, S, D, n, ref);
    CK(hipDeviceSynchronize());
    struct V {
        std::string name;
        bool check;
        std::function<void()> f;
        float best = 1e30f, sum = 0;
    };
    std::vector<V> vs;
    auto add = [&](std::string nm, bool c, std::function<void()> f) { vs.push_back({nm, c, f}); };
    add("PLAIN S1 float4/thread (no sum)", false,
        [=] { hipLaunchKernelGGL(cp_s1, dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, S, D, n16); });
    add("WAVE4K (product shape)", true,
        [=] { hipLaunchKernelGGL(sum_wave4k<false>, dim3((n + 3) / 4), dim3(256), 0, 0, S, D, n, out); });
    add("WAVE4K nt stores", true,
        [=] { hipLaunchKernelGGL(sum_wave4k<true>, dim3((n + 3) / 4), dim3(256), 0, 0, S, D, n, out); });
    add("TB-LDS T256", true,
        [=] { hipLaunchKernelGGL((sum_tb_lds<256, false>), dim3(n), dim3(256), 0, 0, S, D, n, out); });
    add("TB-LDS T256 nt", true,
        [=] { hipLaunchKernelGGL((sum_tb_lds<256, true>), dim3(n), dim3(256), 0, 0, S, D, n, out); });
    add("TB-LDS T512", true,
        [=] { hipLaunchKernelGGL((sum_tb_lds<512, false>), dim3(n / 2), dim3(512), 0, 0, S, D, n, out); });
    add("TB-LDS T1024", true,
        [=] { hipLaunchKernelGGL((sum_tb_lds<1024, false>), dim3(n / 4), dim3(1024), 0, 0, S, D, n, out); });
    add("TB-ATOM (memset + kernel)", true, [=] {
        CK(hipMemsetAsync(out, 0, n * 4ull, 0));
        hipLaunchKernelGGL(sum_tb_atom, dim3(n), dim3(256), 0, 0, S, D, n, out);
    });
    add("TB2-LDS T128", true, [=] { hipLaunchKernelGGL(sum_tb2_lds, dim3(n), dim3(128), 0, 0, S, D, n, out); });
    std::vector<unsigned> hr(n), ho(n);
    CK(hipMemcpy(hr.data(), ref, n * 4ull, hipMemcpyDeviceToHost));
    for (auto &v : vs) {  // warm + check
        CK(hipMemset(out, 0xA5, n * 4ull));
        v.f();
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        if (v.check) {
            CK(hipMemcpy(ho.data(), out, n * 4ull, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (unsigned k = 0; k < n; ++k) bad += ho[k] != hr[k];
            if (bad) {
                fprintf(stderr, "%s: %zu wrong sums\n", v.name.c_str(), bad);
                return 1;
            }
        }
    }
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
    printf("# copy5.hip: %zu B src -> dst (%u x 4 KiB fragments), %% of 8 TB/s counts read + write\n", bytes, n);
    for (auto &v : vs) {
        const double avg = v.sum / (rounds * reps) / 1e3;
        const double gb = 2.0 * bytes / avg / 1e9;
        printf("%-34s avg %7.3f ms best %7.3f ms  %7.1f GB/s  %5.1f%% of 8 TB/s%s\n", v.name.c_str(), avg * 1e3,
               v.best, gb, gb / 80.0, v.check ? "  (sums checked)" : "");
    }
    return 0;
}
