// sync_latency.hip -- host round trip of one tiny kernel on a stream, three ways of learning
// that it finished: hipStreamSynchronize; hipStreamWriteValue64 of a sequence number into
// host-coherent pinned memory, polled by the host; and the kernel itself storing the sequence
// number there (system scope), polled.  Median of 2000 round trips each.
// Build: hipcc --offload-arch=gfx950 -O3 sync_latency.hip -o sync_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
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

__global__ void work(const unsigned *in, unsigned *out) {
    unsigned x = in[threadIdx.x];
    for (int i = 0; i < 8; ++i) x = x * 2654435761u + 1u;
    out[threadIdx.x] = x;
}

__global__ void work_signal(const unsigned *in, unsigned *out, unsigned long long *sig, unsigned long long seq) {
    unsigned x = in[threadIdx.x];
    for (int i = 0; i < 8; ++i) x = x * 2654435761u + 1u;
    out[threadIdx.x] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(sig, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    unsigned *in, *out;
    CK(hipMalloc(&in, 256 * 4));
    CK(hipMalloc(&out, 256 * 4));
    CK(hipMemset(in, 1, 256 * 4));
    unsigned long long *sig = nullptr, *sig_d = nullptr;
    CK(hipHostMalloc((void **)&sig, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void **)&sig_d, sig, 0));
    *sig = 0;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int reps = 2000;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    unsigned long long seq = 0;
    for (int mode = 0; mode < 3; ++mode) {
        std::vector<double> t;
        for (int i = 0; i < reps + 100; ++i) {
            const auto a = now();
            if (mode == 0) {
                hipLaunchKernelGGL(work, dim3(1), dim3(256), 0, s, in, out);
                CK(hipStreamSynchronize(s));
            } else if (mode == 1) {
                hipLaunchKernelGGL(work, dim3(1), dim3(256), 0, s, in, out);
                CK(hipStreamWriteValue64(s, sig_d, ++seq, 0));
                const auto t0 = now();
                while (__atomic_load_n(sig, __ATOMIC_ACQUIRE) != seq) {
                    if (us(t0, now()) > 1e6) { fprintf(stderr, "timeout mode 1\n"); return 1; }
                }
            } else {
                hipLaunchKernelGGL(work_signal, dim3(1), dim3(256), 0, s, in, out, sig_d, ++seq);
                const auto t0 = now();
                while (__atomic_load_n(sig, __ATOMIC_ACQUIRE) != seq) {
                    if (us(t0, now()) > 1e6) { fprintf(stderr, "timeout mode 2\n"); return 1; }
                }
            }
            const auto b = now();
            if (i >= 100) t.push_back(us(a, b));
        }
        CK(hipStreamSynchronize(s));
        static const char *names[] = {"launch + hipStreamSynchronize", "launch + hipStreamWriteValue64 + poll",
                                      "launch (kernel stores the flag) + poll"};
        printf("%-40s median %7.2f us\n", names[mode], median(t));
    }
    return 0;
}
