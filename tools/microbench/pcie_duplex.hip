// pcie_duplex.hip -- the host<->device ceilings behind the host-message path (bench.py --e2e):
// H2D / D2H alone and concurrently (two streams), a pitched 2D D2H into 4,176-byte slots, a kernel
// storing straight into page-locked host memory (zero-copy writes), hipHostRegister of a 256 MiB
// pageable buffer, and memcpy into pinned memory on 1-4 threads.  Prints GiB/s per line.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -pthread pcie_duplex.hip -o pcie_duplex
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                       \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// each thread copies 16-byte chunks of row r (len bytes) from src (packed) to dst + r*stride
__global__ void __launch_bounds__(256) store_rows(const uint4 *__restrict__ src, uint8_t *dst, size_t len, size_t stride,
                                                  size_t rows) {
    const size_t per = len / 16;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < per * rows; i += (size_t)gridDim.x * 256) {
        const size_t r = i / per, c = i % per;
        uint4 v = src[i];
        *(uint4 *)(dst + r * stride + c * 16) = v;
    }
}

int main() {
    const size_t N = 256u << 20;
    uint8_t *h = nullptr, *h2 = nullptr, *d = nullptr, *d2 = nullptr;
    CK(hipHostMalloc((void **)&h, N + (8u << 20), hipHostMallocDefault));
    CK(hipHostMalloc((void **)&h2, N + (8u << 20), hipHostMallocDefault));
    CK(hipMalloc((void **)&d, N));
    CK(hipMalloc((void **)&d2, N));
    std::memset(h, 1, N);
    std::memset(h2, 2, N);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const int reps = 8;
    auto rate = [&](const char *what, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        double t0 = now();
        for (int i = 0; i < reps; ++i) fn();
        CK(hipDeviceSynchronize());
        double t = (now() - t0) / reps;
        std::printf("%-58s %8.2f GiB/s  (%.3f ms per 256 MiB)\n", what, N / t / (1 << 30), t * 1e3);
        std::fflush(stdout);
    };
    rate("H2D 256 MiB, one copy", [&] { CK(hipMemcpyAsync(d, h, N, hipMemcpyHostToDevice, s1)); });
    rate("H2D 256 MiB in 16 MiB copies", [&] {
        for (size_t o = 0; o < N; o += 16u << 20) CK(hipMemcpyAsync(d + o, h + o, 16u << 20, hipMemcpyHostToDevice, s1));
    });
    rate("H2D 256 MiB in 64 MiB copies", [&] {
        for (size_t o = 0; o < N; o += 64u << 20) CK(hipMemcpyAsync(d + o, h + o, 64u << 20, hipMemcpyHostToDevice, s1));
    });
    rate("H2D from host+8 (unaligned source)", [&] { CK(hipMemcpyAsync(d, h + 8, N, hipMemcpyHostToDevice, s1)); });
    rate("D2H 256 MiB, one copy", [&] { CK(hipMemcpyAsync(h2, d2, N, hipMemcpyDeviceToHost, s2)); });
    rate("H2D || D2H (two streams; rate per direction)", [&] {
        CK(hipMemcpyAsync(d, h, N, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(h2, d2, N, hipMemcpyDeviceToHost, s2));
    });
    rate("H2D || D2H in 16 MiB copies (per direction)", [&] {
        for (size_t o = 0; o < N; o += 16u << 20) {
            CK(hipMemcpyAsync(d + o, h + o, 16u << 20, hipMemcpyHostToDevice, s1));
            CK(hipMemcpyAsync(h2 + o, d2 + o, 16u << 20, hipMemcpyDeviceToHost, s2));
        }
    });
    const size_t L = 4096, S = 4176, rows = N / S;  // 4 KiB payloads into 4,176-byte slots (bytes moved: rows*L)
    const double scale = (double)(rows * L) / N;
    auto rate_rows = [&](const char *what, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        double t0 = now();
        for (int i = 0; i < reps; ++i) fn();
        CK(hipDeviceSynchronize());
        double t = (now() - t0) / reps;
        std::printf("%-58s %8.2f GiB/s of payload\n", what, N * scale / t / (1 << 30));
        std::fflush(stdout);
    };
    rate_rows("D2H 2D 4096 -> 4176-byte slots (host+72)", [&] {
        CK(hipMemcpy2DAsync(h2 + 72, S, d2, L, L, rows, hipMemcpyDeviceToHost, s2));
    });
    rate_rows("D2H 2D in 16 MiB pieces", [&] {
        const size_t pr = (16u << 20) / L;
        for (size_t r = 0; r < rows; r += pr)
            CK(hipMemcpy2DAsync(h2 + 72 + r * S, S, d2 + r * L, L, L, std::min(pr, rows - r), hipMemcpyDeviceToHost, s2));
    });
    rate_rows("H2D || D2H 2D in 16 MiB pieces (per direction)", [&] {
        const size_t pr = (16u << 20) / L;
        for (size_t r = 0; r < rows; r += pr) {
            CK(hipMemcpyAsync(d + r * L, h + r * L, std::min(pr, rows - r) * L, hipMemcpyHostToDevice, s1));
            CK(hipMemcpy2DAsync(h2 + 72 + r * S, S, d2 + r * L, L, L, std::min(pr, rows - r), hipMemcpyDeviceToHost, s2));
        }
    });
    for (int g : {256, 1024, 4096}) {
        char w[96];
        std::snprintf(w, sizeof w, "kernel stores into pinned slots (zero-copy), %d WGs", g);
        rate_rows(w, [&] { store_rows<<<g, 256, 0, s2>>>((const uint4 *)d2, h2 + 72, L, S, rows); });
        std::snprintf(w, sizeof w, "H2D || kernel stores into pinned slots, %d WGs", g);
        rate_rows(w, [&] {
            CK(hipMemcpyAsync(d, h, rows * L, hipMemcpyHostToDevice, s1));
            store_rows<<<g, 256, 0, s2>>>((const uint4 *)d2, h2 + 72, L, S, rows);
        });
    }
    // pageable buffers the runtime has never seen: its own staging of H2D and D2H
    {
        std::vector<uint8_t> fresh(N), fresh2(N);
        std::memset(fresh.data(), 4, N);
        std::memset(fresh2.data(), 5, N);
        rate("H2D from a fresh pageable buffer (runtime staging)", [&] {
            CK(hipMemcpyAsync(d, fresh.data(), N, hipMemcpyHostToDevice, s1));
        });
        rate("H2D from pageable, 16 MiB copies (runtime staging)", [&] {
            for (size_t o = 0; o < N; o += 16u << 20)
                CK(hipMemcpyAsync(d + o, fresh.data() + o, 16u << 20, hipMemcpyHostToDevice, s1));
        });
        rate("D2H into a fresh pageable buffer (runtime staging)", [&] {
            CK(hipMemcpyAsync(fresh2.data(), d2, N, hipMemcpyDeviceToHost, s2));
        });
        rate_rows("D2H 2D into pageable slots (runtime), 16 MiB pieces", [&] {
            const size_t pr = (16u << 20) / L;
            for (size_t r = 0; r < rows; r += pr)
                CK(hipMemcpy2DAsync(fresh2.data() + 72 + r * S, S, d2 + r * L, L, L, std::min(pr, rows - r),
                                    hipMemcpyDeviceToHost, s2));
        });
        rate_rows("H2D pageable || D2H 2D pageable slots, 16 MiB pieces", [&] {
            const size_t pr = (16u << 20) / L;
            for (size_t r = 0; r < rows; r += pr) {
                CK(hipMemcpyAsync(d + r * L, fresh.data() + r * L, std::min(pr, rows - r) * L, hipMemcpyHostToDevice, s1));
                CK(hipMemcpy2DAsync(fresh2.data() + 72 + r * S, S, d2 + r * L, L, L, std::min(pr, rows - r),
                                    hipMemcpyDeviceToHost, s2));
            }
        });
        rate_rows("H2D pageable || D2H 2D pinned slots, 16 MiB pieces", [&] {
            const size_t pr = (16u << 20) / L;
            for (size_t r = 0; r < rows; r += pr) {
                CK(hipMemcpyAsync(d + r * L, fresh.data() + r * L, std::min(pr, rows - r) * L, hipMemcpyHostToDevice, s1));
                CK(hipMemcpy2DAsync(h2 + 72 + r * S, S, d2 + r * L, L, L, std::min(pr, rows - r), hipMemcpyDeviceToHost, s2));
            }
        });
    }
    rate("D2H 256 MiB, one copy (again)", [&] { CK(hipMemcpyAsync(h2, d2, N, hipMemcpyDeviceToHost, s2)); });
    rate("H2D 256 MiB in 16 MiB copies (again)", [&] {
        for (size_t o = 0; o < N; o += 16u << 20) CK(hipMemcpyAsync(d + o, h + o, 16u << 20, hipMemcpyHostToDevice, s1));
    });
    // hipHostRegister of pageable memory
    std::vector<uint8_t> pg(N);
    std::memset(pg.data(), 3, N);
    for (int i = 0; i < 3; ++i) {
        double t0 = now();
        CK(hipHostRegister(pg.data(), N, hipHostRegisterDefault));
        double t1 = now();
        CK(hipHostUnregister(pg.data()));
        double t2 = now();
        std::printf("hipHostRegister 256 MiB pageable: %.3f ms (%.2f GiB/s), unregister %.3f ms\n", (t1 - t0) * 1e3,
                    N / (t1 - t0) / (1 << 30), (t2 - t1) * 1e3);
    }
    rate("H2D from pageable (runtime staging)", [&] { CK(hipMemcpyAsync(d, pg.data(), N, hipMemcpyHostToDevice, s1)); });
    for (int nt : {1, 2, 4, 8}) {
        double best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
            double t0 = now();
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t)
                th.emplace_back([&, t] {
                    const size_t a = N / nt * t, b = t + 1 == nt ? N : N / nt * (t + 1);
                    std::memcpy(h + a, pg.data() + a, b - a);
                });
            for (auto &x : th) x.join();
            best = std::min(best, now() - t0);
        }
        std::printf("memcpy pageable -> pinned, %d threads: %8.2f GiB/s\n", nt, N / best / (1 << 30));
    }
    std::printf("done\n");
    return 0;
}
