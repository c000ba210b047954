// crc_ablation.hip -- where does crc_regular_kernel's time go?
// Times the product kernel (variant 0) against two ablations of the SAME kernel:
//   1 = loads only (rows XOR-folded, no lookups)   -> the memory side alone
//   2 = lookups only (register data, no HBM)        -> the LDS/VALU side alone
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 crc_ablation.hip -o crc_ablation
#include "../../lampi_amd/csrc/crc_tables.cc"
#include "../../lampi_amd/csrc/frag_csum.hip"

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

using namespace lampi;

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 30);
    std::vector<uint32_t> img = build_table_image();
    uint32_t *dimg;
    CK(hipMalloc(&dimg, img.size() * 4));
    CK(hipMemcpy(dimg, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    uint8_t *buf;
    CK(hipMalloc(&buf, bytes));
    launch_fill_stream(buf, bytes, 2, 0, 256, 0);  // random payload (stream seed 2)
    uint32_t *out;
    CK(hipMalloc(&out, (bytes / 1024) * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[3] = {"product", "loads-only", "lookups-only"};
    for (size_t L : {4096ul, 16384ul}) {
        const uint32_t n = (uint32_t)(bytes / L);
        for (uint32_t fpw : {8u, 16u, 32u, 64u}) {
            const dim3 grid((n + kWaves * fpw - 1) / (kWaves * fpw));
            for (int v = 0; v < 3; ++v) {
                auto launch = [&] {
                    if (v == 0)
                        hipLaunchKernelGGL(crc_regular_kernel<0>, grid, dim3(kBlock), 0, 0, buf, n, fpw, L, 0xFFFFFFFFu,
                                           dimg, out);
                    else if (v == 1)
                        hipLaunchKernelGGL(crc_regular_kernel<1>, grid, dim3(kBlock), 0, 0, buf, n, fpw, L, 0xFFFFFFFFu,
                                           dimg, out);
                    else
                        hipLaunchKernelGGL(crc_regular_kernel<2>, grid, dim3(kBlock), 0, 0, buf, n, fpw, L, 0xFFFFFFFFu,
                                           dimg, out);
                };
                launch();
                CK(hipDeviceSynchronize());
                const int reps = 10;
                CK(hipEventRecord(e0));
                for (int r = 0; r < reps; ++r) launch();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double s = ms / 1e3 / reps;
                printf("L=%5zu fpw=%2u %-13s grid=%6u  %8.3f ms  %8.1f GB/s  %5.1f%% of 8 TB/s\n", L, fpw, names[v],
                       grid.x, s * 1e3, bytes / s / 1e9, bytes / s / 8e12 * 100);
                fflush(stdout);
            }
        }
    }
    return 0;
}
