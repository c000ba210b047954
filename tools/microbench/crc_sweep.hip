// crc_sweep.hip -- crc_regular_kernel (the product kernel) over chains K, ring depth D and
// fragments per wave, three interleaved rounds per configuration (best and median reported:
// box-to-box and run-to-run spread is +-1-2%); every configuration's checksums are checked
// against the product launcher's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 crc_sweep.hip -o crc_sweep
#include "../../lampi_amd/csrc/crc_tables.cc"
#include "../../lampi_amd/csrc/frag_csum.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

using namespace lampi;

static uint8_t *g_dst = nullptr;  // copy destination (fused bcopy configurations)

struct Cfg {
    std::string name;
    uint32_t L, fpw;
    std::function<void(const uint8_t *, uint32_t, uint32_t, uint32_t, const uint32_t *, uint32_t *)> go;
    std::vector<double> ms;
};

template <int K, int D, bool kSum = false>
static Cfg make_copy(uint32_t L, uint32_t fpw) {
    Cfg c;
    char nm[64];
    snprintf(nm, sizeof nm, "copy%s K=%d D=%d", kSum ? "+sum" : "+crc", K, D);
    c.name = nm;
    c.L = L;
    c.fpw = fpw;
    c.go = [](const uint8_t *buf, uint32_t n, uint32_t fpw, uint32_t L, const uint32_t *img, uint32_t *out) {
        const dim3 grid((n + kWaves * fpw - 1) / (kWaves * fpw));
        hipLaunchKernelGGL((crc_regular_kernel<K, true, true, D, 1, kSum>), grid, dim3(kBlock), 0, 0, buf, n, fpw,
                           (size_t)L, 0xFFFFFFFFu, img, out, g_dst, (size_t)L);
    };
    return c;
}

template <int K, int D, int V = 1>
static Cfg make(uint32_t L, uint32_t fpw) {
    Cfg c;
    char nm[64];
    snprintf(nm, sizeof nm, "K=%d D=%d V=%d", K, D, V);
    c.name = nm;
    c.L = L;
    c.fpw = fpw;
    c.go = [](const uint8_t *buf, uint32_t n, uint32_t fpw, uint32_t L, const uint32_t *img, uint32_t *out) {
        const uint32_t nv = n / V;  // V > 1: the rows of V*4096-byte virtual fragments are 4 KiB fragments
        const dim3 grid((nv + kWaves * fpw - 1) / (kWaves * fpw));
        hipLaunchKernelGGL((crc_regular_kernel<K, false, false, D, V>), grid, dim3(kBlock), 0, 0, buf, nv, fpw,
                           (size_t)L * V, 0xFFFFFFFFu, img, out, nullptr, (size_t)0);
    };
    return c;
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 30);
    // payload offsets into one allocation (the schedule's speed depends on where the batch sits)
    std::vector<size_t> shifts;
    for (int a = 2; a < argc; ++a) shifts.push_back(strtoull(argv[a], 0, 0));
    if (shifts.empty()) shifts.push_back(0);
    const size_t max_shift = *std::max_element(shifts.begin(), shifts.end());
    std::vector<uint32_t> img = build_table_image();
    uint32_t *dimg;
    CK(hipMalloc(&dimg, img.size() * 4));
    CK(hipMemcpy(dimg, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    uint8_t *alloc;
    CK(hipMalloc(&alloc, bytes + max_shift));
    uint32_t *out;
    CK(hipMalloc(&out, (bytes / 4096) * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    std::vector<Cfg> cfgs;
    cfgs.push_back(make<2, 3, 2>(4096, 12));
    for (uint32_t fpw : {8u, 12u, 16u, 24u, 32u}) cfgs.push_back(make_copy<2, 3>(4096, fpw));
    for (uint32_t fpw : {12u, 32u}) cfgs.push_back(make_copy<2, 3, true>(4096, fpw));
    CK(hipMalloc(&g_dst, bytes));
    for (size_t shift : shifts) {
    uint8_t *buf = alloc + shift;
    printf("payload at %p (allocation + %zu)\n", (void *)buf, shift);
    launch_fill_stream(buf, bytes, 2, 0, 256, 0);
    for (Cfg &c : cfgs) c.ms.clear();
    std::vector<uint32_t> want4, want16, got;
    for (uint32_t L : {4096u, 16384u}) {
        const uint32_t n = (uint32_t)(bytes / L);
        std::vector<uint32_t> &w = L == 4096 ? want4 : want16;
        w.resize(n);
        CK(launch_crc_regular(buf, n, L, 0xFFFFFFFFu, out, dimg, 256, 0));
        CK(hipMemcpy(w.data(), out, (size_t)n * 4, hipMemcpyDeviceToHost));
    }
    for (Cfg &c : cfgs) {  // correctness once per configuration
        const uint32_t n = (uint32_t)(bytes / c.L);
        CK(hipMemset(out, 0, (size_t)n * 4));
        c.go(buf, n, c.fpw, c.L, dimg, out);
        CK(hipDeviceSynchronize());
        got.resize(n);
        CK(hipMemcpy(got.data(), out, (size_t)n * 4, hipMemcpyDeviceToHost));
        if (c.name.find("+sum") == std::string::npos && got != (c.L == 4096 ? want4 : want16)) printf("!!! %s L=%u fpw=%u: checksums differ\n", c.name.c_str(), c.L, c.fpw);
    }
    for (int round = 0; round < 3; ++round) {
        for (Cfg &c : cfgs) {
            const uint32_t n = (uint32_t)(bytes / c.L);
            c.go(buf, n, c.fpw, c.L, dimg, out);
            const int reps = 8;
            CK(hipEventRecord(e0));
            for (int r = 0; r < reps; ++r) c.go(buf, n, c.fpw, c.L, dimg, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            c.ms.push_back(ms / reps);
        }
    }
    for (Cfg &c : cfgs) {
        std::sort(c.ms.begin(), c.ms.end());
        const double best = c.ms.front(), med = c.ms[c.ms.size() / 2];
        const double mv = c.name.compare(0, 4, "copy") == 0 ? 2.0 : 1.0;  // copies: bytes read + written
        printf("%s L=%5u fpw=%2u  best %6.3f ms %5.1f%%  median %6.3f ms %5.1f%%\n", c.name.c_str(), c.L, c.fpw, best,
               mv * bytes / (best * 1e-3) / 8e10, med, mv * bytes / (med * 1e-3) / 8e10);
    }
    fflush(stdout);
    }
    return 0;
}
