// regular_occ.hip -- crc_regular_kernel (config B schedule) at more waves per CU: one chain per
// wave in 8/12-wave workgroups (waves_per_eu caps the VGPRs) against the product's two chains
// in 4-wave workgroups; three interleaved rounds of ten back-to-back launches per configuration,
// checksums compared with the product's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 regular_occ.hip -o regular_occ
#include "../../lampi_amd/csrc/crc_tables.cc"
#include "../../lampi_amd/csrc/frag_csum.hip"

#include <algorithm>
#include <cstdio>
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

struct Cfg {
    std::string name;
    std::function<void(const uint8_t *, uint32_t *)> go;
    int vgprs;
    std::vector<double> ms;
};

// n fragments of L bytes visited in kV*L row order (n even for kV = 2)
template <int K, int D, int kV, int kWv, int kCap>
static Cfg make(const char *nm, size_t n, uint32_t L, uint32_t fpw, const uint32_t *img) {
    Cfg c;
    c.name = nm;
    c.go = [=](const uint8_t *buf, uint32_t *out) {
        const size_t nv = n / kV;
        const dim3 grid((unsigned)((nv + (size_t)kWv * fpw - 1) / ((size_t)kWv * fpw)));
        hipLaunchKernelGGL((crc_regular_kernel<K, false, false, D, kV, false, kWv, kCap>), grid, dim3(64 * kWv), 0,
                           0, buf, (uint32_t)nv, fpw, (size_t)kV * L, 0xFFFFFFFFu, img, out, nullptr, (size_t)0);
    };
    hipFuncAttributes a;
    CK(hipFuncGetAttributes(&a, (const void *)crc_regular_kernel<K, false, false, D, kV, false, kWv, kCap>));
    c.vgprs = a.numRegs;
    return c;
}

static double batch_ms(const std::function<void()> &go, int k) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) go();
    CK(hipEventRecord(e0));
    for (int i = 0; i < k; ++i) go();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / k;
}

int main() {
    std::vector<uint32_t> himg = build_table_image();
    uint32_t *img;
    CK(hipMalloc(&img, himg.size() * 4));
    CK(hipMemcpy(img, himg.data(), himg.size() * 4, hipMemcpyHostToDevice));
    const size_t bytes = 16ull << 30;
    uint8_t *buf;
    CK(hipMalloc(&buf, bytes));
    CK(launch_fill_stream(buf, bytes, 2, 0, 256, 0));
    uint32_t *out, *ref;
    CK(hipMalloc(&out, (4u << 20) * 4));
    CK(hipMalloc(&ref, (4u << 20) * 4));
    for (uint32_t L : {4096u, 16384u}) {
        const size_t n = bytes / L;
        std::vector<Cfg> cs;
        if (L == 4096) {
            cs.push_back(make<2, 3, 2, 4, 0>("product K2 D3 4 waves fpw 12", n, L, 12, img));
            cs.push_back(make<1, 3, 2, 8, 0>("K1 D3 8 waves fpw 6", n, L, 6, img));
            cs.push_back(make<1, 3, 2, 12, 6>("K1 D3 12 waves fpw 4", n, L, 4, img));
            cs.push_back(make<1, 3, 2, 12, 6>("K1 D3 12 waves fpw 8", n, L, 8, img));
            cs.push_back(make<2, 3, 2, 8, 4>("K2 D3 8 waves fpw 6", n, L, 6, img));
        } else {
            cs.push_back(make<2, 3, 1, 4, 0>("product K2 D3 4 waves fpw 6", n, L, 6, img));
            cs.push_back(make<1, 3, 1, 12, 6>("K1 D3 12 waves fpw 2", n, L, 2, img));
            cs.push_back(make<1, 3, 1, 12, 6>("K1 D3 12 waves fpw 4", n, L, 4, img));
        }
        std::vector<uint32_t> want(n), got(n);
        cs[0].go(buf, ref);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(want.data(), ref, n * 4, hipMemcpyDeviceToHost));
        for (int round = 0; round < 3; ++round)
            for (auto &c : cs) c.ms.push_back(batch_ms([&] { c.go(buf, out); }, 10));
        for (auto &c : cs) {
            c.go(buf, out);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
            std::sort(c.ms.begin(), c.ms.end());
            printf("%5u B  %-32s %3d VGPRs  %.3f ms  %5.1f%% of 8 TB/s (rounds %.1f..%.1f%%)  %s\n", L, c.name.c_str(),
                   c.vgprs, c.ms[1], bytes / (c.ms[1] * 1e-3) / 8e12 * 100, bytes / (c.ms[2] * 1e-3) / 8e12 * 100,
                   bytes / (c.ms[0] * 1e-3) / 8e12 * 100, got == want ? "ok" : "MISMATCH");
        }
    }
    return 0;
}
