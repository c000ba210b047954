// frags_sweep.hip -- crc_stream_kernel (the general-fragment product kernel) on config C
// (659,114 Zipf-sized fragments, 4 GiB) and on 4M x 4 KiB descriptors (config B through
// descriptors): ring depth, chains per wave, fragments per workgroup and the occupancy sweep;
// the regular kernel on the uniform batch for comparison.  Checksums of the product variant are
// compared with the regular kernel's on the uniform batch.  (Until commit d95cfff this was
// frags_ablation.hip and also ran ablated kernel variants -- loads + task walk only, no table
// lookups -- through a template switch of the product kernel: profiles/r01_stream_ablation.txt.)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 frags_sweep.hip -o frags_sweep
#include "../../lampi_amd/csrc/crc_tables.cc"
#include "../../lampi_amd/csrc/frag_csum.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
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

static uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static std::vector<uint32_t> zipf_lengths(uint64_t min_total) {
    double cdf[1025], z = 0.0, acc = 0.0;
    for (int r = 1; r <= 1024; ++r) z += pow((double)r, -1.1);
    cdf[0] = 0.0;
    for (int r = 1; r <= 1024; ++r) cdf[r] = (acc += pow((double)r, -1.1) / z);
    cdf[1024] = 1.0;
    std::vector<uint32_t> out;
    uint64_t total = 0;
    for (uint64_t k = 0; total < min_total; ++k) {
        const double u = (double)(mix64(0x5A1Full + k) >> 11) * (1.0 / 9007199254740992.0);
        int lo = 1, hi = 1024;
        while (lo < hi) {
            const int mid = (lo + hi) / 2;
            if (cdf[mid] > u) hi = mid; else lo = mid + 1;
        }
        out.push_back(64u * (uint32_t)lo);
        total += 64u * (uint32_t)lo;
    }
    return out;
}

template <int kD = 2, int kK = 1, int kWv = 12, int kCap = 6>
static void launch_stream(const lampi_frag_desc *d, size_t n, const uint32_t *img, uint32_t *out, uint32_t fpg = 0,
                          size_t pad_lds = 0) {
    if (fpg == 0) fpg = frags_per_wg(n);
    hipLaunchKernelGGL((crc_stream_kernel<DescSource, kD, kK, false, kWv, kCap>), frags_grid(n, fpg),
                       dim3(64 * kWv), pad_lds, 0, DescSource{d}, n, fpg, img, out);
}

template <int kD, int kK, int kWv, int kCap>
static int stream_vgprs() {
    hipFuncAttributes a;
    CK(hipFuncGetAttributes(&a, (const void *)crc_stream_kernel<DescSource, kD, kK, false, kWv, kCap>));
    return a.numRegs;
}

static double time_ms(const std::function<void()> &go, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 10; ++i) go();
    CK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        go();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

// average over k back-to-back launches between two events (after 3 warm-up launches)
static double time_batch_ms(const std::function<void()> &go, int k) {
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
    std::vector<uint32_t> img = build_table_image();
    uint32_t *dimg;
    CK(hipMalloc(&dimg, img.size() * 4));
    CK(hipMemcpy(dimg, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    const size_t bytes = 16ull << 30;
    uint8_t *buf;
    CK(hipMalloc(&buf, bytes));
    launch_fill_stream(buf, bytes, 2, 0, 256, 0);
    uint32_t *out, *ref;
    CK(hipMalloc(&out, (4u << 20) * 4));
    CK(hipMalloc(&ref, (4u << 20) * 4));

    printf("stream VGPRs: product (K1 kD2, 12 waves/WG, 6 waves/SIMD) %d, K1 kD2 8 waves/WG %d, K1 kD3 %d, K2 kD2 %d\n",
           stream_vgprs<2, 1, 12, 6>(), stream_vgprs<2, 1, 8, 0>(), stream_vgprs<3, 1, 8, 0>(), stream_vgprs<2, 2, 4, 0>());
    for (int cfg = 0; cfg < 2; ++cfg) {
        std::vector<lampi_frag_desc> h;
        uint64_t total = 0;
        if (cfg == 0) {
            for (uint32_t L : zipf_lengths(4ull << 30)) {
                h.push_back({(uint64_t)(uintptr_t)(buf + total), L, 0xFFFFFFFFu});
                total += L;
            }
        } else {
            for (size_t i = 0; i < (4u << 20); ++i) h.push_back({(uint64_t)(uintptr_t)(buf + 4096 * i), 4096, 0xFFFFFFFFu});
            total = 16ull << 30;
        }
        lampi_frag_desc *d;
        CK(hipMalloc(&d, h.size() * sizeof(lampi_frag_desc)));
        CK(hipMemcpy(d, h.data(), h.size() * sizeof(lampi_frag_desc), hipMemcpyHostToDevice));
        const size_t n = h.size();
        const char *cname = cfg == 0 ? "config C (Zipf, 4 GiB)" : "4M x 4 KiB descriptors";
        struct V {
            const char *name;
            std::function<void()> go;
        } vs[] = {{"product (12 waves/WG, fpg 96)", [&] { launch_stream<>(d, n, dimg, out); }},
                  {"12 waves/WG fpg 256", [&] { launch_stream<>(d, n, dimg, out, 256); }},
                  {"12 waves/WG fpg 128", [&] { launch_stream<>(d, n, dimg, out, 128); }},
                  {"12 waves/WG fpg 48", [&] { launch_stream<>(d, n, dimg, out, 48); }},
                  {"8 waves/WG K1 kD2 fpg 96", [&] { launch_stream<2, 1, 8, 0>(d, n, dimg, out, 96); }},
                  {"8 waves/WG K1 kD2 fpg 256", [&] { launch_stream<2, 1, 8, 0>(d, n, dimg, out, 256); }},
                  {"4 waves/WG K2 kD2", [&] { launch_stream<2, 2, 4, 0>(d, n, dimg, out); }}};
        // three interleaved rounds, back-to-back launches (as bench.py times them): run-to-run clock
        // and box drift are larger than most differences measured here
        const size_t nv = sizeof(vs) / sizeof(vs[0]);
        std::vector<std::vector<double>> res(nv);
        for (int round = 0; round < 3; ++round)
            for (size_t i = 0; i < nv; ++i) res[i].push_back(time_batch_ms(vs[i].go, 10));
        for (size_t i = 0; i < nv; ++i) {
            std::sort(res[i].begin(), res[i].end());
            const double ms = res[i][1];
            printf("%-24s %-28s %8.3f ms  %6.1f%% of 8 TB/s (rounds %.1f..%.1f%%)\n", cname, vs[i].name, ms,
                   total / (ms * 1e-3) / 8e12 * 100, total / (res[i][2] * 1e-3) / 8e12 * 100,
                   total / (res[i][0] * 1e-3) / 8e12 * 100);
        }
        // occupancy sweep: waves per CU = waves per workgroup x workgroups per CU;
        // LDS (~76 KiB per workgroup) allows two workgroups per CU, extra dynamic LDS forces one.
        // 32 waves per CU would need <= 64 VGPRs and <= 80 KiB for 16-wave workgroups: 80 VGPRs rule it out.
        struct O {
            int waves;
            const char *how;
            std::function<void()> go;
        } occ[] = {{4, "K2, 4 waves/WG, 1 WG/CU", [&] { launch_stream<2, 2, 4, 0>(d, n, dimg, out, 0, 16u << 10); }},
                   {8, "K2, 4 waves/WG, 2 WG/CU", [&] { launch_stream<2, 2, 4, 0>(d, n, dimg, out); }},
                   {8, "K1, 8 waves/WG, 1 WG/CU", [&] { launch_stream<2, 1, 8, 0>(d, n, dimg, out, 0, 16u << 10); }},
                   {12, "K1, 12 waves/WG, 1 WG/CU", [&] { launch_stream<>(d, n, dimg, out, 0, 16u << 10); }},
                   {16, "K1, 8 waves/WG, 2 WG/CU", [&] { launch_stream<2, 1, 8, 0>(d, n, dimg, out); }},
                   {24, "K1, 12 waves/WG, 2 WG/CU", [&] { launch_stream<>(d, n, dimg, out); }}};
        for (auto &o : occ) {
            const double ms = time_ms(o.go, 9);
            printf("%-24s occupancy %2d waves/CU (%s): %6.1f%% of 8 TB/s\n", cname, o.waves, o.how,
                   total / (ms * 1e-3) / 8e12 * 100);
        }
        if (cfg == 1) {
            const double ms = time_ms([&] { launch_crc_regular(buf, n, 4096, 0xFFFFFFFFu, ref, dimg, 512, 0); }, 15);
            printf("%-24s %-18s %8.3f ms  %6.1f%% of 8 TB/s\n", cname, "regular kernel", ms, total / (ms * 1e-3) / 8e12 * 100);
            launch_stream<>(d, n, dimg, out);
            CK(hipDeviceSynchronize());
            std::vector<uint32_t> a(n), b(n);
            CK(hipMemcpy(a.data(), out, n * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), ref, n * 4, hipMemcpyDeviceToHost));
            printf("product == regular kernel: %s\n", a == b ? "yes" : "NO");
        }
        CK(hipFree(d));
    }
    return 0;
}
