// recv_ceiling.hip -- the copy ceiling of the GM receive step's exact shape: 16,384 fragments of
// 65,456 bytes read from GM receive slots (64 KiB stride, payload at slot + 72: 8 bytes past a 16-byte boundary)
// and written to one contiguous application buffer (fragment k at app + 65,456 k: 16-byte aligned).  No checksum:
// plain copies, read + write bytes counted against 8 TB/s.
//   rows     : the product's shape (crc_light_frag_copy_kernel<RecvSource> with 16 row groups): one wave per 4 KiB
//              row of a right-aligned 64 KiB frame (front padding 80 bytes), lane l the 16-byte chunks at
//              1024 q + 16 l of the row, 4-wave workgroups holding LDS bytes of static LDS (36 KiB: four per CU,
//              as the table-light kernel), non-temporal unaligned 16-byte loads and stores
//   rows_al  : the same with the payload at slot + 64 (16-byte aligned source): what the misalignment costs
//   rows_fs  : rows, the source read as aligned 16-byte chunks and funnel-shifted across lanes (wave_shr:1)
//   rows_lds0: rows without the LDS (residency by registers only)
//   wgrow    : one 256-thread workgroup per frame row, thread t the 16 bytes at 16 t (the textbook copy in the slots)
//   rows_lds80: rows holding 80 KiB of LDS (two workgroups per CU)
//   wgrow4   : rows' workgroup span (four consecutive rows) with wave w taking quarter w of each row
//   rows_xf  : rows with the four waves of a workgroup on row r of four different fragments
//   rows_lc  : rows with lane-contiguous 64-byte pieces (the read kernels' layout)
//   flat     : the textbook float4 copy of the same bytes as one contiguous aligned range (no slots)
// Three interleaved rounds, 20 launches each.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 recv_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("HIP %d at %d\n", (int)e_, __LINE__);                        \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 __attribute__((aligned(1))) gsrc_a1;
typedef __attribute__((address_space(1))) const u32x4 __attribute__((aligned(16))) gsrc_a16;
typedef __attribute__((address_space(1))) u32x4 __attribute__((aligned(1))) gdst_a1;

constexpr size_t kN = 16384, kL = 65456, kSlot = 65536, kRows = 16, kP = kRows * 4096 - kL;  // 80

template <int kLds>
__global__ void __launch_bounds__(256) rows_kernel(const uint8_t *__restrict__ ring, size_t hdr, uint8_t *__restrict__ app) {
    __shared__ uint32_t pad[kLds > 0 ? kLds / 4 : 1];
    if constexpr (kLds > 0)
        if (threadIdx.x == 1024) pad[0] = 0;  // (never: keeps the LDS allocated)
    const size_t item = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const size_t f = item / kRows;
    const uint32_t r = (uint32_t)(item % kRows);
    const uint8_t *src = ring + f * kSlot + hdr;
    uint8_t *dst = app + f * kL;
    u32x4 d[4];
    int64_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        o[q] = (int64_t)r * 4096 + 1024 * q + 16 * lane - (int64_t)kP;
        if (o[q] >= 0) d[q] = __builtin_nontemporal_load((gsrc_a1 *)(src + o[q]));
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (o[q] >= 0) __builtin_nontemporal_store(d[q], (gdst_a1 *)(dst + o[q]));
    // (the frame's first chunk of row 0 starts 80 bytes before the fragment: chunks o < 0 are padding; the
    // 16 bytes at o = -16..-1 never exist since kP % 16 == 0)
}

// aligned source chunks funnel-shifted: the fragment's byte b lies in aligned chunk (src + b) & ~15; with the source
// 8 bytes off the grid, the 16 bytes a lane stores are the high half of its aligned chunk c and the low half of c + 1
__global__ void __launch_bounds__(256) rows_fs_kernel(const uint8_t *__restrict__ ring, size_t hdr, uint8_t *__restrict__ app) {
    __shared__ uint32_t pad[36 * 1024 / 4];
    if (threadIdx.x == 1024) pad[0] = 0;
    const size_t item = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const size_t f = item / kRows;
    const uint32_t r = (uint32_t)(item % kRows);
    const uint8_t *src = ring + f * kSlot + hdr;
    uint8_t *dst = app + f * kL;
    const uintptr_t mis = (uintptr_t)src & 15u;  // 8
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t o = (int64_t)r * 4096 + 1024 * q + 16 * lane - (int64_t)kP;
        // aligned chunk holding byte o, and the next one (the next lane's, by a wave shift; lane 63 loads its own)
        const int64_t a = o - (int64_t)mis;  // (src + a) is 16-byte aligned
        const bool in = a + 16 > 0 && a < (int64_t)kL;
        u32x4 lo = in ? __builtin_nontemporal_load((gsrc_a16 *)(src + a)) : u32x4{0, 0, 0, 0};
        u32x4 hi;
        hi.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo.x, 0x130, 0xF, 0xF, false);  // wave_shl:1
        hi.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo.y, 0x130, 0xF, 0xF, false);
        hi.z = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo.z, 0x130, 0xF, 0xF, false);
        hi.w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo.w, 0x130, 0xF, 0xF, false);
        if (lane == 63 && a + 16 < (int64_t)kL + 16) hi = __builtin_nontemporal_load((gsrc_a16 *)(src + a + 16));
        // bytes 8..15 of lo then 0..7 of hi (mis == 8)
        const u32x4 v{lo.z, lo.w, hi.x, hi.y};
        if (o >= 0) __builtin_nontemporal_store(v, (gdst_a1 *)(dst + o));
    }
}

// one 256-thread workgroup per frame row, thread t the chunk at 16 t (the textbook copy inside the slot layout: wave w
// a 1 KiB quarter of the row)
__global__ void __launch_bounds__(256) wgrow_kernel(const uint8_t *__restrict__ ring, size_t hdr, uint8_t *__restrict__ app) {
    const size_t item = blockIdx.x;
    const size_t f = item / kRows;
    const uint32_t r = (uint32_t)(item % kRows);
    const uint8_t *src = ring + f * kSlot + hdr;
    uint8_t *dst = app + f * kL;
    const int64_t o = (int64_t)r * 4096 + 16 * threadIdx.x - (int64_t)kP;
    if (o >= 0) __builtin_nontemporal_store(__builtin_nontemporal_load((gsrc_a1 *)(src + o)), (gdst_a1 *)(dst + o));
}

// rows, but the four waves of a workgroup on four different fragments (row r of fragments 4i .. 4i + 3)
__global__ void __launch_bounds__(256) rows_xf_kernel(const uint8_t *__restrict__ ring, size_t hdr, uint8_t *__restrict__ app) {
    __shared__ uint32_t pad[36 * 1024 / 4];
    if (threadIdx.x == 1024) pad[0] = 0;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const size_t b = blockIdx.x;                 // (fragment quad, row)
    const size_t f = (b / kRows) * 4 + w;
    const uint32_t r = (uint32_t)(b % kRows);
    const uint8_t *src = ring + f * kSlot + hdr;
    uint8_t *dst = app + f * kL;
    u32x4 d[4];
    int64_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        o[q] = (int64_t)r * 4096 + 1024 * q + 16 * lane - (int64_t)kP;
        if (o[q] >= 0) d[q] = __builtin_nontemporal_load((gsrc_a1 *)(src + o[q]));
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (o[q] >= 0) __builtin_nontemporal_store(d[q], (gdst_a1 *)(dst + o[q]));
}

// rows with lane-contiguous 64-byte pieces (lane l: bytes 64 l .. 64 l + 63 of the row, four loads each): the read
// kernels' layout
__global__ void __launch_bounds__(256) rows_lc_kernel(const uint8_t *__restrict__ ring, size_t hdr, uint8_t *__restrict__ app) {
    __shared__ uint32_t pad[36 * 1024 / 4];
    if (threadIdx.x == 1024) pad[0] = 0;
    const size_t item = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const size_t f = item / kRows;
    const uint32_t r = (uint32_t)(item % kRows);
    const uint8_t *src = ring + f * kSlot + hdr;
    uint8_t *dst = app + f * kL;
    u32x4 d[4];
    int64_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        o[q] = (int64_t)r * 4096 + 64 * lane + 16 * q - (int64_t)kP;
        if (o[q] >= 0) d[q] = __builtin_nontemporal_load((gsrc_a1 *)(src + o[q]));
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (o[q] >= 0) __builtin_nontemporal_store(d[q], (gdst_a1 *)(dst + o[q]));
}

// four consecutive rows per workgroup as rows does, but wave w takes quarter w of every row (chunk 1024 w + 16 l of
// rows 4b .. 4b + 3): 1 KiB wave instructions interleaved across the waves, four loads per lane
__global__ void __launch_bounds__(256) wgrow4_kernel(const uint8_t *__restrict__ ring, size_t hdr, uint8_t *__restrict__ app) {
    __shared__ uint32_t pad[36 * 1024 / 4];
    if (threadIdx.x == 1024) pad[0] = 0;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const size_t item0 = (size_t)blockIdx.x * 4;
    u32x4 d[4];
    int64_t o[4];
    const uint8_t *src[4];
    uint8_t *dst[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const size_t item = item0 + k, f = item / kRows;
        const uint32_t r = (uint32_t)(item % kRows);
        src[k] = ring + f * kSlot + hdr;
        dst[k] = app + f * kL;
        o[k] = (int64_t)r * 4096 + 1024 * w + 16 * lane - (int64_t)kP;
        if (o[k] >= 0) d[k] = __builtin_nontemporal_load((gsrc_a1 *)(src[k] + o[k]));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (o[k] >= 0) __builtin_nontemporal_store(d[k], (gdst_a1 *)(dst[k] + o[k]));
}

__global__ void __launch_bounds__(256) flat_kernel(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

int main() {
    uint8_t *ring = nullptr, *app = nullptr, *flat = nullptr;
    CK(hipMalloc(&ring, kN * kSlot));
    CK(hipMalloc(&app, kN * kL + 4096));
    CK(hipMalloc(&flat, kN * kL + 4096));
    std::vector<uint8_t> h(kN * kSlot);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < h.size(); i += 8) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        std::memcpy(&h[i], &x, 8);
    }
    CK(hipMemcpy(ring, h.data(), h.size(), hipMemcpyHostToDevice));
    const double bytes = 2.0 * kN * kL;
    const unsigned wgs = (unsigned)(kN * kRows / 4);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char *name, auto launch) {
        for (int i = 0; i < 5; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 20; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double s = ms / 20 / 1e3;
        std::printf("%-10s %8.1f us  %6.1f GB/s  %5.1f%%\n", name, s * 1e6, bytes / s / 1e9, bytes / s / 8e12 * 100);
    };
    // correctness of the shapes (every fragment's bytes delivered)
    auto check = [&](const char *name, size_t hdr) {
        std::vector<uint8_t> a(kN * kL);
        CK(hipMemcpy(a.data(), app, a.size(), hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t f = 0; f < kN; f += 97)
            bad += std::memcmp(&a[f * kL], &h[f * kSlot + hdr], kL) != 0;
        std::printf("%-10s check %s\n", name, bad ? "BAD" : "ok");
    };
    for (int round = 0; round < 3; ++round) {
        std::printf("round %d\n", round);
        timed("rows", [&] { hipLaunchKernelGGL(rows_kernel<36 * 1024>, dim3(wgs), dim3(256), 0, 0, ring, 72, app); });
        if (round == 0) check("rows", 72);
        timed("rows_al", [&] { hipLaunchKernelGGL(rows_kernel<36 * 1024>, dim3(wgs), dim3(256), 0, 0, ring, 64, app); });
        if (round == 0) check("rows_al", 64);
        timed("rows_fs", [&] { hipLaunchKernelGGL(rows_fs_kernel, dim3(wgs), dim3(256), 0, 0, ring, 72, app); });
        if (round == 0) check("rows_fs", 72);
        timed("rows_lds0", [&] { hipLaunchKernelGGL(rows_kernel<0>, dim3(wgs), dim3(256), 0, 0, ring, 72, app); });
        timed("rows_lds80", [&] { hipLaunchKernelGGL(rows_kernel<80 * 1024>, dim3(wgs), dim3(256), 0, 0, ring, 72, app); });
        timed("wgrow4", [&] { hipLaunchKernelGGL(wgrow4_kernel, dim3(wgs), dim3(256), 0, 0, ring, 72, app); });
        if (round == 0) check("wgrow4", 72);
        timed("wgrow", [&] {
            hipLaunchKernelGGL(wgrow_kernel, dim3((unsigned)(kN * kRows)), dim3(256), 0, 0, ring, 72, app);
        });
        if (round == 0) check("wgrow", 72);
        timed("rows_xf", [&] { hipLaunchKernelGGL(rows_xf_kernel, dim3(wgs), dim3(256), 0, 0, ring, 72, app); });
        if (round == 0) check("rows_xf", 72);
        timed("rows_lc", [&] { hipLaunchKernelGGL(rows_lc_kernel, dim3(wgs), dim3(256), 0, 0, ring, 72, app); });
        if (round == 0) check("rows_lc", 72);
        timed("flat", [&] {
            const size_t n16 = kN * kL / 16;
            hipLaunchKernelGGL(flat_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, 0, (const u32x4 *)ring,
                               (u32x4 *)flat, n16);
        });
    }
    return 0;
}
