// copy_walk.hip -- why does a wave that walks a 16-row fragment copy slower than sixteen waves of one
// row each?  (The table-light CRC copy of GM's 65,456-byte payloads: 62% walking, 70-72% as one row per
// wave with LAMPI_CSUM_ROWS_HINT(16), while the read-only walk reads at 80%: DESIGN.md 4.5.1.)  The same
// question without the CRC: 1 GiB of 64 KiB fragments copied as 4 KiB rows (four coalesced 16-byte
// chunks per lane), 4-wave workgroups with 36 KiB of LDS (four per CU, as the light kernel), X dependent
// LDS lookups per 16 bytes as the CRC's latency proxy, non-temporal loads and stores:
//   row   one row per wave (16 waves per fragment)
//   walk  one wave per fragment, its 16 rows in order, the next row's loads in flight (the product)
//   ilv   a workgroup's four waves on its four fragments one at a time, wave w taking rows w, w+4, ...
//   blk   the same, wave w taking rows 4w .. 4w+3 of each
//   ro    walk, read-only (no stores)
//   ahd2  walk with two rows in flight
//   rowd  row, the row's address read from a descriptor array first (the descriptor batches' dependency)
//   rowdp rowd, each workgroup also touching the descriptors of workgroup blockIdx.x + 2048 (prefetch to L2)
//   blkW  W-wave workgroups (W = 8, 16) on W fragments one at a time, wave w taking rows w*16/W ..
//         (36 KiB of LDS per four waves: the same sixteen waves per CU)
// Prints GB/s (read + write; read only for ro) and the fraction of 8 TB/s.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 copy_walk.hip -o copy_walk
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                   \
    do {                                                        \
        hipError_t e_ = (x);                                    \
        if (e_ != hipSuccess) {                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_)); \
            std::exit(1);                                       \
        }                                                       \
    } while (0)

constexpr int kRows = 16;  // rows per fragment
constexpr size_t kFrag = 4096 * kRows;
enum { ROW, WALK, ILV, BLK, RO, AHD2, BLK8, BLK16, ROWD, ROWDP };

template <int X>
__device__ __forceinline__ uint32_t work(const uint32_t *lds, const u32x4 (&v)[4], uint32_t acc) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 4 * X; ++k) acc = lds[((acc ^ v[q][k & 3]) & 255u) * 4 + (k & 3)] ^ acc;
    return acc;
}

__device__ __forceinline__ void load_row(const uint8_t *src, size_t row, uint32_t lane, u32x4 (&v)[4]) {
    const u32x4 *s = reinterpret_cast<const u32x4 *>(src + row * 4096) + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = __builtin_nontemporal_load(s + 64 * q);
    __builtin_amdgcn_sched_barrier(0);  // (the scheduler sank prefetches below the next row's lookups)
}
__device__ __forceinline__ void store_row(uint8_t *dst, size_t row, uint32_t lane, const u32x4 (&v)[4]) {
    u32x4 *d = reinterpret_cast<u32x4 *>(dst + row * 4096) + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(v[q], d + 64 * q);
}

// row index (global, 4 KiB units) of step i of this wave
template <int M>
__device__ __forceinline__ size_t row_of(size_t b, uint32_t w, int i) {
    if (M == ILV) return (4 * b + (i >> 2)) * kRows + (size_t)(w + 4 * (i & 3));
    if (M == BLK) return (4 * b + (i >> 2)) * kRows + (size_t)(4 * w + (i & 3));
    if (M == BLK8) return (8 * b + (i >> 1)) * kRows + (size_t)(2 * w + (i & 1));
    if (M == BLK16) return (16 * b + i) * kRows + (size_t)w;
    return (4 * b + w) * kRows + (size_t)i;  // WALK, RO, AHD2
}

template <int M>
constexpr int waves_of() { return M == BLK8 ? 8 : M == BLK16 ? 16 : 4; }

template <int M, int X>
__global__ void __launch_bounds__(64 * waves_of<M>()) copy_walk(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                 size_t nfrag, uint32_t *sink, const uint64_t *__restrict__ desc) {
    constexpr int kW = waves_of<M>();
    __shared__ uint32_t lds[9216 * (kW / 4)];  // 36 KiB per four waves: sixteen waves per CU
    for (uint32_t i = threadIdx.x; i < sizeof(lds) / 16; i += 64 * kW)
        reinterpret_cast<u32x4 *>(lds)[i] = u32x4{i, i * 3u, i ^ 7u, i + 11u};
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const size_t b = blockIdx.x;
    uint32_t acc = lane;
    if (M == ROWD || M == ROWDP) {
        const size_t item = b * 4 + w;
        if (M == ROWDP && threadIdx.x < 4) {  // the descriptors of a later workgroup, into L2
            const size_t later = min((b + 2048) * 4 + threadIdx.x, nfrag * kRows - 1);
            uint32_t x = (uint32_t)__builtin_nontemporal_load(desc + later);
            asm volatile("" ::"v"(x));
        }
        const size_t row = __builtin_amdgcn_readfirstlane((uint32_t)desc[item]);  // (row index: < 2^32)
        u32x4 v[4];
        load_row(src, row, lane, v);
        __syncthreads();
        acc = work<X>(lds, v, acc);
        store_row(dst, row, lane, v);
    } else if (M == ROW) {
        const size_t row = b * 4 + w;
        u32x4 v[4];
        load_row(src, row, lane, v);
        __syncthreads();
        acc = work<X>(lds, v, acc);
        store_row(dst, row, lane, v);
    } else if (M == AHD2) {
        u32x4 v0[4], v1[4], v2[4];
        load_row(src, row_of<M>(b, w, 0), lane, v0);
        load_row(src, row_of<M>(b, w, 1), lane, v1);
        __syncthreads();
        for (int i = 0; i < kRows; i += 3) {
            if (i + 2 < kRows) load_row(src, row_of<M>(b, w, i + 2), lane, v2);
            acc = work<X>(lds, v0, acc);
            store_row(dst, row_of<M>(b, w, i), lane, v0);
            if (i + 1 >= kRows) break;
            if (i + 3 < kRows) load_row(src, row_of<M>(b, w, i + 3), lane, v0);
            acc = work<X>(lds, v1, acc);
            store_row(dst, row_of<M>(b, w, i + 1), lane, v1);
            if (i + 2 >= kRows) break;
            if (i + 4 < kRows) load_row(src, row_of<M>(b, w, i + 4), lane, v1);
            acc = work<X>(lds, v2, acc);
            store_row(dst, row_of<M>(b, w, i + 2), lane, v2);
        }
    } else {
        u32x4 v0[4], v1[4];
        load_row(src, row_of<M>(b, w, 0), lane, v0);
        __syncthreads();
        for (int i = 0; i < kRows; i += 2) {
            load_row(src, row_of<M>(b, w, i + 1), lane, v1);
            acc = work<X>(lds, v0, acc);
            if (M != RO) store_row(dst, row_of<M>(b, w, i), lane, v0);
            if (i + 2 < kRows) load_row(src, row_of<M>(b, w, i + 2), lane, v0);
            acc = work<X>(lds, v1, acc);
            if (M != RO) store_row(dst, row_of<M>(b, w, i + 1), lane, v1);
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the lookups alive
}

template <int M, int X>
static void run(const uint8_t *src, uint8_t *dst, size_t nfrag, uint32_t *sink, const uint64_t *desc, const char *tag) {
    constexpr int kW = waves_of<M>();
    const bool rows = M == ROW || M == ROWD || M == ROWDP;
    const unsigned grid = rows ? (unsigned)(nfrag * kRows / 4) : (unsigned)(nfrag / kW);
    for (int i = 0; i < 20; ++i) copy_walk<M, X><<<grid, 64 * kW>>>(src, dst, nfrag, sink, desc);
    CK(hipDeviceSynchronize());
    hipEvent_t a, e;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&e));
    CK(hipEventRecord(a));
    const int reps = 20;
    for (int i = 0; i < reps; ++i) copy_walk<M, X><<<grid, 64 * kW>>>(src, dst, nfrag, sink, desc);
    CK(hipEventRecord(e));
    CK(hipEventSynchronize(e));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, e));
    const double bytes = (M == RO ? 1.0 : 2.0) * nfrag * kFrag;
    const double gbs = bytes / (ms / reps * 1e-3) / 1e9;
    std::printf("%-6s X=%d: %7.1f GB/s = %.3f\n", tag, X, gbs, gbs / 8000.0);
    std::fflush(stdout);
}

template <int X>
static void all(const uint8_t *src, uint8_t *dst, size_t nfrag, uint32_t *sink, const uint64_t *desc) {
    run<ROW, X>(src, dst, nfrag, sink, desc, "row");
    run<ROWD, X>(src, dst, nfrag, sink, desc, "rowd");
    run<ROWDP, X>(src, dst, nfrag, sink, desc, "rowdp");
    run<WALK, X>(src, dst, nfrag, sink, desc, "walk");
    run<ILV, X>(src, dst, nfrag, sink, desc, "ilv");
    run<BLK, X>(src, dst, nfrag, sink, desc, "blk");
    run<RO, X>(src, dst, nfrag, sink, desc, "ro");
    run<AHD2, X>(src, dst, nfrag, sink, desc, "ahd2");
    run<BLK8, X>(src, dst, nfrag, sink, desc, "blk8");
    run<BLK16, X>(src, dst, nfrag, sink, desc, "blk16");
}

int main(int argc, char **argv) {
    const size_t nfrag = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 16384;  // default 1 GiB
    std::printf("%zu fragments of 64 KiB\n", nfrag);
    uint8_t *src, *dst;
    uint32_t *sink;
    CK(hipMalloc(&src, nfrag * kFrag));
    CK(hipMalloc(&dst, nfrag * kFrag));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 0x5A, nfrag * kFrag));
    // descriptors: row i of the batch is row i (identity), one 8-byte word each
    uint64_t *desc;
    const size_t nrows = nfrag * kRows;
    CK(hipMalloc(&desc, nrows * 8));
    uint64_t *h = (uint64_t *)std::malloc(nrows * 8);
    for (size_t i = 0; i < nrows; ++i) h[i] = i;
    CK(hipMemcpy(desc, h, nrows * 8, hipMemcpyHostToDevice));
    std::free(h);
    all<4>(src, dst, nfrag, sink, desc);
    std::printf("done\n");
    return 0;
}
