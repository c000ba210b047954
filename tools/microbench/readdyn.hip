// readdyn.hip -- raw read bandwidth of a PERSISTENT grid that hands out 4 KiB fragments
// dynamically, in address order, so the whole chip sweeps a compact window (the shape that
// reached 83% non-persistent).  Queue modes:
//   0: one global counter                 (fragments in order)
//   1: 8 counters, queue q owns chunks q, q+8, q+16, ... (interleaved), waves use their XCD's
//      queue and steal from the others when it runs dry
// Each wave grabs `chunk` fragments per atomic and keeps one grab in flight.
// Build: hipcc --offload-arch=gfx950 -O3 readdyn.hip -o readdyn
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                                \
        }                                                                                           \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 7u; }

// returns the first fragment of the grabbed chunk, or nfrag when everything is handed out
template <int kQ>
__device__ __forceinline__ unsigned grab(unsigned *q, unsigned nfrag, unsigned chunk, unsigned home, int lane) {
    if (kQ == 0) {
        unsigned g = 0;
        if (lane == 0) g = atomicAdd(q, chunk);
        g = __builtin_amdgcn_readfirstlane(g);
        return g < nfrag ? g : nfrag;
    }
    const unsigned nchunks = (nfrag + chunk - 1) / chunk;
    for (unsigned s = 0; s < 8; ++s) {
        const unsigned qi = (home + s) & 7u;
        const unsigned mine = (nchunks > qi) ? (nchunks - qi + 7) / 8 : 0;  // chunks qi, qi+8, ...
        unsigned g = 0;
        if (lane == 0) g = atomicAdd(q + qi * 32, 1u);
        g = __builtin_amdgcn_readfirstlane(g);
        if (g < mine) return (qi + 8 * g) * chunk;
    }
    return nfrag;
}

template <int kQ>
__global__ void rd_dyn(const u32x4 *__restrict__ p, unsigned nfrag, unsigned chunk, unsigned *q, unsigned *out) {
    extern __shared__ unsigned lds[];
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) lds[0] = blockIdx.x;
    const unsigned home = kQ ? xcc_id() : 0u;
    unsigned acc = 0;
    unsigned cur = grab<kQ>(q, nfrag, chunk, home, lane);
    while (cur < nfrag) {
        const unsigned nxt = grab<kQ>(q, nfrag, chunk, home, lane);  // one grab ahead
        const unsigned end = min(nfrag, cur + chunk);
        for (unsigned f = cur; f < end; ++f) {
            const u32x4 *r = p + (size_t)f * 256 + lane * 4;
            u32x4 a = r[0], b = r[1], c = r[2], d = r[3];
            acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
        }
        cur = nxt;
    }
    if (acc == 0x9E3779B9u) out[0] = acc + lds[0];
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 30);
    const unsigned nfrag = (unsigned)(bytes / 4096);
    void *buf;
    unsigned *out, *q;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&q, 8 * 32 * 4));
    CK(hipMemset(buf, 0x5A, bytes));
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Cfg {
        int qmode, block, wg_per_cu, lds;
        unsigned chunk;
    };
    const Cfg cfgs[] = {
        {0, 256, 8, 0, 4},      {0, 256, 8, 0, 16},     {1, 256, 8, 0, 1},      {1, 256, 8, 0, 2},
        {1, 256, 8, 0, 4},      {1, 256, 8, 0, 16},     {1, 512, 3, 49152, 2},  {1, 512, 3, 49152, 4},
        {1, 1024, 1, 98816, 2}, {1, 1024, 1, 98816, 4}, {1, 256, 4, 32768, 2},  {1, 256, 4, 32768, 4},
        {1, 512, 2, 65536, 4},  {1, 512, 4, 0, 4},      {1, 1024, 2, 0, 4},     {1, 256, 6, 24576, 4},
    };
    for (const Cfg &c : cfgs) {
        const int grid = cus * c.wg_per_cu;
        auto launch = [&] {
            CK(hipMemsetAsync(q, 0, 8 * 32 * 4, 0));
            if (c.qmode == 0)
                hipLaunchKernelGGL(rd_dyn<0>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.chunk, q,
                                   out);
            else
                hipLaunchKernelGGL(rd_dyn<1>, dim3(grid), dim3(c.block), c.lds, 0, (const u32x4 *)buf, nfrag, c.chunk, q,
                                   out);
        };
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 8;
        float tot = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        const double s = tot / 1e3 / reps;
        printf("q=%d block=%4d wg/cu=%d lds=%6d chunk=%3u  %7.3f ms  %7.1f GB/s (%5.1f%%)\n", c.qmode, c.block,
               c.wg_per_cu, c.lds, c.chunk, s * 1e3, bytes / s / 1e9, bytes / s / 8e10);
        fflush(stdout);
    }
    return 0;
}
