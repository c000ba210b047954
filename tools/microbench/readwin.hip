// readwin.hip -- persistent grids that keep the chip-wide read window tight.
//   PS : persistent, grid = resident workgroups G; workgroup b's step i reads chunk i*G + b
//        (chunk = 4 waves x cpw fragments, wave w reads fragments w, w+4, ... of the chunk)
//   TK : persistent, workgroup-level tickets: lane 0 of wave 0 takes the next chunk from its
//        XCD's counter (chunks of counter q: q, q+8, q+16, ...), broadcast through LDS;
//        the ticket for chunk k+1 is fetched while chunk k is read.
// All loads in flight per wave: depth fragments.  64 KiB dynamic LDS -> 2 workgroups per CU.
// Build: hipcc --offload-arch=gfx950 -O3 readwin.hip -o readwin
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

__device__ __forceinline__ unsigned xor_frag(const u32x4 *p, unsigned f, unsigned lane) {
    const u32x4 *q = p + (size_t)f * 256 + lane * 4;
    u32x4 a = q[0], b = q[1], c = q[2], d = q[3];
    return a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
}

// chunk = 4*cpw consecutive fragments; wave w reads w, w+4, ..., cpw of them
__device__ __forceinline__ unsigned read_chunk(const u32x4 *p, unsigned nfrag, unsigned chunk, unsigned cpw,
                                               unsigned wib, unsigned lane) {
    unsigned acc = 0;
    const unsigned b0 = chunk * 4 * cpw + wib;
    for (unsigned i = 0; i < cpw; i += 4) {
        unsigned f[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            f[d] = b0 + 4 * (i + d);
            if (f[d] >= nfrag || i + d >= cpw) f[d] = b0 < nfrag ? b0 : 0;
        }
        u32x4 v[4][4];
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int k = 0; k < 4; ++k) v[d][k] = p[(size_t)f[d] * 256 + lane * 4 + k];
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc ^= v[d][k].x ^ v[d][k].y ^ v[d][k].z ^ v[d][k].w;
    }
    return acc;
}

__global__ void __launch_bounds__(256) rd_ps(const u32x4 *__restrict__ p, unsigned nfrag, unsigned cpw, unsigned *out) {
    extern __shared__ unsigned lds[];
    const unsigned lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    if (threadIdx.x == 0) lds[0] = blockIdx.x;
    const unsigned nchunk = (nfrag + 4 * cpw - 1) / (4 * cpw);
    unsigned acc = 0;
    for (unsigned c = blockIdx.x; c < nchunk; c += gridDim.x) acc ^= read_chunk(p, nfrag, c, cpw, wib, lane);
    if (acc == 0x9E3779B9u) out[0] = acc + lds[0];
}

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 7u; }

// next chunk from the home queue (chunks q, q+8, ...), stealing from others when it is dry
__device__ __forceinline__ unsigned take(unsigned *q, unsigned nchunk, unsigned home) {
    for (unsigned s = 0; s < 8; ++s) {
        const unsigned qi = (home + s) & 7u;
        const unsigned mine = nchunk > qi ? (nchunk - qi + 7) / 8 : 0;
        const unsigned g = atomicAdd(q + qi * 32, 1u);
        if (g < mine) return qi + 8 * g;
    }
    return nchunk;
}

__global__ void __launch_bounds__(256) rd_tk(const u32x4 *__restrict__ p, unsigned nfrag, unsigned cpw, unsigned *q,
                                             unsigned *out) {
    extern __shared__ unsigned lds[];
    const unsigned lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const unsigned nchunk = (nfrag + 4 * cpw - 1) / (4 * cpw);
    const unsigned home = xcc_id();
    if (threadIdx.x == 0) {
        lds[0] = take(q, nchunk, home);
        lds[1] = take(q, nchunk, home);
    }
    __syncthreads();
    unsigned cur = lds[0], nxt = lds[1];
    unsigned acc = 0;
    unsigned slot = 0;
    while (cur < nchunk) {
        // fetch the ticket after next while this chunk is read
        unsigned t2 = 0;
        if (threadIdx.x == 0) t2 = nxt < nchunk ? take(q, nchunk, home) : nchunk;
        acc ^= read_chunk(p, nfrag, cur, cpw, wib, lane);
        if (threadIdx.x == 0) lds[2 + slot] = t2;
        __syncthreads();
        cur = nxt;
        nxt = lds[2 + slot];
        slot ^= 1;
    }
    if (acc == 0x9E3779B9u) out[0] = acc + lds[0];
}

// per-wave tickets, kLook grabs in flight: ticket = `cpw` consecutive fragments; queue q
// (the wave's XCD) hands out chunks q, q+8, ... so all XCDs sweep one window together
template <int kLook>
__global__ void __launch_bounds__(256) rd_tw(const u32x4 *__restrict__ p, unsigned nfrag, unsigned cpw, unsigned *q,
                                             unsigned *out) {
    extern __shared__ unsigned lds[];
    const unsigned lane = threadIdx.x & 63;
    if (threadIdx.x == 0) lds[0] = blockIdx.x;
    const unsigned nchunk = (nfrag + cpw - 1) / cpw;
    const unsigned home = xcc_id();
    unsigned tk[kLook];
#pragma unroll
    for (int i = 0; i < kLook; ++i) {
        unsigned g = 0;
        if (lane == 0) g = take(q, nchunk, home);
        tk[i] = __builtin_amdgcn_readfirstlane(g);
    }
    unsigned acc = 0;
    for (;;) {
        const unsigned cur = tk[0];
        if (cur >= nchunk) break;
#pragma unroll
        for (int i = 0; i + 1 < kLook; ++i) tk[i] = tk[i + 1];
        unsigned g = 0;
        if (lane == 0) g = take(q, nchunk, home);
        tk[kLook - 1] = __builtin_amdgcn_readfirstlane(g);
        const unsigned f0 = cur * cpw;
        for (unsigned i = 0; i < cpw; i += 2) {
            unsigned fa = f0 + i, fb = f0 + i + 1;
            if (fa >= nfrag) fa = f0;
            if (fb >= nfrag || i + 1 >= cpw) fb = fa;
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = p[(size_t)fa * 256 + lane * 4 + k];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[4 + k] = p[(size_t)fb * 256 + lane * 4 + k];
#pragma unroll
            for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
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
        char mode;
        unsigned cpw;
        int wg_per_cu;
    };
    const Cfg cfgs[] = {{'P', 8, 2}, {'2', 4, 2}, {'2', 8, 2}, {'2', 16, 2}, {'4', 4, 2},
                        {'4', 8, 2}, {'4', 16, 2}, {'4', 8, 8}, {'2', 8, 4}};
    for (const Cfg &c : cfgs) {
        const int grid = cus * c.wg_per_cu;
        auto launch = [&] {
            if (c.mode == 'P') {
                hipLaunchKernelGGL(rd_ps, dim3(grid), dim3(256), 65536, 0, (const u32x4 *)buf, nfrag, c.cpw, out);
            } else if (c.mode == '2' || c.mode == '4') {
                CK(hipMemsetAsync(q, 0, 8 * 32 * 4, 0));
                const int lds = c.wg_per_cu <= 2 ? 65536 : (c.wg_per_cu <= 4 ? 32768 : 0);
                if (c.mode == '2')
                    hipLaunchKernelGGL(rd_tw<2>, dim3(grid), dim3(256), lds, 0, (const u32x4 *)buf, nfrag, c.cpw, q, out);
                else
                    hipLaunchKernelGGL(rd_tw<4>, dim3(grid), dim3(256), lds, 0, (const u32x4 *)buf, nfrag, c.cpw, q, out);
            } else {
                CK(hipMemsetAsync(q, 0, 8 * 32 * 4, 0));
                hipLaunchKernelGGL(rd_tk, dim3(grid), dim3(256), 65536, 0, (const u32x4 *)buf, nfrag, c.cpw, q, out);
            }
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
        printf("%c cpw=%2u wg/cu=%d grid=%5d  %7.3f ms  %7.1f GB/s (%5.1f%%)\n", c.mode, c.cpw, c.wg_per_cu, grid,
               s * 1e3, bytes / s / 1e9, bytes / s / 8e10);
        fflush(stdout);
    }
    return 0;
}
