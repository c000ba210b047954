// Read-bandwidth and LDS-lookup microbenchmarks for the fragment-CRC kernel design.
// Measures, on one MI355X:
//   1. coalesced dwordx4 streaming read (the HBM-read roofline we can actually reach)
//   2. one wave per 4 KiB block, lane-contiguous 64 B (4 x dwordx4 at 64 B lane stride)
//   3. one wave per 16 KiB block, lane-contiguous 256 B (16 x dwordx4 at 256 B lane stride)
//   4. one wave per 4 KiB block, coalesced (lane reads 16 B of each 1 KiB row)
//   5. LDS table lookups/clk with v_perm-formed addresses (replicated, conflict-free layout)
// Build: hipcc --offload-arch=gfx950 -O3 readbw.hip -o readbw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__device__ __forceinline__ unsigned x4(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

__global__ void rd_coal(const uint4* __restrict__ p, size_t n16, unsigned* out) {
  unsigned acc = 0;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= x4(a) ^ x4(b) ^ x4(c) ^ x4(d);
  }
  for (; i < n16; i += stride) acc ^= x4(p[i]);
  if (acc == 0x9E3779B9u) out[0] = acc;
}

// one wave per block of 64*G bytes, lane-contiguous G bytes (G/16 dwordx4 per lane)
template <int G>
__global__ void rd_lane(const uint4* __restrict__ p, size_t nblk, unsigned* out) {
  const int lane = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nwave = ((size_t)gridDim.x * blockDim.x) >> 6;
  unsigned acc = 0;
  for (size_t b = wave; b < nblk; b += nwave) {
    const uint4* q = p + b * (64 * G / 16) + lane * (G / 16);
    uint4 v[G / 16];
#pragma unroll
    for (int i = 0; i < G / 16; ++i) v[i] = q[i];
#pragma unroll
    for (int i = 0; i < G / 16; ++i) acc ^= x4(v[i]);
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

// one wave per block of 64*G bytes, coalesced: lane reads 16 B of each 1 KiB row
template <int G>
__global__ void rd_rows(const uint4* __restrict__ p, size_t nblk, unsigned* out) {
  const int lane = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nwave = ((size_t)gridDim.x * blockDim.x) >> 6;
  unsigned acc = 0;
  for (size_t b = wave; b < nblk; b += nwave) {
    const uint4* q = p + b * (64 * G / 16) + lane;
    uint4 v[G / 16];
#pragma unroll
    for (int i = 0; i < G / 16; ++i) v[i] = q[i * 64];
#pragma unroll
    for (int i = 0; i < G / 16; ++i) acc ^= x4(v[i]);
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

// LDS lookup throughput: 64 KiB table, 4 tables x 256 entries x 16 copies (row = 256 B),
// lanes 0-15 / 16-31 use tables of opposite parity in the same instruction.
__global__ void __launch_bounds__(1024) lds_lookup(unsigned* out, int iters, unsigned seed) {
  extern __shared__ __attribute__((aligned(16))) unsigned tab[];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) tab[i] = i * 0x9E3779B9u;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned c = (lane & 15) * 4;
  const unsigned lanec = c | ((c + 64) << 8) | ((c + 128) << 16) | ((c + 192) << 24);
  const bool hi = (lane & 16) != 0;
  // selector: byte0 <- lanec byte t (src1 bytes are 0..3), byte1 <- x byte k (src0 bytes 4..7)
  unsigned sel[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int t = hi ? (i ^ 1) : i;
    sel[i] = (unsigned)t | ((unsigned)(4 + t) << 8) | (0x0Cu << 16) | (0x0Cu << 24);
  }
  unsigned x0 = seed ^ threadIdx.x * 0x85EBCA6Bu, x1 = x0 * 3 + 1, x2 = x0 * 5 + 7, x3 = x0 * 9 + 3;
  for (int it = 0; it < iters; ++it) {
    unsigned y0 = 0, y1 = 0, y2 = 0, y3 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y0 ^= tab[__builtin_amdgcn_perm(x0, lanec, sel[i]) >> 2];
      y1 ^= tab[__builtin_amdgcn_perm(x1, lanec, sel[i]) >> 2];
      y2 ^= tab[__builtin_amdgcn_perm(x2, lanec, sel[i]) >> 2];
      y3 ^= tab[__builtin_amdgcn_perm(x3, lanec, sel[i]) >> 2];
    }
    x0 ^= y0; x1 ^= y1; x2 ^= y2; x3 ^= y3;
  }
  unsigned r = x0 ^ x1 ^ x2 ^ x3;
  if (r == 0x9E3779B9u) out[0] = r;
}

int main(int argc, char** argv) {
  size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 30));
  int cus = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  cus = prop.multiProcessorCount;
  printf("device %s CUs=%d clock=%d kHz\n", prop.name, cus, prop.clockRate);
  void* buf;
  unsigned* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0x5A, bytes));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch, double nbytes) {
    launch();
    CK(hipDeviceSynchronize());
    const int reps = 5;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    double s = ms / 1e3 / reps;
    printf("%-40s %8.3f ms  %8.1f GB/s\n", name, s * 1e3, nbytes / s / 1e9);
    fflush(stdout);
  };
  const uint4* p = (const uint4*)buf;
  size_t n16 = bytes / 16;
  for (int bs : {256, 512, 1024}) {
    for (int per : {1, 2, 4, 8, 16}) {
      int grid = cus * per * (1024 / bs);
      if (bs * per * (1024 / bs) > 2048 * 4) continue;
      char nm[128];
      snprintf(nm, sizeof nm, "coal bs=%d grid=%d", bs, grid);
      timeit(nm, [&] { rd_coal<<<grid, bs>>>(p, n16, out); }, (double)bytes);
    }
  }
  for (int bs : {256, 1024}) {
    for (int per : {2, 4, 8}) {
      int grid = cus * per * (1024 / bs);
      char nm[128];
      snprintf(nm, sizeof nm, "lane64 bs=%d grid=%d", bs, grid);
      timeit(nm, [&] { rd_lane<64><<<grid, bs>>>(p, bytes / 4096, out); }, (double)bytes);
      snprintf(nm, sizeof nm, "rows4K bs=%d grid=%d", bs, grid);
      timeit(nm, [&] { rd_rows<64><<<grid, bs>>>(p, bytes / 4096, out); }, (double)bytes);
      snprintf(nm, sizeof nm, "lane256 bs=%d grid=%d", bs, grid);
      timeit(nm, [&] { rd_lane<256><<<grid, bs>>>(p, bytes / 16384, out); }, (double)bytes);
      snprintf(nm, sizeof nm, "rows16K bs=%d grid=%d", bs, grid);
      timeit(nm, [&] { rd_rows<256><<<grid, bs>>>(p, bytes / 16384, out); }, (double)bytes);
    }
  }
  // non-persistent: one wave per block, full grid
  {
    size_t nblk = bytes / 4096;
    int grid = (int)(nblk / 4);
    timeit("lane64 nonpersistent bs=256", [&] { rd_lane<64><<<grid, 256>>>(p, nblk, out); }, (double)bytes);
    timeit("rows4K nonpersistent bs=256", [&] { rd_rows<64><<<grid, 256>>>(p, nblk, out); }, (double)bytes);
  }
  // LDS lookup throughput
  {
    const int iters = 4096;
    for (int bs : {256, 512, 1024}) {
      int grid = cus * (1024 / bs) * 2;
      size_t lookups = (size_t)grid * bs * iters * 16;
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      lds_lookup<<<grid, bs, 65536>>>(out, 16, 1);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      lds_lookup<<<grid, bs, 65536>>>(out, iters, 1);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      double per_s = lookups / (ms / 1e3);
      printf("lds_lookup bs=%d grid=%d: %.3f ms, %.2f Tlookup/s = %.2f lookups/clk/CU @2.4GHz\n", bs, grid, ms,
             per_s / 1e12, per_s / cus / 2.4e9);
    }
  }
  CK(hipFree(buf));
  printf("done\n");
  return 0;
}
