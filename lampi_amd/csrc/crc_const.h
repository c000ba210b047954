// crc_const.h -- compile-time GF(2) algebra for CRC-32/MPEG-2 (constexpr, host and device).
//
// The same quantities as crc_tables.cc computes at run time, evaluated by the compiler so a
// kernel can build its slicing and Horner tables from immediates instead of loading a basis
// image (frag_csum.hip, stage_tables): the table staging then waits on no memory at all.
// crc_tables.cc checks every value here against its own run-time tables (build_table_image).
//
// Semantics follow the reference table generator ulm_initialize_crc_table
// (src/util/MemFunctions.cc:1242-1261): polynomial 0x04C11DB7, MSB-first.
#pragma once
#include <cstdint>

namespace lampi {
namespace cx {

constexpr uint32_t kPoly = 0x04C11DB7u;

constexpr uint32_t bswap(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// Sarwate table entry T[i]: byte i in bits 31..24 shifted through eight polynomial steps
constexpr uint32_t sarwate(uint32_t i) {
    uint32_t r = i << 24;
    for (int k = 0; k < 8; ++k) r = (r & 0x80000000u) ? (r << 1) ^ kPoly : (r << 1);
    return r;
}

// register after one zero byte
constexpr uint32_t zero_byte(uint32_t c) { return (c << 8) ^ sarwate(c >> 24); }

// slicing-by-4 table S_j[i] in the swapped domain (crc_tables.cc slice_tables)
constexpr uint32_t slice(int j, uint32_t i) {
    uint32_t v = sarwate(i);
    for (int k = 0; k < 3 - j; ++k) v = zero_byte(v);
    return bswap(v);
}

// 32x32 GF(2) matrix as column images, c[b] = M(1 << b)
struct Mat {
    uint32_t c[32];
};

constexpr uint32_t apply(const Mat &m, uint32_t v) {
    uint32_t r = 0;
    for (int b = 0; b < 32; ++b)
        if ((v >> b) & 1u) r ^= m.c[b];
    return r;
}

constexpr Mat mul(const Mat &a, const Mat &b) {  // a o b
    Mat r{};
    for (int k = 0; k < 32; ++k) r.c[k] = apply(a, b.c[k]);
    return r;
}

// register after n zero bytes (square and multiply from the one-byte step)
constexpr Mat shift(uint64_t n) {
    Mat one{}, acc{};
    for (int b = 0; b < 32; ++b) {
        one.c[b] = zero_byte(1u << b);
        acc.c[b] = 1u << b;
    }
    for (; n; n >>= 1) {
        if (n & 1u) acc = mul(one, acc);
        one = mul(one, one);
    }
    return acc;
}

// bswap o m o bswap: the same map on byte-swapped registers
constexpr Mat swapped(const Mat &m) {
    Mat r{};
    for (int b = 0; b < 32; ++b) r.c[b] = bswap(apply(m, bswap(1u << b)));
    return r;
}

// Slicing-table basis: S_j is linear in its index, so S_j[i] = XOR of lo[j][b] over the set
// bits b < 5 of i, XOR hi[j][i >> 5].
struct SliceBasis {
    uint32_t lo[4][5];  // S_j[1 << b]
    uint32_t hi[4][8];  // S_j[32 k]
};

constexpr SliceBasis slice_basis() {
    SliceBasis s{};
    for (int j = 0; j < 4; ++j) {
        for (int b = 0; b < 5; ++b) s.lo[j][b] = slice(j, 1u << b);
        for (int k = 0; k < 8; ++k) s.hi[j][k] = slice(j, 32u * (uint32_t)k);
    }
    return s;
}

}  // namespace cx
}  // namespace lampi
