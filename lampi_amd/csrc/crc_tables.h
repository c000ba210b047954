// crc_tables.h -- host-side GF(2) algebra for CRC-32/MPEG-2 and the lookup tables the
// gfx950 kernels stage into LDS.
//
// The CRC register update (ref src/util/MemFunctions.cc:1343-1364) is linear over GF(2)
// in (register, data), which gives the two identities every kernel relies on:
//   crc(s, A || B) = shift_|B|(crc(s, A)) ^ crc(0, B)          (split / combine)
//   crc(s, B)      = crc(0, B ^ bytes_BE(s)) for |B| >= 4       (init = data injection)
// where shift_n(c) is the register after n zero bytes.  No carry-less multiply exists on
// CDNA4, so shift_n is applied through precomputed nibble tables (8 lookups).
//
// The kernels hold the register byte-swapped ("swapped domain", C = bswap(c)) so that a
// little-endian 32-bit load XORs straight into it; every table here is in that domain.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace lampi {

constexpr uint32_t kCrcPoly = 0x04C11DB7u;
constexpr uint32_t kCrcInit = 0xFFFFFFFFu;

// Geometry of the row kernel: a fragment is cut into rows of 64 lanes x 64 bytes.
constexpr int kWave = 64;
constexpr int kLaneBytes = 64;
constexpr int kRowBytes = kWave * kLaneBytes;  // 4096

// Layout of the device table image (u32 words) -- copied into LDS by the kernels.
//   [kImgCombine, +8192)  per-lane final shift by 64*(63-l) bytes, nibble tables,
//                         word index p*1024 + v*64 + l  (LDS byte addr p*4096 + v*256 + 4l:
//                         lane l always hits bank l%32 -> conflict free)
//   [kImgHorner, +128)    shift by kRowBytes-kLaneBytes (4032) bytes, p*16 + v
//   [kImgSlice, +1024)    slicing-by-4 tables S_j[i] at j*256 + i (replicated in LDS)
constexpr size_t kImgCombine = 0;
constexpr size_t kImgHorner = 8192;
constexpr size_t kImgSlice = 8192 + 128;
constexpr size_t kImgWords = 8192 + 128 + 1024;

inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 32x32 GF(2) matrix stored as column images: col[b] = M * (1 << b).
struct Gf2Mat {
    uint32_t col[32];
    uint32_t apply(uint32_t v) const {
        uint32_t r = 0;
        for (int b = 0; b < 32; ++b)
            if (v >> b & 1u) r ^= col[b];
        return r;
    }
};

Gf2Mat mat_mul(const Gf2Mat &a, const Gf2Mat &b);  // a o b
Gf2Mat mat_identity();
Gf2Mat shift_matrix(uint64_t nbytes);               // register after nbytes zero bytes
Gf2Mat swapped(const Gf2Mat &m);                    // bswap o m o bswap

const uint32_t *sarwate_table();                    // T[i], MSB-first
uint32_t crc_bytes(uint32_t crc, const uint8_t *p, size_t n);  // host scalar (table init checks)

// Nibble tables of a swapped-domain linear map m: out[p*16 + v] = m(v << 4p).
void nibble_tables(const Gf2Mat &m_swapped, uint32_t out[128]);

// Full device table image, kImgWords words.
std::vector<uint32_t> build_table_image();

}  // namespace lampi
