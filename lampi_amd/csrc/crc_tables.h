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

// Layout of the device basis image (u32 words); each workgroup expands it into its LDS
// tables (frag_csum.hip, stage_tables):
//   [kImgSliceT, +1024)      slicing-by-4 tables transposed: word 4i + j = S_j[i]
//   [kImgCombineCols, +2048) per-lane final shift by 64*(63-l) bytes (swapped domain), as
//                            matrix columns: word l*32 + b = M_l(1 << b)
//   [kImgHornerCols, +32)    shift by kRowBytes - kLaneBytes = 4032 bytes, columns b
//   [kImgCombine16Cols, +2048), [kImgHorner16Cols, +32): the same for the coalesced layout
//                            of the fused-copy kernel (lane l owns the 16-byte chunks at
//                            16l + 1024k of each row): final shift 16*(63-l), step 1008 bytes
// Nibble tables are XORs of four columns: M(v << 4p) = XOR_{bit b of v} col[4p + b].
constexpr size_t kImgSliceT = 0;
constexpr size_t kImgCombineCols = 1024;
constexpr size_t kImgHornerCols = 1024 + 2048;
constexpr size_t kImgCombine16Cols = kImgHornerCols + 32;
constexpr size_t kImgHorner16Cols = kImgCombine16Cols + 2048;
//   [kImgPow2Cols, +1024)    shift by 2^b bytes, b = 0..31, NORMAL domain: word b*32 + c = column c
//                            (chained checksums: crc(s, A || B) = shift_|B|(crc(s, A)) ^ crc(0, B))
constexpr size_t kImgPow2Cols = kImgHorner16Cols + 32;
//   [kImgZero, +16)          zeros: the row loads of crc_stream_kernel read chunks wholly outside a
//                            fragment from here
constexpr size_t kImgZero = kImgPow2Cols + 1024;
//   [kImgLightNib, +11*144)  nibble tables (swapped domain, out[p*16 + v] of nibble_tables, 128 words
//                            each, 144 apart so that tables 4 + g, g = 0..3, start on banks 16g) of the
//                            table-light fused copy (crc_light_copy_kernel): table 0 shifts by 1024
//                            bytes (a lane's next chunk of the row), table 1 + j by 16 * 2^j bytes,
//                            j = 0..2 (the three levels of its lane tree), table 4 + g by 128 * (7 - g)
//                            bytes, g = 0..6 (the eight-lane groups to the row end)
constexpr size_t kImgLightNib = kImgZero + 16;
constexpr int kLightTables = 11;
constexpr int kLightTableWords = 144;
//   [kImgSliceBasis, +64)    slicing-table basis of table j at 16 j: words 0..4 S_j[1 << b], 5..12 S_j[32 k],
//                            13..15 zero (S_j is linear in its index; the table-light copy builds its
//                            tables from these instead of selecting compile-time constants per lane)
constexpr size_t kImgSliceBasis = kImgLightNib + kLightTables * kLightTableWords;
constexpr size_t kImgWords = kImgSliceBasis + 64;
constexpr int kChunkBytes = 16;                          // coalesced layout: 16-byte chunks
constexpr int kChunkStep = kRowBytes / 4 - kChunkBytes;  // 1008 zero bytes between a lane's chunks

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

// Slicing tables S_j[i], j = 0..3 (swapped domain): for X = C ^ w (w a little-endian
// 32-bit load), C' = S_0[X.b0] ^ S_1[X.b1] ^ S_2[X.b2] ^ S_3[X.b3].
void slice_tables(uint32_t S[4][256]);

// Device basis image, kImgWords words.
std::vector<uint32_t> build_table_image();

}  // namespace lampi
