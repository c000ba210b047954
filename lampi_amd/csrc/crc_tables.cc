// crc_tables.cc -- see crc_tables.h.
#include "crc_tables.h"

#include <cstdio>
#include <cstdlib>

#include "crc_const.h"

#include <cstring>
#include <mutex>

namespace lampi {

namespace {
uint32_t g_T[256];
std::once_flag g_T_once;

void build_T() {
    // entry i: byte i placed in bits 31..24, shifted through 8 polynomial steps
    // (semantics of ref ulm_initialize_crc_table, MemFunctions.cc:1242-1261)
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t r = i << 24;
        for (int k = 0; k < 8; ++k) r = (r & 0x80000000u) ? (r << 1) ^ kCrcPoly : (r << 1);
        g_T[i] = r;
    }
}

inline uint32_t zero_byte(uint32_t c) { return (c << 8) ^ g_T[c >> 24]; }
}  // namespace

const uint32_t *sarwate_table() {
    std::call_once(g_T_once, build_T);
    return g_T;
}

uint32_t crc_bytes(uint32_t crc, const uint8_t *p, size_t n) {
    const uint32_t *T = sarwate_table();
    for (size_t i = 0; i < n; ++i) crc = (crc << 8) ^ T[(crc >> 24) ^ p[i]];
    return crc;
}

Gf2Mat mat_identity() {
    Gf2Mat m;
    for (int b = 0; b < 32; ++b) m.col[b] = 1u << b;
    return m;
}

Gf2Mat mat_mul(const Gf2Mat &a, const Gf2Mat &b) {
    Gf2Mat r;
    for (int k = 0; k < 32; ++k) r.col[k] = a.apply(b.col[k]);
    return r;
}

Gf2Mat shift_matrix(uint64_t nbytes) {
    sarwate_table();
    Gf2Mat one;  // one zero byte
    for (int b = 0; b < 32; ++b) one.col[b] = zero_byte(1u << b);
    Gf2Mat acc = mat_identity(), sq = one;
    for (uint64_t n = nbytes; n; n >>= 1) {
        if (n & 1) acc = mat_mul(sq, acc);
        sq = mat_mul(sq, sq);
    }
    return acc;
}

Gf2Mat swapped(const Gf2Mat &m) {
    Gf2Mat r;
    for (int b = 0; b < 32; ++b) r.col[b] = bswap32(m.apply(bswap32(1u << b)));
    return r;
}

void nibble_tables(const Gf2Mat &ms, uint32_t out[128]) {
    for (int p = 0; p < 8; ++p)
        for (uint32_t v = 0; v < 16; ++v) out[p * 16 + v] = ms.apply(v << (4 * p));
}

void slice_tables(uint32_t S[4][256]) {
    const uint32_t *T = sarwate_table();
    uint32_t Tk[4][256];
    for (int i = 0; i < 256; ++i) {
        Tk[0][i] = T[i];
        for (int k = 1; k < 4; ++k) Tk[k][i] = zero_byte(Tk[k - 1][i]);
    }
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 256; ++i) S[j][i] = bswap32(Tk[3 - j][i]);
}

std::vector<uint32_t> build_table_image() {
    std::vector<uint32_t> img(kImgWords, 0);

    uint32_t S[4][256];
    slice_tables(S);
    for (int i = 0; i < 256; ++i)
        for (int j = 0; j < 4; ++j) img[kImgSliceT + 4 * i + j] = S[j][i];

    // per-lane final shift: lane l's last byte sits 64*(63-l) bytes before the row end
    const Gf2Mat step = shift_matrix(kLaneBytes);
    Gf2Mat m = mat_identity();  // shift by 64*(63-l), built from l = 63 downwards
    for (int l = kWave - 1; l >= 0; --l) {
        const Gf2Mat ms = swapped(m);
        for (int b = 0; b < 32; ++b) img[kImgCombineCols + l * 32 + b] = ms.col[b];
        m = mat_mul(step, m);
    }

    // Horner step between rows: the next 64-byte piece of a lane starts 4032 bytes later
    const Gf2Mat h = swapped(shift_matrix(kRowBytes - kLaneBytes));
    for (int b = 0; b < 32; ++b) img[kImgHornerCols + b] = h.col[b];

    // coalesced layout: lane l's last chunk ends 16*(63-l) bytes before the row end, and
    // consecutive chunks of a lane (also across rows) are 1008 bytes apart
    const Gf2Mat step16 = shift_matrix(kChunkBytes);
    m = mat_identity();
    for (int l = kWave - 1; l >= 0; --l) {
        const Gf2Mat ms = swapped(m);
        for (int b = 0; b < 32; ++b) img[kImgCombine16Cols + l * 32 + b] = ms.col[b];
        m = mat_mul(step16, m);
    }
    const Gf2Mat h16 = swapped(shift_matrix(kChunkStep));
    for (int b = 0; b < 32; ++b) img[kImgHorner16Cols + b] = h16.col[b];

    // the kernels build the slicing and Horner tables from compile-time constants (crc_const.h):
    // they must equal the run-time algebra here, bit for bit
    constexpr cx::SliceBasis sb = cx::slice_basis();
    constexpr cx::Mat ch = cx::swapped(cx::shift(kRowBytes - kLaneBytes));
    constexpr cx::Mat ch16 = cx::swapped(cx::shift(kChunkStep));
    bool same = true;
    for (int j = 0; j < 4; ++j) {
        for (int b = 0; b < 5; ++b) same &= sb.lo[j][b] == S[j][1u << b];
        for (int k = 0; k < 8; ++k) same &= sb.hi[j][k] == S[j][32 * k];
    }
    for (int b = 0; b < 32; ++b) same &= ch.c[b] == h.col[b] && ch16.c[b] == h16.col[b];
    if (!same) {
        fprintf(stderr, "lampi: compile-time CRC tables differ from the run-time ones\n");
        abort();
    }

    for (int j = 0; j < 4; ++j) {
        for (int b = 0; b < 5; ++b) img[kImgSliceBasis + 16 * j + b] = S[j][1u << b];
        for (int k = 0; k < 8; ++k) img[kImgSliceBasis + 16 * j + 5 + k] = S[j][32 * k];
    }

    // the table-light fused copy's shifts: 1024 bytes, 16 * 2^j bytes (j = 0..2), 128 * (7 - g) (g = 0..6)
    for (int t = 0; t < kLightTables; ++t) {
        const uint64_t nbytes = t == 0 ? 1024u : t < 4 ? (16ull << (t - 1)) : 128ull * (uint64_t)(7 - (t - 4));
        nibble_tables(swapped(shift_matrix(nbytes)), &img[kImgLightNib + kLightTableWords * (size_t)t]);
    }

    // powers of two for arbitrary shifts, normal domain (squaring from one byte)
    Gf2Mat pw = shift_matrix(1);
    for (int e = 0; e < 32; ++e) {
        for (int c = 0; c < 32; ++c) img[kImgPow2Cols + e * 32 + c] = pw.col[c];
        pw = mat_mul(pw, pw);
    }
    return img;
}

}  // namespace lampi
