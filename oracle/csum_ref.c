/*
 * oracle/csum_ref.c -- CPU restatement of LA-MPI's 32-bit fragment checksums.
 *
 * TEST INFRASTRUCTURE ONLY (see csum_ref.h).  Never linked into the product.
 * Parity: pinned against the compiled reference (oracle/_ref) through
 * tests/golden/ fixtures and against SURVEY.md 8(c) KATs / BASELINE.md digests.
 */
#include "csum_ref.h"

#include <string.h>
#include <time.h>
#include <stdlib.h>
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- CRC-32/MPEG-2 */

static uint32_t g_table[256];
static int g_table_ready = 0;

/* MSB-first table for polynomial 0x04C11DB7: entry i is the register after
 * shifting the byte i (placed in bits 31..24) through 8 polynomial steps.
 * Semantics of ref MemFunctions.cc:1242-1261.  Built once, before any thread
 * can race on it (the reference's lazy init at :1271-1273 is racy). */
static void build_table(void)
{
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t r = i << 24;
        for (int b = 0; b < 8; ++b)
            r = (r & 0x80000000u) ? ((r << 1) ^ ORACLE_CRC_POLY) : (r << 1);
        g_table[i] = r;
    }
    g_table_ready = 1;
}

__attribute__((constructor)) static void oracle_init(void) { build_table(); }

const uint32_t *oracle_crc_table(void)
{
    if (!g_table_ready) build_table();
    return g_table;
}

/* One table step per byte, stream order, no reflection, no final XOR:
 * crc = (crc << 8) ^ T[(crc >> 24) ^ byte]   (ref MemFunctions.cc:1343-1364). */
uint32_t oracle_uicrc(const void *src, size_t len, uint32_t partial)
{
    const uint8_t *p = (const uint8_t *)src;
    uint32_t crc = partial;
    for (size_t i = 0; i < len; ++i)
        crc = (crc << 8) ^ g_table[((crc >> 24) ^ p[i]) & 0xFFu];
    return crc;
}

/* Copies copylen bytes; the CRC runs over max(copylen, crclen) bytes of src --
 * bytes past copylen are read but not copied (ref MemFunctions.cc:1266,
 * :1299-1303, :1314-1317; receive side uses it, src/path/gm/recvFrag.h:174). */
uint32_t oracle_bcopy_uicrc(const void *src, void *dst, size_t copylen, size_t crclen,
                            uint32_t partial)
{
    const uint8_t *s = (const uint8_t *)src;
    uint8_t *d = (uint8_t *)dst;
    uint32_t crc = partial;
    size_t n = copylen > crclen ? copylen : crclen;
    for (size_t i = 0; i < copylen; ++i) {
        uint8_t b = s[i];
        d[i] = b;
        crc = (crc << 8) ^ g_table[((crc >> 24) ^ b) & 0xFFu];
    }
    for (size_t i = copylen; i < n; ++i)
        crc = (crc << 8) ^ g_table[((crc >> 24) ^ s[i]) & 0xFFu];
    return crc;
}

/* ---------------------------------------------------------------- 32-bit additive sum */

static inline uint32_t load_le32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* Sum mod 2^32 of little-endian 32-bit words of the chained byte stream.
 * State (*pint, *plen): *plen bytes (1..3) of the current word have been seen and
 * *pint is that word's value; each call returns the increment to the running sum
 * (callers accumulate with +=, src/path/gm/sendFrag.cc:202-204).  A trailing partial
 * word counts with its missing high bytes as zero.  *plen == 0 (or 4) means word
 * aligned and *pint is ignored.  Semantics of ref MemFunctions.cc:1073-1222. */
uint32_t oracle_uicsum(const void *src, size_t len, uint32_t *pint, uint32_t *plen)
{
    const uint8_t *p = (const uint8_t *)src;
    uint32_t sum = 0;
    uint32_t k = *plen;
    if (k >= 4) k = 0;
    if (k) {
        uint32_t old = *pint, w = old;
        size_t take = 4 - k;
        if (take > len) take = len;
        for (size_t j = 0; j < take; ++j) {
            uint32_t sh = 8u * (uint32_t)(k + j);
            w = (w & ~(0xFFu << sh)) | ((uint32_t)p[j] << sh);
        }
        sum += w - old;
        p += take;
        len -= take;
        if (k + take < 4) {          /* word still incomplete: carry it */
            *pint = w;
            *plen = k + (uint32_t)take;
            return sum;
        }
    }
    size_t nw = len / 4;
    for (size_t i = 0; i < nw; ++i) sum += load_le32(p + 4 * i);
    p += 4 * nw;
    size_t r = len & 3u;
    uint32_t tail = 0;
    for (size_t j = 0; j < r; ++j) tail |= (uint32_t)p[j] << (8 * j);
    sum += tail;
    *pint = tail;
    *plen = (uint32_t)r;
    return sum;
}

/* Copy copylen bytes; sum max(copylen, csumlen) bytes of src with the same chaining
 * state (ref MemFunctions.cc:518-875, residue handling :821-872). */
uint32_t oracle_bcopy_uicsum(const void *src, void *dst, size_t copylen, size_t csumlen,
                             uint32_t *pint, uint32_t *plen)
{
    if (copylen) memcpy(dst, src, copylen);
    return oracle_uicsum(src, copylen > csumlen ? copylen : csumlen, pint, plen);
}

/* csum (ref MemFunctions.cc:913-1071): the same chaining with 64-bit little-endian words
 * (unsigned long on LP64), sum mod 2^64; lastPartialLength in 0..7 (8+ treated as 0). */
uint64_t oracle_csum64(const void *src, size_t len, uint64_t *plong, uint64_t *plen)
{
    const uint8_t *p = (const uint8_t *)src;
    uint64_t sum = 0;
    uint64_t k = *plen;
    if (k >= 8) k = 0;
    if (k) {
        uint64_t old = *plong, w = old;
        size_t take = 8 - (size_t)k;
        if (take > len) take = len;
        for (size_t j = 0; j < take; ++j) {
            unsigned sh = 8u * (unsigned)(k + j);
            w = (w & ~(0xFFull << sh)) | ((uint64_t)p[j] << sh);
        }
        sum += w - old;
        p += take;
        len -= take;
        if (k + take < 8) {
            *plong = w;
            *plen = k + take;
            return sum;
        }
    }
    size_t nw = len / 8;
    for (size_t i = 0; i < nw; ++i) {
        uint64_t w = 0;
        for (int j = 0; j < 8; ++j) w |= (uint64_t)p[8 * i + (size_t)j] << (8 * j);
        sum += w;
    }
    p += 8 * nw;
    size_t r = len & 7u;
    uint64_t tail = 0;
    for (size_t j = 0; j < r; ++j) tail |= (uint64_t)p[j] << (8 * j);
    sum += tail;
    *plong = tail;
    *plen = r;
    return sum;
}

/* bcopy_csum (ref MemFunctions.cc:142-516): copy copylen bytes, csum max(copylen, csumlen). */
uint64_t oracle_bcopy_csum64(const void *src, void *dst, size_t copylen, size_t csumlen, uint64_t *plong,
                             uint64_t *plen)
{
    if (copylen) memcpy(dst, src, copylen);
    return oracle_csum64(src, copylen > csumlen ? copylen : csumlen, plong, plen);
}

uint32_t oracle_header_checksum(const void *header, size_t crclen, int word_count, int usecrc)
{
    if (usecrc) {
        uint32_t c = oracle_uicrc(header, crclen, ORACLE_CRC_INIT);
        /* stored byte-swapped on little-endian so CRC(header || stored) == 0 */
        return (c >> 24) | ((c >> 8) & 0xFF00u) | ((c << 8) & 0xFF0000u) | (c << 24);
    }
    uint32_t s = 0;
    const uint8_t *p = (const uint8_t *)header;
    for (int i = 0; i < word_count; ++i) s += load_le32(p + 4 * (size_t)i);
    return s;
}

/* ---------------------------------------------------------------- synthetic payloads */

static inline uint64_t mix64(uint64_t z)
{
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}

void oracle_fill_stream(uint8_t *dst, uint64_t seed, uint64_t byte_off, size_t n)
{
    size_t i = 0;
    while (i < n) {
        uint64_t pos = byte_off + i;
        uint64_t w = mix64(seed + (pos / 8 + 1) * 0x9E3779B97F4A7C15ull);
        unsigned b = (unsigned)(pos & 7u);
        if (b == 0 && n - i >= 8) {
            memcpy(dst + i, &w, 8);   /* host is little-endian (x86-64) */
            i += 8;
        } else {
            dst[i++] = (uint8_t)(w >> (8 * b));
        }
    }
}

static int resolve_threads(int nthreads)
{
#ifdef _OPENMP
    return nthreads > 0 ? nthreads : omp_get_max_threads();
#else
    (void)nthreads;
    return 1;
#endif
}

static uint32_t frag_value(const uint8_t *p, size_t L, int mode)
{
    if (mode == 0) return oracle_uicrc(p, L, ORACLE_CRC_INIT);
    uint32_t a = 0, b = 0;
    return oracle_uicsum(p, L, &a, &b);
}

void oracle_uniform_batch(uint64_t seed, uint64_t k0, size_t n, size_t L, int mode,
                          int nthreads, uint32_t *out)
{
    int nt = resolve_threads(nthreads);
#pragma omp parallel num_threads(nt)
    {
        uint8_t *buf = (uint8_t *)malloc(L ? L : 1);
#pragma omp for schedule(static)
        for (long long i = 0; i < (long long)n; ++i) {
            uint64_t k = k0 + (uint64_t)i;
            oracle_fill_stream(buf, seed, k * (uint64_t)L, L);
            out[i] = frag_value(buf, L, mode);
        }
        free(buf);
    }
}

void oracle_uniform_digest(uint64_t seed, size_t n, size_t L, int mode, int nshard, int shard,
                           int nthreads, uint32_t dig[2])
{
    int nt = resolve_threads(nthreads);
    uint32_t gx = 0, gs = 0;
#pragma omp parallel num_threads(nt)
    {
        uint8_t *buf = (uint8_t *)malloc(L ? L : 1);
        uint32_t x = 0, s = 0;
#pragma omp for schedule(static)
        for (long long k = shard; k < (long long)n; k += nshard) {
            oracle_fill_stream(buf, seed, (uint64_t)k * (uint64_t)L, L);
            uint32_t c = frag_value(buf, L, mode);
            x ^= c;
            s += c * (uint32_t)(2 * (uint64_t)k + 1);
        }
#pragma omp critical
        {
            gx ^= x;
            gs += s;
        }
        free(buf);
    }
    dig[0] = gx;
    dig[1] = gs;
}

void oracle_desc_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                       const uint32_t *partial, size_t n, int mode, int nthreads, uint32_t *out)
{
    int nt = resolve_threads(nthreads);
#pragma omp parallel for num_threads(nt) schedule(dynamic, 64)
    for (long long i = 0; i < (long long)n; ++i) {
        if (mode == 0) {
            out[i] = oracle_uicrc(base + off[i], len[i], partial ? partial[i] : ORACLE_CRC_INIT);
        } else {
            uint32_t a = 0, b = 0;
            out[i] = oracle_uicsum(base + off[i], len[i], &a, &b);
        }
    }
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

double oracle_time_uniform(uint64_t seed, size_t n, size_t L, int mode, int nthreads,
                           uint32_t *xor_out)
{
    int nt = resolve_threads(nthreads);
    size_t total = n * L;
    uint8_t *buf = (uint8_t *)malloc(total ? total : 1);
    oracle_fill_stream(buf, seed, 0, total);
    uint32_t x = 0;
    double t0 = now_s();
#pragma omp parallel for num_threads(nt) schedule(static) reduction(^ : x)
    for (long long k = 0; k < (long long)n; ++k) x ^= frag_value(buf + (size_t)k * L, L, mode);
    double t1 = now_s();
    free(buf);
    if (xor_out) *xor_out = x;
    return t1 - t0;
}

/* Time `fn` (a uicrc-shaped function: the restatement's oracle_uicrc or the reference's
 * uicrc(const void*, unsigned long, unsigned int)) over n fragments of L bytes in buf,
 * nthreads threads, init register 0xFFFFFFFF.  Returns seconds; XOR of results in *xor_out;
 * the per-fragment values in out[0..n) when out is not NULL (the caller's parity check). */
typedef uint32_t (*oracle_crc_fn)(const void *, unsigned long, unsigned int);

double oracle_time_fn(void *fn, const uint8_t *buf, size_t n, size_t L, int nthreads, uint32_t *xor_out,
                      uint32_t *out)
{
    oracle_crc_fn f = (oracle_crc_fn)fn;
    int nt = resolve_threads(nthreads);
    uint32_t x = 0;
    double t0 = now_s();
#pragma omp parallel for num_threads(nt) schedule(static) reduction(^ : x)
    for (long long k = 0; k < (long long)n; ++k) {
        uint32_t c = f(buf + (size_t)k * L, (unsigned long)L, ORACLE_CRC_INIT);
        if (out) out[k] = c;
        x ^= c;
    }
    double t1 = now_s();
    if (xor_out) *xor_out = x;
    return t1 - t0;
}

/* ---- config C: mixed fragment sizes ---------------------------------------
 * Length of fragment k = 64*r bytes, r in [1, 1024] drawn Zipf(s = 1.1) by inverse CDF from
 * the counter-based uniform u_k = (mix(0x5A1F + k) >> 11) * 2^-53.  Fragments are packed
 * back to back (64-byte aligned, since every length is a multiple of 64) until the total
 * reaches min_total bytes.  Returns the number of fragments; writes up to cap lengths. */
size_t oracle_zipf_lengths(uint64_t min_total, size_t cap, uint32_t *len_out)
{
    static double cdf[1025];
    static int ready = 0;
    if (!ready) {
        double z = 0.0;
        for (int r = 1; r <= 1024; ++r) z += pow((double)r, -1.1);
        double acc = 0.0;
        cdf[0] = 0.0;
        for (int r = 1; r <= 1024; ++r) {
            acc += pow((double)r, -1.1) / z;
            cdf[r] = acc;
        }
        cdf[1024] = 1.0;
        ready = 1;
    }
    uint64_t total = 0;
    size_t k = 0;
    while (total < min_total) {
        double u = (double)(mix64(0x5A1Full + k) >> 11) * (1.0 / 9007199254740992.0);
        int lo = 1, hi = 1024;  /* smallest r with cdf[r] > u */
        while (lo < hi) {
            int mid = (lo + hi) / 2;
            if (cdf[mid] > u) hi = mid; else lo = mid + 1;
        }
        uint32_t L = 64u * (uint32_t)lo;
        if (k < cap && len_out) len_out[k] = L;
        total += L;
        ++k;
    }
    return k;
}
