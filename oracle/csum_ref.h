/*
 * oracle/csum_ref.h -- CPU restatement of LA-MPI's fragment-checksum routines.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product library (lampi_amd/csrc,
 * liblampi_csum.so) links, loads or calls this code.  It is imported only by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
 * checker and as the reported CPU baseline.
 *
 * Parity status: PINNED.  Every function here is checked bit-for-bit against
 *   (a) the reference itself: /root/reference/src/util/MemFunctions.cc compiled
 *       unmodified by oracle/Makefile into oracle/_ref/libref_memfunctions.so,
 *       via the committed fixtures in tests/golden/ (tests/golden/make_golden.py);
 *   (b) the known-answer values of SURVEY.md section 8(c) and the BASELINE.md digests.
 *
 * Clean-room: written from the semantics in SURVEY.md section 0/8, not from the
 * reference source.  The CRC is the same byte-serial table loop the reference
 * runs (one table step per byte), so timing it is a fair CPU baseline.
 */
#ifndef LAMPI_ORACLE_CSUM_REF_H
#define LAMPI_ORACLE_CSUM_REF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_CRC_POLY 0x04C11DB7u   /* src/util/MemFunctions.h:36 */
#define ORACLE_CRC_INIT 0xFFFFFFFFu   /* src/util/MemFunctions.h:37 */

/* 256-entry MSB-first table (ref: ulm_initialize_crc_table, MemFunctions.cc:1242-1261). */
const uint32_t *oracle_crc_table(void);

/* uicrc(src, len, partial)  (ref: MemFunctions.cc:1331-1367; wrapper :1371-1374). */
uint32_t oracle_uicrc(const void *src, size_t len, uint32_t partial);

/* bcopy_uicrc: copy copylen bytes, CRC max(copylen, crclen) bytes of src
 * (ref: MemFunctions.cc:1263-1321; wrapper :1325-1329). */
uint32_t oracle_bcopy_uicrc(const void *src, void *dst, size_t copylen, size_t crclen,
                            uint32_t partial);

/* uicsum with (lastPartialInt, lastPartialLength) chaining state
 * (ref: MemFunctions.cc:1073-1222; wrapper :1226-1231). */
uint32_t oracle_uicsum(const void *src, size_t len, uint32_t *pint, uint32_t *plen);

/* bcopy_uicsum: copy copylen bytes, sum max(copylen, csumlen) bytes of src
 * (ref: MemFunctions.cc:518-875; wrapper :882-893). */
uint64_t oracle_csum64(const void *src, size_t len, uint64_t *plong, uint64_t *plen);
uint64_t oracle_bcopy_csum64(const void *src, void *dst, size_t copylen, size_t csumlen, uint64_t *plong,
                             uint64_t *plen);
uint32_t oracle_bcopy_uicsum(const void *src, void *dst, size_t copylen, size_t csumlen,
                             uint32_t *pint, uint32_t *plen);

/* BasePath_t::headerChecksum (ref: src/path/common/path.h:280-314).
 * usecrc != 0: byte-swapped uicrc(header, crclen); else sum of word_count LE u32. */
uint32_t oracle_header_checksum(const void *header, size_t crclen, int word_count, int usecrc);

/* ---- synthetic payloads ---------------------------------------
 * word64[i] of stream `seed` = mix(seed + (i+1)*0x9E3779B97F4A7C15), little-endian,
 * mix = splitmix64 finalizer.  Writes stream bytes [byte_off, byte_off + n). */
void oracle_fill_stream(uint8_t *dst, uint64_t seed, uint64_t byte_off, size_t n);

/* Per-fragment checksums of a uniform batch: fragment k = stream bytes [k*L, (k+1)*L).
 * mode 0 = CRC (uicrc, init 0xFFFFFFFF), 1 = SUM (uicsum, fresh state).
 * Fragments [k0, k0 + n) are written to out[0..n).  nthreads <= 0: all cores. */
void oracle_uniform_batch(uint64_t seed, uint64_t k0, size_t n, size_t L, int mode,
                          int nthreads, uint32_t *out);

/* Digests over fragments k in [0, n) with k % nshard == shard:
 *   dig[0] = XOR of c_k, dig[1] = sum of c_k * (2k+1) mod 2^32. */
void oracle_uniform_digest(uint64_t seed, size_t n, size_t L, int mode, int nshard, int shard,
                           int nthreads, uint32_t dig[2]);

/* Descriptor batch over a host copy of device memory: c_i = checksum of
 * base[off[i] .. off[i]+len[i]) with CRC partial[i] (mode 0) or fresh SUM state (mode 1). */
void oracle_desc_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                       const uint32_t *partial, size_t n, int mode, int nthreads, uint32_t *out);

/* Time the CPU baseline: checksum n fragments of L bytes of stream `seed` (payload generated
 * up front, untimed) with nthreads threads; returns seconds of the checksum loop only. */
double oracle_time_uniform(uint64_t seed, size_t n, size_t L, int mode, int nthreads,
                           uint32_t *xor_out);

/* Config C: Zipf(1.1) lengths 64*r, r in [1,1024], from u_k = mix(0x5A1F+k)>>11,
 * packed until the total reaches min_total.  Returns the count; writes up to cap lengths. */
size_t oracle_zipf_lengths(uint64_t min_total, size_t cap, uint32_t *len_out);

/* Time a uicrc-shaped function pointer over n fragments of L bytes of buf (see .c). */
double oracle_time_fn(void *fn, const uint8_t *buf, size_t n, size_t L, int nthreads, uint32_t *xor_out,
                      uint32_t *out);

#ifdef __cplusplus
}
#endif
#endif
