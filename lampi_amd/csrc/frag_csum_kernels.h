// frag_csum_kernels.h -- launchers for the gfx950 kernels in frag_csum.hip (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

#include "../../include/lampi_csum.h"

namespace lampi {

// Uniform message fragments of whole 4 KiB rows take the regular kernels (read-only checksums),
// except where the piece streams measured faster (tools/microbench/bigfrag_scan.py,
// profiles/r02_bigfrag_ab.txt, 1 and 16 GiB batches, A/B on one box): 64 KiB fragments in CRC
// (regular 61-71% of the HBM roofline -- its concurrent chains sit 64 KiB apart; 48, 96, 128,
// 256 KiB and 1 MiB run at 77-79% -- against 67-76%) and 33-64 KiB fragments in SUM (68-76%
// against 74-78%; from 128 KiB on the two are within a point).
inline bool regular_msg_frag(size_t frag_len, bool sum) {
    return sum ? (frag_len <= (32u << 10) || frag_len > (64u << 10)) : frag_len != (64u << 10);
}

// CRC messages whose fragments run on the read-only table-light kernel (launch_crc_msg): 8-16 rows,
// or longer in messages of at most 2 GiB (row groups; the regular kernel keeps the larger ones)
inline bool crc_light_msg(size_t frag_len, size_t msg_len) {
    (void)msg_len;  // (up to round 4: > 16 rows only in messages up to 2 GiB; profiles/r05/crc_light_msg_ab.txt)
    const size_t rows = (frag_len + 4095) / 4096;
    return rows >= 8 && rows < ((size_t)1 << 32);
}

// Workgroups for the persistent CRC kernel on `device` (one 1024-thread WG per CU).
int crc_grid(int device);

// Descriptor batches; plan (LAMPI_CSUM_BY_BYTES): byte-balanced for n <= 32768, a plan kernel first;
// otherwise the one-launch count split.
// rows_hint (LAMPI_CSUM_ROWS_HINT): row segments per fragment (RowSegSource), 1 = none
hipError_t diag_stream_timeline(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img,
                                uint64_t *stamps, hipStream_t s, uint32_t *nwg);
hipError_t diag_regular_timeline(const uint8_t *base, size_t n, uint32_t *out, const uint32_t *img, uint64_t *stamps,
                                 hipStream_t s, uint32_t *nwg);
hipError_t launch_crc_desc(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img, int grid,
                           hipStream_t s, bool plan = false, uint32_t rows_hint = 1);
// One wavefront per fragment (crc_rows_kernel / sum_rows_kernel), mode = lampi_csum_mode.
hipError_t launch_desc_per_wave(const lampi_frag_desc *d, size_t n, uint32_t *out, int mode, const uint32_t *img,
                                hipStream_t s);
hipError_t launch_crc_msg(const uint8_t *base, size_t msg_len, size_t frag_len, uint32_t partial, size_t n,
                          uint32_t *out, const uint32_t *img, int grid, hipStream_t s);
// Regular batch: frag_len % 4096 == 0, base 16-byte aligned, n full fragments.
hipError_t launch_crc_regular(const uint8_t *base, size_t n, size_t frag_len, uint32_t partial, uint32_t *out,
                              const uint32_t *img, int grid, hipStream_t s);
// Fused copy + checksum (bcopy_uicrc / bcopy_uicsum per descriptor), mode = lampi_csum_mode (NONE: copies only,
// out = n words of scratch).
// rows_hint (LAMPI_CSUM_ROWS_HINT): row groups per fragment, 1 = one wave (SUM: workgroup) walks every row
hipError_t launch_bcopy_desc(const lampi_copy_desc *d, size_t n, uint32_t *out, int mode, const uint32_t *img,
                             hipStream_t s, uint32_t rows_hint = 1);
// Fused copy of regular batches: fragment f -> dst + f*dst_stride (dst, dst_stride 4-byte aligned).
hipError_t launch_crc_regular_copy(const uint8_t *base, size_t n, size_t frag_len, uint32_t partial, uint8_t *dst,
                                   size_t dst_stride, uint32_t *out, const uint32_t *img, hipStream_t s);
// Fragments of a message, each copied to dst + k*dst_stride with its checksum fused.
hipError_t launch_msg_bcopy(const uint8_t *base, size_t msg_len, size_t frag_len, uint32_t partial, uint8_t *dst,
                            size_t dst_stride, size_t n, uint32_t *out, int mode, const uint32_t *img, hipStream_t s);
// RecvDesc_t::CopyToApp per descriptor (copy min(length, app_len), checksum length, verify).
hipError_t launch_copy_to_app(const lampi_recv_desc *d, size_t n, const uint8_t *expected, size_t exp_stride,
                              int64_t *copied, uint32_t *csum, uint32_t *mask, uint32_t *nbad, int mode,
                              const uint32_t *img, hipStream_t s, uint32_t rows_hint = 1);
// headerChecksum per header / receiver header check / CheckData (mask bit set = corrupt).
hipError_t launch_header_csum(const uint8_t *hdrs, size_t n, size_t stride, uint32_t crclen, uint32_t word_count,
                              int mode, const uint32_t *img, uint8_t *out, size_t out_stride, hipStream_t s);
hipError_t launch_header_check(const uint8_t *hdrs, size_t n, size_t stride, uint32_t hdr_bytes, uint32_t word_count,
                               uint32_t csum_offset, int mode, const uint32_t *img, uint32_t *mask, uint32_t *nbad,
                               hipStream_t s);
hipError_t launch_header_compare(const uint8_t *hdrs, size_t n, size_t stride, uint32_t crclen, uint32_t csum_offset,
                                 int mode, const uint32_t *img, uint32_t *mask, uint32_t *nbad, hipStream_t s);
hipError_t launch_check_data(const uint32_t *calc, const uint8_t *expected, size_t exp_stride, const uint8_t *lengths,
                             size_t len_stride, size_t n, uint32_t *mask, uint32_t *nbad, hipStream_t s);
// dst + i*stride = vals[i] (4-byte aligned records).
hipError_t launch_scatter_u32(const uint32_t *vals, size_t n, uint8_t *dst, size_t stride, hipStream_t s);
// The verdict of a chain batch delivered as CopyToApp's non-contiguous branch (launch_chain, chain_fold_kernel):
// copied == nullptr -- checksums only; otherwise copied[f] / mask / *nbad as lampi_copy_to_app_batch against the
// 32-bit value at expected + f * exp_stride; init: CRC from CRC_INITIAL_REGISTER, not the first piece's partial.
struct ChainVerdict {
    const uint8_t *expected = nullptr;
    size_t exp_stride = 0;
    int64_t *copied = nullptr;
    uint32_t *mask = nullptr;
    uint32_t *nbad = nullptr;
    uint32_t init = 0, nocheck = 0;
};
// Chained checksums over typemap pieces; vals / phase: npieces words of scratch each.  mode may be
// LAMPI_CSUM_NONE (copies only, checksums 0).
hipError_t launch_chain(const lampi_copy_desc *d, size_t npieces, const uint32_t *first, size_t nfrags, uint32_t *out,
                        int mode, const uint32_t *img, uint32_t *vals, uint32_t *phase, hipStream_t s,
                        const ChainVerdict *verdict = nullptr);
// 64-bit csum: per-descriptor sums (phased: desc.partial = byte phase 0..7) and the chained finish.
hipError_t launch_sum64_desc(const lampi_frag_desc *d, size_t n, uint64_t *out, bool phased, hipStream_t s);
// The host path's last kernels (combine / finish / a single piece) store their result, then, when
// sig is given, seq into *sig at system scope: the host polls it (lampi_csum.cc wait_done).
hipError_t launch_sum64_finish(const uint64_t *vals, uint32_t nv, const uint8_t *src, uint64_t len, uint64_t plong,
                               uint64_t plen, uint64_t *out3, hipStream_t s, uint64_t *sig = nullptr,
                               uint64_t seq = 0);
// SUM per descriptor / per fragment of a message: piece streams when img (the table image, for its
// zero chunk) is given, one wavefront per fragment (sum_rows_kernel) otherwise.
hipError_t launch_sum_desc(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img, int grid,
                           hipStream_t s, bool plan = false, uint32_t rows_hint = 1);
hipError_t launch_sum_msg(const uint8_t *base, size_t msg_len, size_t frag_len, size_t n, uint32_t *out,
                          const uint32_t *img, int grid, hipStream_t s);
hipError_t launch_crc_combine(const uint32_t *vals, uint32_t n, const uint32_t *tabs, uint32_t npow,
                              uint32_t *out, hipStream_t s, uint64_t *sig = nullptr, uint64_t seq = 0);
hipError_t launch_sum_finish(const uint32_t *partials, uint32_t npart, const uint8_t *src, uint64_t len,
                             uint32_t pint, uint32_t plen, uint32_t *out3, hipStream_t s, uint64_t *sig = nullptr,
                             uint64_t seq = 0);
hipError_t launch_host_one(const uint8_t *addr, uint32_t len, uint32_t partial, uint32_t *out, int mode,
                           const uint32_t *img, hipStream_t s, uint64_t *sig, uint64_t seq);
hipError_t launch_fill_frags(uint64_t *dst, size_t n, uint64_t frag_words, uint64_t seed, uint64_t k0,
                             uint64_t kstep, int grid, hipStream_t s);
hipError_t launch_fill_stream(uint8_t *dst, size_t nbytes, uint64_t seed, uint64_t byte_off, int grid,
                              hipStream_t s);

// The calling thread's device scratch (stream_scratch, frag_csum.hip): free its buffer for stream s
// (before s is destroyed) or all of its buffers (lampi_host_release); bytes held over all threads.
void release_stream_scratch(hipStream_t s);
void release_thread_scratch();
int64_t device_scratch_bytes();

}  // namespace lampi
