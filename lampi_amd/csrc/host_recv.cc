// host_recv.cc -- the receive half of the host-memory path of liblampi_csum.so
// (lampi_host_copy_to_app_batch, lampi_host_header_check_batch, lampi_host_header_compare_batch;
// include/lampi_csum.h).
//
// LA-MPI's receive loop drains every pending NIC event in one call (gmPath::receive, ref
// src/path/gm/path.cc:286-313; IB src/path/ib/path.cc:630-741).  Per fragment it checks the header
// (gm/path.cc:364-393; IB recompute-and-compare, ib/path.cc:652-680), matches it to a posted
// receive and delivers the payload: RecvDesc_t::CopyToApp (src/path/common/BaseDesc.cc:288-342)
// copies min(length_m, AppBufferLen) bytes into the application buffer with the checksum of all
// length_m bytes fused (CopyFunction, gm/recvFrag.h:165-182: bcopy_uicrc / bcopy_uicsum with
// copylen < csumlen; IB recvFrag.cc:182-200) and compares it with the header's dataChecksum
// (CheckData, gm/recvFrag.h:213-257; IB recvFrag.cc:229-245).
//
// Here the caller hands over the whole batch of drained fragments at once: payloads anywhere in a
// host NIC ring (page-locked or pageable), the application bytes go to host addresses.  The
// per-thread pipeline of host_msg.cc carries it:
//
//   s_in : H2D of chunk i -- the ring bytes under its fragments, coalesced into as few DMA
//          transfers as the layout allows: a dense run of fragments (gaps <= 1/16 of the payload,
//          e.g. GM's payloads 80 bytes apart, IB's 112) is one 1D copy, fragments at a constant
//          slot pitch with wide gaps (4 KiB payloads in 64 KiB slots) one 2D copy, anything else
//          one copy each
//   s_k  : the fused CopyToApp kernel over the chunk (launch_copy_to_app, the device path's own
//          kernel; the row-group count comes from the fragments' mean length, which the host knows)
//          into per-fragment results, the delivered bytes packed into an output chunk so that every
//          run of fragments contiguous in the application buffer goes back in one D2H
//   s_out: D2H of those runs straight into the application buffers
//
// Results come back in one D2H at the end.  No payload byte is touched by the CPU; it reads only the
// descriptors the caller built.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <vector>

#include "../../include/lampi_csum.h"
#include "crc_tables.h"
#include "frag_csum_kernels.h"
#include "host_internal.h"
#include "host_pipe.h"
#include "host_plan.h"

namespace lampi {
namespace {

#define TRY LAMPI_TRY

uint32_t to_copy(const lampi_host_recv_frag &x) {
    return x.app_len <= 0 ? 0u : (x.app_len < (int64_t)x.length ? (uint32_t)x.app_len : x.length);
}

// The batch as the planner sees it: fragment j reads its `length` ring bytes (all checksummed) and
// writes lengthToCopy of them to its application address -- or nothing at all when lengthToCopy is 0.
// (checksumming off, LAMPI_CSUM_NONE: only the lengthToCopy bytes are read)
struct RecvItems {
    const lampi_host_recv_frag *f;
    size_t n;
    bool copy_only;
    size_t size() const { return n; }
    PlanItem get(size_t j) const {
        const uint32_t c = to_copy(f[j]);
        if (!c) return PlanItem{0, 0, nullptr, 0};
        return PlanItem{f[j].frag_off, copy_only ? c : f[j].length, (uint8_t *)f[j].app, c};
    }
    bool boundary(size_t) const { return true; }
};

// Rows per fragment for the row-group schedule of the chunk's copy kernel: the fragments' mean
// length in 4 KiB rows (GM's 65,456-byte payloads: 16 -> 69-70% of read + write against 59%
// walking the rows in one wave); 1 for fragments of about a row or less.
uint32_t chunk_rows_hint(const ChunkPlan &c) {
    if (c.nread == 0) return 1;
    const uint64_t mean = c.payload / c.nread;
    const uint64_t rows = (mean + kRowBytes - 1) / kRowBytes;
    return rows >= 2 ? (uint32_t)std::min<uint64_t>(rows, 0xFFF) : 1u;
}

// Per-thread planning scratch, kept between calls (no allocation per call once grown).
struct RecvScratch {
    std::vector<size_t> din, dout;
    std::vector<InXfer> in;
    std::vector<OutXfer> out;
};
thread_local RecvScratch t_recv;

hipError_t host_recv(const uint8_t *h_ring, size_t ring_bytes, const lampi_host_recv_frag *f, size_t n,
                     int64_t *h_copied, uint32_t *h_csum, uint32_t *h_mask, uint32_t *h_nbad, int mode,
                     uint32_t hint_override) {
    RecvScratch &rs = t_recv;
    if (rs.din.size() < n) {
        rs.din.resize(n);
        rs.dout.resize(n);
    }
    const RecvItems items{f, n, mode == LAMPI_CSUM_NONE};
    PlanRules rules;
    rules.ring = true;
    rules.ring_bytes = ring_bytes;
    StreamPlanner<RecvItems> pl(items, rules, chunk_target(true), rs.din.data(), rs.dout.data());
    PipeState *pp = nullptr;
    TRY(pipe_ctx(&pp));
    PipeState &p = *pp;
    const uint32_t *img = nullptr;
    TRY(device_tables(p.dev, &img));
    TRY(ensure_chunks(p, std::max<size_t>(pl.in_need(), 256)));
    TRY(ensure_out_chunks(p, std::max<size_t>(pl.out_need(), 256)));

    // the call's descriptors (each chunk's go up with it; the expected checksum rides in the
    // descriptor's reserved word, where the kernel reads it with a 32-byte stride) and results (one D2H
    // at the end); the kernel's own mask and count land in a scratch the host never reads: the verdict
    // is copied[i] == -1
    const size_t o_copied = align_up(n * sizeof(lampi_recv_desc), 256);
    const size_t o_csum = align_up(o_copied + n * sizeof(int64_t), 256);
    const size_t o_scratch = align_up(o_csum + n * sizeof(uint32_t), 256);
    const size_t total = o_scratch + ((n + 31) / 32 + 2) * sizeof(uint32_t);
    TRY(ensure_meta(p, total));
    lampi_recv_desc *hd = (lampi_recv_desc *)p.hmeta;
    uint8_t *dm = p.dmeta;
    uint32_t *dmask = (uint32_t *)(dm + o_scratch), *dnbad = dmask + (n + 31) / 32 + 1;

    PipeDrain drain(p);  // any early return below leaves nothing in flight
    ChunkPlan k;
    for (size_t c = 0; pl.next(k, rs.in, rs.out); ++c) {
        const int b = (int)(c % kBufs);
        uint8_t *din = p.dchunk + (size_t)b * p.chunk_bytes;
        uint8_t *dout = p.dout + (size_t)b * p.out_bytes;
        const size_t f0 = k.j0, f1 = k.j1;
        for (size_t j = f0; j < f1; ++j) {
            const bool moves = to_copy(f[j]) != 0;  // others read and write nothing: any valid address
            hd[j] = lampi_recv_desc{(uint64_t)(uintptr_t)(moves ? din + rs.din[j] : din),
                                    (uint64_t)(uintptr_t)(moves ? dout + rs.dout[j] : dout), f[j].app_len,
                                    f[j].length, f[j].expected};
        }
        // chunk b's buffers are free once chunk c - kBufs was copied to the app and sent back
        if (c >= (size_t)kBufs) {
            TRY(hipStreamWaitEvent(p.s_in, p.k_done[b], 0));
            TRY(hipStreamWaitEvent(p.s_in, p.out_done[b], 0));
        }
        if (f1 > f0)
            TRY(hipMemcpyAsync(dm + f0 * sizeof(lampi_recv_desc), hd + f0, (f1 - f0) * sizeof(lampi_recv_desc),
                               hipMemcpyHostToDevice, p.s_in));
        TRY(issue_in(rs.in, h_ring, din, p.s_in));
        TRY(hipEventRecord(p.in_done[b], p.s_in));
        TRY(hipStreamWaitEvent(p.s_k, p.in_done[b], 0));
        const uint32_t hint = hint_override ? hint_override : chunk_rows_hint(k);
        const lampi_recv_desc *dd = (const lampi_recv_desc *)dm + f0;
        TRY(launch_copy_to_app(dd, f1 - f0, (const uint8_t *)dd + offsetof(lampi_recv_desc, reserved),
                               sizeof(lampi_recv_desc), (int64_t *)(dm + o_copied) + f0,
                               (uint32_t *)(dm + o_csum) + f0, dmask, dnbad, mode, img, p.s_k, hint));
        TRY(hipEventRecord(p.k_done[b], p.s_k));
        TRY(hipStreamWaitEvent(p.s_out, p.k_done[b], 0));
        TRY(issue_out(rs.out, dout, p.s_out));
        TRY(hipEventRecord(p.out_done[b], p.s_out));
    }
    TRY(hipMemcpyAsync(p.hmeta + o_copied, dm + o_copied, o_scratch - o_copied, hipMemcpyDeviceToHost, p.s_k));
    TRY(hipStreamSynchronize(p.s_k));
    TRY(hipStreamSynchronize(p.s_out));
    drain.armed = false;

    const int64_t *hc = (const int64_t *)(p.hmeta + o_copied);
    std::memcpy(h_copied, hc, n * sizeof(int64_t));
    std::memcpy(h_csum, p.hmeta + o_csum, n * sizeof(uint32_t));
    std::memset(h_mask, 0, (n + 31) / 32 * sizeof(uint32_t));
    uint32_t nbad = 0;
    for (size_t i = 0; i < n; ++i)
        if (hc[i] < 0) {
            h_mask[i / 32] |= 1u << (i % 32);
            ++nbad;
        }
    *h_nbad = nbad;
    return hipSuccess;
}

// The header checks of a batch of received fragments: each header's first `need` bytes are gathered
// from the ring into pinned records (the CPU moves header bytes only), checked on the device a chunk
// at a time, and the chunk's mask words and failure count come back.
enum class HdrKind { kResidue, kCompare };
struct HdrArgs {
    HdrKind kind;
    uint32_t hdr_bytes, word_count, crclen, csum_offset;
};
constexpr size_t kHdrChunkBytes = 4u << 20;

hipError_t host_headers(const uint8_t *ring, const uint64_t *offs, size_t n, size_t need, const HdrArgs &a,
                        uint32_t *h_mask, uint32_t *h_nbad, int mode) {
    const size_t rec = align_up(std::max<size_t>(need, 4), 4);
    const size_t per = std::max<size_t>(64, (kHdrChunkBytes / rec) & ~(size_t)63);  // whole mask words
    const size_t nch = (n + per - 1) / per;
    PipeState *pp = nullptr;
    TRY(pipe_ctx(&pp));
    PipeState &p = *pp;
    const uint32_t *img = nullptr;
    TRY(device_tables(p.dev, &img));
    const size_t slot = align_up(std::min(n, per) * rec, 256);
    TRY(ensure_chunks(p, slot));
    const size_t mwords = (n + 31) / 32;
    const size_t o_res = kBufs * slot, o_nbad = o_res + align_up(mwords * sizeof(uint32_t), 256);
    const size_t total = o_nbad + nch * sizeof(uint32_t);
    TRY(ensure_meta(p, total));  // pinned: kBufs gather slots, then the results; device: the results
    uint8_t *dres = p.dmeta;     // [mask words | nbad per chunk] at device offset 0
    const size_t d_nbad = o_nbad - o_res;

    PipeDrain drain(p);
    for (size_t c = 0; c < nch; ++c) {
        const int b = (int)(c % kBufs);
        const size_t i0 = c * per, m = std::min(per, n - i0);
        uint8_t *hs = p.hmeta + (size_t)b * slot;
        uint8_t *ds = p.dchunk + (size_t)b * p.chunk_bytes;
        if (c >= (size_t)kBufs) {
            TRY(hipEventSynchronize(p.in_done[b]));  // the pinned slot's last H2D is done
            TRY(hipStreamWaitEvent(p.s_in, p.k_done[b], 0));
        }
        for (size_t i = 0; i < m; ++i) std::memcpy(hs + i * rec, ring + offs[i0 + i], need);
        TRY(hipMemcpyAsync(ds, hs, m * rec, hipMemcpyHostToDevice, p.s_in));
        TRY(hipEventRecord(p.in_done[b], p.s_in));
        TRY(hipStreamWaitEvent(p.s_k, p.in_done[b], 0));
        uint32_t *mk = (uint32_t *)dres + i0 / 32, *nb = (uint32_t *)(dres + d_nbad) + c;
        if (a.kind == HdrKind::kResidue)
            TRY(launch_header_check(ds, m, rec, a.hdr_bytes, a.word_count, a.csum_offset, mode, img, mk, nb, p.s_k));
        else
            TRY(launch_header_compare(ds, m, rec, a.crclen, a.csum_offset, mode, img, mk, nb, p.s_k));
        TRY(hipEventRecord(p.k_done[b], p.s_k));
    }
    TRY(hipMemcpyAsync(p.hmeta + o_res, dres, total - o_res, hipMemcpyDeviceToHost, p.s_k));
    TRY(hipStreamSynchronize(p.s_k));
    drain.armed = false;
    std::memcpy(h_mask, p.hmeta + o_res, mwords * sizeof(uint32_t));
    uint32_t nbad = 0;
    for (size_t c = 0; c < nch; ++c) nbad += ((const uint32_t *)(p.hmeta + o_nbad))[c];
    *h_nbad = nbad;
    return hipSuccess;
}

int check_headers_args(const void *h_ring, size_t ring_bytes, const uint64_t *offs, size_t n, size_t need,
                       uint32_t csum_offset, uint32_t *h_mask, uint32_t *h_nbad, int mode) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32) return (int)hipErrorInvalidValue;
    if (!h_nbad || (csum_offset & 3u) || n > 0xFFFFFFFFull) return (int)hipErrorInvalidValue;
    if (n && (!h_ring || !offs || !h_mask)) return (int)hipErrorInvalidValue;
    for (size_t i = 0; i < n; ++i)
        if (offs[i] > ring_bytes || need > ring_bytes - offs[i]) return (int)hipErrorInvalidValue;
    return 0;
}

}  // namespace
}  // namespace lampi

using namespace lampi;

extern "C" {

int lampi_host_copy_to_app_batch(const void *h_ring, size_t ring_bytes, const lampi_host_recv_frag *h_frags, size_t n,
                                 int64_t *h_copied, uint32_t *h_csum, uint32_t *h_mask, uint32_t *h_nbad, int mode) {
    const uint32_t hint = LAMPI_CSUM_ROWS_HINT_OF(mode);
    mode &= ~LAMPI_CSUM_ROWS_HINT_MASK;
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32 && mode != LAMPI_CSUM_NONE)
        return (int)hipErrorInvalidValue;
    if (!h_nbad || n > 0xFFFFFFFFull) return (int)hipErrorInvalidValue;
    if (n == 0) {
        *h_nbad = 0;
        return 0;
    }
    if (!h_frags || !h_copied || !h_csum || !h_mask) return (int)hipErrorInvalidValue;
    for (size_t j = 0; j < n; ++j) {
        const lampi_host_recv_frag &x = h_frags[j];
        if (to_copy(x) == 0) continue;  // its bytes are never read: no constraint on frag_off / app
        if (!h_ring || !x.app || x.length > kHostMaxFrag || x.frag_off > ring_bytes ||
            x.length > ring_bytes - x.frag_off)
            return (int)hipErrorInvalidValue;
    }
    return (int)host_recv((const uint8_t *)h_ring, ring_bytes, h_frags, n, h_copied, h_csum, h_mask, h_nbad, mode,
                          hint);
}

int lampi_host_header_check_batch(const void *h_ring, size_t ring_bytes, const uint64_t *h_hdr_offs, size_t n,
                                  uint32_t hdr_bytes, uint32_t word_count, uint32_t csum_offset, uint32_t *h_mask,
                                  uint32_t *h_nbad, int mode) {
    // CRC mode reads the whole header (the stored checksum included); SUM mode word_count words and
    // the stored checksum
    const size_t need = mode == LAMPI_CSUM_CRC32 ? (size_t)hdr_bytes
                                                 : std::max<size_t>(4 * (size_t)word_count, (size_t)csum_offset + 4);
    const int rc = check_headers_args(h_ring, ring_bytes, h_hdr_offs, n, need, csum_offset, h_mask, h_nbad, mode);
    if (rc) return rc;
    if (n == 0) {
        *h_nbad = 0;
        return 0;
    }
    const HdrArgs a{HdrKind::kResidue, hdr_bytes, word_count, 0u, csum_offset};
    return (int)host_headers((const uint8_t *)h_ring, h_hdr_offs, n, need, a, h_mask, h_nbad, mode);
}

int lampi_host_header_compare_batch(const void *h_ring, size_t ring_bytes, const uint64_t *h_hdr_offs, size_t n,
                                    uint32_t crclen, uint32_t csum_offset, uint32_t *h_mask, uint32_t *h_nbad,
                                    int mode) {
    const size_t need = std::max<size_t>(crclen, (size_t)csum_offset + 4);
    const int rc = check_headers_args(h_ring, ring_bytes, h_hdr_offs, n, need, csum_offset, h_mask, h_nbad, mode);
    if (rc) return rc;
    if (n == 0) {
        *h_nbad = 0;
        return 0;
    }
    const HdrArgs a{HdrKind::kCompare, 0u, 0u, crclen, csum_offset};
    return (int)host_headers((const uint8_t *)h_ring, h_hdr_offs, n, need, a, h_mask, h_nbad, mode);
}

}  // extern "C"
