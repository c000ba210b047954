// host_chain.cc -- chained checksums over typemap pieces in host memory (lampi_host_chain_csum_batch,
// include/lampi_csum.h): the host-memory form of lampi_chain_csum_batch.
//
// A non-contiguous datatype is sent as a list of typemap pieces per fragment: the send loop gathers
// them into the fragment's payload with the checksum threaded through the pieces
// (gmSendFragDesc::init, ref src/path/gm/sendFrag.cc:157-217: `csum = bcopy_uicrc(src, dst, len, len,
// csum)` / `csum += bcopy_uicsum(...)`; IB src/path/ib/sendFrag.cc:140-203); the receiver scatters a
// fragment back into the typemap pieces of the application buffer the same way
// (non_contiguous_copy, src/path/common/BaseDesc.cc:72-163).  Both are one call here: the pieces'
// source bytes go up in as few DMA transfers as their layout allows (touching pieces one copy, a
// strided vector's equal elements one 2D copy), the chain kernels of the device path
// (launch_chain) checksum and copy them, and the copies come back the same way (a gathered payload
// one copy, scattered equal elements one 2D copy) -- on the per-thread pipeline of host_msg.cc.
// The DMA engines read exactly the pieces' bytes and write exactly their copies.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/lampi_csum.h"
#include "frag_csum_kernels.h"
#include "host_internal.h"
#include "host_pipe.h"
#include "host_plan.h"

namespace lampi {
namespace {

#define TRY LAMPI_TRY

uint32_t piece_len(const lampi_host_piece &x) { return std::max(x.copylen, x.csumlen); }

// Pieces as the planner sees them (absolute addresses, base 0); a chunk may start only at a fragment's
// first piece, so every fragment's pieces are checksummed by one launch.
struct ChainItems {
    const lampi_host_piece *p;
    size_t n;
    const std::vector<uint8_t> *starts;  // starts[j]: piece j opens a fragment (or lies outside them all)
    size_t size() const { return n; }
    PlanItem get(size_t j) const {
        const lampi_host_piece &x = p[j];
        return PlanItem{(uint64_t)(uintptr_t)x.src, piece_len(x), (uint8_t *)x.dst, x.dst ? x.copylen : 0u};
    }
    bool boundary(size_t j) const { return (*starts)[j] != 0; }
};

struct ChainScratch {
    std::vector<size_t> din, dout;
    std::vector<uint8_t> starts;
    std::vector<InXfer> in;
    std::vector<OutXfer> out;
};
thread_local ChainScratch t_chain;

// Verdict arrays of lampi_host_chain_copy_to_app_batch (null: checksums only).
struct HostChainVerdict {
    const uint32_t *expected = nullptr;
    int64_t *copied = nullptr;
    uint32_t *mask = nullptr;
    uint32_t *nbad = nullptr;
};

hipError_t host_chain(const lampi_host_piece *pc, size_t npieces, const uint32_t *first, size_t nfrags,
                      uint32_t *h_out, int mode, const HostChainVerdict *hv = nullptr) {
    ChainScratch &cs = t_chain;
    if (cs.din.size() < npieces) {
        cs.din.resize(npieces);
        cs.dout.resize(npieces);
    }
    // pieces outside [first[0], first[nfrags]) belong to no fragment: never read
    const size_t pa = first[0], pb = first[nfrags];
    cs.starts.assign(npieces, 1);
    for (size_t j = pa; j < pb; ++j) cs.starts[j] = 0;
    for (size_t f = 0; f < nfrags; ++f)
        if (first[f] < npieces) cs.starts[first[f]] = 1;
    // pieces outside every fragment move nothing
    struct Masked {
        ChainItems it;
        size_t pa, pb;
        size_t size() const { return it.size(); }
        PlanItem get(size_t j) const { return j < pa || j >= pb ? PlanItem{0, 0, nullptr, 0} : it.get(j); }
        bool boundary(size_t j) const { return it.boundary(j); }
    } masked{ChainItems{pc, npieces, &cs.starts}, pa, pb};

    StreamPlanner<Masked> pl(masked, PlanRules{}, chunk_target(true), cs.din.data(), cs.dout.data());
    PipeState *pp = nullptr;
    TRY(pipe_ctx(&pp));
    PipeState &p = *pp;
    const uint32_t *img = nullptr;
    TRY(device_tables(p.dev, &img));
    TRY(ensure_chunks(p, pl.in_need()));
    TRY(ensure_out_chunks(p, pl.out_need()));

    // descriptors (each chunk's go up with it) | chunk-relative CSR offsets | results | chain scratch
    const size_t o_first = align_up(npieces * sizeof(lampi_copy_desc), 256);
    const size_t nfirst = nfrags + npieces + 2;  // each chunk's nf + 1 entries; chunks <= pieces + 1
    const size_t o_out = align_up(o_first + nfirst * sizeof(uint32_t), 256);
    const size_t o_vals = align_up(o_out + nfrags * sizeof(uint32_t), 256);
    const size_t total = o_vals + 2 * std::max<size_t>(npieces, 1) * sizeof(uint32_t);
    TRY(ensure_meta(p, total));
    lampi_copy_desc *hd = (lampi_copy_desc *)p.hmeta;
    uint32_t *hf = (uint32_t *)(p.hmeta + o_first);
    uint8_t *dm = p.dmeta;
    uint32_t *dvals = (uint32_t *)(dm + o_vals);

    PipeDrain drain(p);
    ChunkPlan k;
    size_t fa = 0, first_used = 0;
    for (size_t c = 0; pl.next(k, cs.in, cs.out); ++c) {
        const int b = (int)(c % kBufs);
        uint8_t *din = p.dchunk + (size_t)b * p.chunk_bytes;
        uint8_t *dout = p.dout + (size_t)b * p.out_bytes;
        // the chunk's fragments: those whose first piece lies in [k.j0, k.j1) -- their pieces all do, as a
        // chunk starts only at a fragment's first piece -- and, in the last chunk, the empty ones after
        const bool last = k.j1 >= npieces;
        size_t fb = fa;
        while (fb < nfrags && (last || first[fb] < k.j1)) ++fb;
        const size_t j0 = first[fa < nfrags ? fa : nfrags], j1 = first[fb];
        for (size_t j = j0; j < j1; ++j) {
            const lampi_host_piece &x = pc[j];
            const uint32_t len = piece_len(x);
            const bool cp = x.dst && x.copylen;
            hd[j] = lampi_copy_desc{(uint64_t)(uintptr_t)(len ? din + cs.din[j] : din),
                                    (uint64_t)(uintptr_t)(cp ? dout + cs.dout[j] : dout), cp ? x.copylen : 0u,
                                    x.csumlen, x.partial, 0u};
        }
        uint32_t *cf = hf + first_used;
        for (size_t f = fa; f <= fb; ++f) cf[f - fa] = (uint32_t)(first[f] - j0);
        if (c >= (size_t)kBufs) {
            TRY(hipStreamWaitEvent(p.s_in, p.k_done[b], 0));
            TRY(hipStreamWaitEvent(p.s_in, p.out_done[b], 0));
        }
        if (j1 > j0)
            TRY(hipMemcpyAsync(dm + j0 * sizeof(lampi_copy_desc), hd + j0, (j1 - j0) * sizeof(lampi_copy_desc),
                               hipMemcpyHostToDevice, p.s_in));
        uint32_t *dcf = (uint32_t *)(dm + o_first) + first_used;
        TRY(hipMemcpyAsync(dcf, cf, (fb - fa + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, p.s_in));
        TRY(issue_in(cs.in, nullptr, din, p.s_in));
        TRY(hipEventRecord(p.in_done[b], p.s_in));
        TRY(hipStreamWaitEvent(p.s_k, p.in_done[b], 0));
        // (a delivery batch's fragments start from CRC_INITIAL_REGISTER, nonContigCopyFunction's first call; its
        // verdicts are taken on the host below from the checksums that come back)
        ChainVerdict init;
        init.init = 1;
        if (fb > fa)
            TRY(launch_chain((const lampi_copy_desc *)dm + j0, j1 - j0, dcf, fb - fa, (uint32_t *)(dm + o_out) + fa,
                             mode, img, dvals + j0, dvals + npieces + j0, p.s_k, hv ? &init : nullptr));
        TRY(hipEventRecord(p.k_done[b], p.s_k));
        TRY(hipStreamWaitEvent(p.s_out, p.k_done[b], 0));
        TRY(issue_out(cs.out, dout, p.s_out));
        TRY(hipEventRecord(p.out_done[b], p.s_out));
        first_used += fb - fa + 1;
        fa = fb;
    }
    TRY(hipMemcpyAsync(p.hmeta + o_out, dm + o_out, nfrags * sizeof(uint32_t), hipMemcpyDeviceToHost, p.s_k));
    TRY(hipStreamSynchronize(p.s_k));
    TRY(hipStreamSynchronize(p.s_out));
    drain.armed = false;
    std::memcpy(h_out, p.hmeta + o_out, nfrags * sizeof(uint32_t));
    if (hv) {  // CopyToApp's non-contiguous verdict (ref BaseDesc.cc:326-340 with CheckData, gm/recvFrag.h:213-257)
        std::memset(hv->mask, 0, (nfrags + 31) / 32 * sizeof(uint32_t));
        uint32_t nbad = 0;
        for (size_t f = 0; f < nfrags; ++f) {
            int64_t copied = 0;
            for (size_t j = first[f]; j < first[f + 1]; ++j) copied += pc[j].copylen;
            const bool bad = mode != LAMPI_CSUM_NONE && copied != 0 && h_out[f] != hv->expected[f];
            hv->copied[f] = bad ? -1 : copied;
            if (bad) {
                hv->mask[f / 32] |= 1u << (f % 32);
                ++nbad;
            }
        }
        *hv->nbad = nbad;
    }
    return hipSuccess;
}

int check_chain_args(const lampi_host_piece *h_pieces, size_t npieces, const uint32_t *h_first, size_t nfrags) {
    if (!h_first || (npieces && !h_pieces) || npieces > 0xFFFFFFFFull || nfrags > 0xFFFFFFFFull)
        return (int)hipErrorInvalidValue;
    if (h_first[nfrags] > npieces) return (int)hipErrorInvalidValue;
    for (size_t f = 0; f < nfrags; ++f) {
        if (h_first[f] > h_first[f + 1]) return (int)hipErrorInvalidValue;
        uint64_t bytes = 0;
        for (size_t j = h_first[f]; j < h_first[f + 1]; ++j) {
            const lampi_host_piece &x = h_pieces[j];
            const uint32_t len = piece_len(x);
            if ((len && !x.src) || (x.copylen && !x.dst)) return (int)hipErrorInvalidValue;
            bytes += len;
        }
        if (bytes > kHostMaxFrag) return (int)hipErrorInvalidValue;
    }
    return 0;
}

}  // namespace
}  // namespace lampi

using namespace lampi;

extern "C" {

int lampi_host_chain_csum_batch(const lampi_host_piece *h_pieces, size_t npieces, const uint32_t *h_first,
                                size_t nfrags, uint32_t *h_out, int mode) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32) return (int)hipErrorInvalidValue;
    if (nfrags == 0) return 0;
    if (!h_out) return (int)hipErrorInvalidValue;
    const int rc = check_chain_args(h_pieces, npieces, h_first, nfrags);
    if (rc) return rc;
    return (int)host_chain(h_pieces, npieces, h_first, nfrags, h_out, mode);
}

int lampi_host_chain_copy_to_app_batch(const lampi_host_piece *h_pieces, size_t npieces, const uint32_t *h_first,
                                       size_t nfrags, const uint32_t *h_expected, int64_t *h_copied, uint32_t *h_csum,
                                       uint32_t *h_mask, uint32_t *h_nbad, int mode) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32 && mode != LAMPI_CSUM_NONE)
        return (int)hipErrorInvalidValue;
    if (!h_nbad) return (int)hipErrorInvalidValue;
    if (nfrags == 0) {
        *h_nbad = 0;
        return 0;
    }
    if (!h_copied || !h_csum || !h_mask || (mode != LAMPI_CSUM_NONE && !h_expected)) return (int)hipErrorInvalidValue;
    const int rc = check_chain_args(h_pieces, npieces, h_first, nfrags);
    if (rc) return rc;
    HostChainVerdict v;
    v.expected = h_expected;
    v.copied = h_copied;
    v.mask = h_mask;
    v.nbad = h_nbad;
    return (int)host_chain(h_pieces, npieces, h_first, nfrags, h_csum, mode, &v);
}

}  // extern "C"
