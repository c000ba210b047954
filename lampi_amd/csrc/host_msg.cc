// host_msg.cc -- the host-memory message path of liblampi_csum.so (lampi_host_msg_csum,
// lampi_host_msg_bcopy; include/lampi_csum.h).
//
// LA-MPI's send loop walks a message in host memory fragment by fragment, copying each payload
// into its NIC buffer with the checksum fused (gmPath::send, ref src/path/gm/path.cc:98-176;
// gmSendFragDesc::init, src/path/gm/sendFrag.cc:147-155) or checksumming a DMA source in place
// (Quadrics, src/path/quadrics/sendFrag.h:861-872).  Here one call takes a range of those
// fragments and runs a chunked pipeline on three per-thread streams:
//
//   s_in : H2D of chunk i, straight from the caller's buffer
//   s_k  : the checksum kernels of chunk i (the same launches as lampi_msg_csum) into a device
//          array of per-fragment results
//   s_out: (bcopy) D2H of chunk i's bytes -- the very bytes the kernel checksummed -- into the
//          caller's fragment slots, one pitched 2D copy per chunk
//
// with kBufs device chunks in flight, so chunk i+1 moves over PCIe while chunk i is checksummed
// and copied out.  The results come back in one D2H at the end.  Page-locked and pageable host
// buffers take the same calls: the runtime stages pageable H2D at the pinned rate (52.7 against
// 53.3 GiB/s, a CPU copy into pinned bounce buffers reached 25, tools/microbench/pcie_duplex.hip,
// profiles/r03/pcie_duplex_run*.txt); pageable slots cost the D2H half its rate (19.8 against
// 32.8 GiB/s beside a concurrent H2D), so NIC rings should be page-locked (lampi_host_register).
// There is no CPU checksum and no CPU copy of payload bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../../include/lampi_csum.h"
#include "frag_csum_kernels.h"
#include "host_internal.h"
#include "host_pipe.h"

namespace lampi {
namespace {

struct PipeCtx {
    PipeState st;
    PipeCtx() = default;
    PipeCtx(const PipeCtx &) = delete;
    PipeCtx &operator=(const PipeCtx &) = delete;
    ~PipeCtx() { release(); }

    // Free everything on the device it was made on; errors are ignored (this also runs at
    // thread exit, where nobody is left to report them to).
    void release() {
        PipeState &p = st;
        if (p.dev < 0) return;
        int cur = -1;
        const bool have_cur = hipGetDevice(&cur) == hipSuccess;
        if (have_cur && cur != p.dev) (void)hipSetDevice(p.dev);
        for (hipStream_t s : {p.s_in, p.s_k, p.s_out})
            if (s) (void)hipStreamSynchronize(s);
        if (p.s_k) release_stream_scratch(p.s_k);  // the light copies' group values of this thread on s_k
        for (uint8_t *d : {p.dchunk, p.dout, p.dmeta})
            if (d) (void)hipFree(d);
        pinned_free(p.hmeta, p.hmeta_cap);
        for (int b = 0; b < kBufs; ++b)
            for (hipEvent_t e : {p.in_done[b], p.k_done[b], p.out_done[b]})
                if (e) (void)hipEventDestroy(e);
        for (hipStream_t s : {p.s_in, p.s_k, p.s_out})
            if (s) (void)hipStreamDestroy(s);
        if (have_cur && cur != p.dev) (void)hipSetDevice(cur);
        st = PipeState{};
    }
};

thread_local PipeCtx t_pipe;

#define TRY LAMPI_TRY

hipError_t grow_device(uint8_t *&ptr, size_t &cap, size_t want, PipeState &p) {
    if (cap >= want) return hipSuccess;
    if (ptr) {
        for (hipStream_t s : {p.s_in, p.s_k, p.s_out}) TRY(hipStreamSynchronize(s));
        TRY(hipFree(ptr));
        ptr = nullptr;
        cap = 0;
    }
    TRY(hipMalloc((void **)&ptr, want));
    cap = want;
    return hipSuccess;
}

}  // namespace

hipError_t pipe_ctx(PipeState **out) {
    int dev = 0;
    TRY(current_device(&dev));
    PipeState &p = t_pipe.st;
    if (p.dev != dev) {
        t_pipe.release();  // device changed (or first use): the old buffers belong to the old device
        p.dev = dev;
        for (hipStream_t *s : {&p.s_in, &p.s_k, &p.s_out}) TRY(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
        for (int b = 0; b < kBufs; ++b)
            for (hipEvent_t *e : {&p.in_done[b], &p.k_done[b], &p.out_done[b]})
                TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    *out = &p;
    return hipSuccess;
}

size_t chunk_target(bool duplex) {
    if (const char *e = std::getenv("LAMPI_HOST_CHUNK_BYTES")) {
        const unsigned long long v = std::strtoull(e, nullptr, 0);
        if (v >= 4096) return (size_t)v;
    }
    return duplex ? kChunkDuplex : kChunkTarget;
}

// every chunk starts 256-byte aligned
hipError_t ensure_chunks(PipeState &p, size_t chunk) {
    chunk = align_up(chunk, 256);
    if (p.chunk_bytes >= chunk) return hipSuccess;
    size_t cap = 0;
    TRY(grow_device(p.dchunk, cap, kBufs * chunk, p));
    p.chunk_bytes = chunk;
    return hipSuccess;
}

hipError_t ensure_out_chunks(PipeState &p, size_t chunk) {
    chunk = align_up(chunk, 256);
    if (p.out_bytes >= chunk) return hipSuccess;
    size_t cap = 0;
    TRY(grow_device(p.dout, cap, kBufs * chunk, p));
    p.out_bytes = chunk;
    return hipSuccess;
}

hipError_t ensure_meta(PipeState &p, size_t bytes) {
    bytes = align_up(std::max<size_t>(bytes, 4096), 4096);
    TRY(grow_device(p.dmeta, p.dmeta_cap, bytes, p));
    if (p.hmeta_cap < bytes) {
        // the previous call synchronized before it returned: nothing reads the old image
        pinned_free(p.hmeta, p.hmeta_cap);
        p.hmeta = nullptr;
        p.hmeta_cap = 0;
        TRY(pinned_alloc((void **)&p.hmeta, bytes, hipHostMallocDefault));
        p.hmeta_cap = bytes;
    }
    return hipSuccess;
}

namespace {

struct Range {
    size_t frag_len, nfrag, last;  // fragments of the call, bytes of its last fragment
};

// D2H of a chunk's fragments [f0, f0 + nf) (bytes d, packed frag_len apart; the last one
// possibly short) into slots h_ring + f*stride, on s_out.
hipError_t copy_out(PipeState &p, uint8_t *h_ring, size_t stride, const uint8_t *d, size_t f0, size_t nf,
                    const Range &r) {
    const bool short_tail = f0 + nf == r.nfrag && r.last != r.frag_len;
    const size_t full = nf - (short_tail ? 1 : 0);
    uint8_t *h = h_ring + f0 * stride;
    if (full == 1 || (full > 1 && stride == r.frag_len))
        TRY(hipMemcpyAsync(h, d, full * r.frag_len, hipMemcpyDeviceToHost, p.s_out));
    else if (full > 1)
        TRY(hipMemcpy2DAsync(h, stride, d, r.frag_len, r.frag_len, full, hipMemcpyDeviceToHost, p.s_out));
    if (short_tail && r.last)
        TRY(hipMemcpyAsync(h + full * stride, d + full * r.frag_len, r.last, hipMemcpyDeviceToHost, p.s_out));
    return hipSuccess;
}

hipError_t host_msg(const uint8_t *h_msg, size_t msg_len, size_t frag_len, size_t k_first, size_t k_count,
                    uint8_t *h_ring, size_t stride, uint32_t partial, uint32_t *h_out, int mode) {
    PipeState *pp = nullptr;
    TRY(pipe_ctx(&pp));
    PipeState &p = *pp;
    int dev = p.dev;
    const uint32_t *img = nullptr;
    TRY(device_tables(dev, &img));

    const size_t b0 = k_first * frag_len;
    const size_t b1 = std::min(msg_len, (k_first + k_count) * frag_len);
    const Range r{frag_len, k_count, b1 - (b0 + (k_count - 1) * frag_len)};
    const size_t fpc = std::max<size_t>(1, chunk_target(h_ring != nullptr) / frag_len);  // fragments per chunk
    const size_t cb = fpc * frag_len;
    TRY(ensure_chunks(p, cb));
    TRY(ensure_meta(p, k_count * sizeof(uint32_t)));
    uint32_t *dres = (uint32_t *)p.dmeta, *hres = (uint32_t *)p.hmeta;
    const bool copy = h_ring != nullptr;
    // checksumming off (bcopy only): the bytes go up and come back into the slots, no kernel, no results
    // (MEMCOPY_FUNC instead of bcopy_uicrc / bcopy_uicsum, ref src/path/gm/sendFrag.cc:153-155)
    const bool none = mode == LAMPI_CSUM_NONE;

    PipeDrain drain(p);  // any early return below leaves nothing in flight
    const size_t nchunks = (k_count + fpc - 1) / fpc;
    for (size_t i = 0; i < nchunks; ++i) {
        const int b = (int)(i % kBufs);
        const size_t f0 = i * fpc, nf = std::min(fpc, k_count - f0);
        const size_t off = b0 + f0 * frag_len, nb = std::min(nf * frag_len, b1 - off);
        uint8_t *d = p.dchunk + (size_t)b * p.chunk_bytes;
        // chunk b is free once chunk i - kBufs was checksummed and copied out (every call, failed
        // ones included, drains the streams before it returns)
        if (i >= (size_t)kBufs) {
            TRY(hipStreamWaitEvent(p.s_in, p.k_done[b], 0));
            if (copy) TRY(hipStreamWaitEvent(p.s_in, p.out_done[b], 0));
        }
        TRY(hipMemcpyAsync(d, h_msg + off, nb, hipMemcpyHostToDevice, p.s_in));
        TRY(hipEventRecord(p.in_done[b], p.s_in));
        TRY(hipStreamWaitEvent(p.s_k, p.in_done[b], 0));
        if (!none) TRY(launch_msg_csum(d, nb, frag_len, partial, dres + f0, mode, dev, img, p.s_k));
        TRY(hipEventRecord(p.k_done[b], p.s_k));
        if (!copy) continue;
        TRY(hipStreamWaitEvent(p.s_out, p.in_done[b], 0));
        TRY(copy_out(p, h_ring, stride, d, f0, nf, r));
        TRY(hipEventRecord(p.out_done[b], p.s_out));
    }
    if (!none) TRY(hipMemcpyAsync(hres, dres, k_count * sizeof(uint32_t), hipMemcpyDeviceToHost, p.s_k));
    TRY(hipStreamSynchronize(p.s_k));
    if (copy) TRY(hipStreamSynchronize(p.s_out));
    drain.armed = false;
    if (!none) std::memcpy(h_out, hres, k_count * sizeof(uint32_t));
    return hipSuccess;
}

// Argument checks shared by both entry points; fills the one empty fragment of an empty message.
// none_ok: LAMPI_CSUM_NONE is accepted (the bcopy: copies only, h_out unused and may be NULL).
int check_args(const void *h_msg, size_t msg_len, size_t frag_len, size_t k_first, size_t k_count,
               uint32_t *h_out, int mode, bool *done, uint32_t partial, bool none_ok = false) {
    *done = false;
    const bool none = none_ok && mode == LAMPI_CSUM_NONE;
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32 && !none) return (int)hipErrorInvalidValue;
    if (frag_len == 0 || frag_len > kHostMaxFrag) return (int)hipErrorInvalidValue;
    const size_t nfr = msg_len ? (msg_len - 1) / frag_len + 1 : 1;
    if (k_first > nfr || k_count > nfr - k_first) return (int)hipErrorInvalidValue;
    if (k_count == 0) {
        *done = true;
        return 0;
    }
    if ((!h_out && !none) || (msg_len && !h_msg)) return (int)hipErrorInvalidValue;
    if (msg_len == 0) {  // one empty fragment: the register unchanged / an empty sum (nothing with checksumming off)
        if (!none) h_out[0] = mode == LAMPI_CSUM_CRC32 ? partial : 0u;
        *done = true;
    }
    return 0;
}

}  // namespace

void release_pipeline() { t_pipe.release(); }

}  // namespace lampi

using namespace lampi;

extern "C" {

int lampi_host_msg_csum(const void *h_msg, size_t msg_len, size_t frag_len, size_t k_first, size_t k_count,
                        uint32_t partial, uint32_t *h_out, int mode) {
    bool done = false;
    const int rc = check_args(h_msg, msg_len, frag_len, k_first, k_count, h_out, mode, &done, partial);
    if (rc || done) return rc;
    return (int)host_msg((const uint8_t *)h_msg, msg_len, frag_len, k_first, k_count, nullptr, 0, partial, h_out,
                         mode);
}

int lampi_host_msg_bcopy(const void *h_msg, size_t msg_len, size_t frag_len, size_t k_first, size_t k_count,
                         void *h_ring, size_t slot_stride, uint32_t partial, uint32_t *h_out, int mode) {
    bool done = false;
    const int rc = check_args(h_msg, msg_len, frag_len, k_first, k_count, h_out, mode, &done, partial, true);
    if (rc || done) return rc;
    if (!h_ring || slot_stride < frag_len) return (int)hipErrorInvalidValue;
    return (int)host_msg((const uint8_t *)h_msg, msg_len, frag_len, k_first, k_count, (uint8_t *)h_ring, slot_stride,
                         partial, h_out, mode);
}

}  // extern "C"
