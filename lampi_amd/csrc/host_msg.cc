// host_msg.cc -- the host-memory message path of liblampi_csum.so (lampi_host_msg_csum,
// lampi_host_msg_bcopy; include/lampi_csum.h).
//
// LA-MPI's send loop walks a message in host memory fragment by fragment, copying each payload
// into its NIC buffer with the checksum fused (gmPath::send, ref src/path/gm/path.cc:98-176;
// gmSendFragDesc::init, src/path/gm/sendFrag.cc:147-155) or checksumming a DMA source in place
// (Quadrics, src/path/quadrics/sendFrag.h:861-872).  Here one call takes a range of those
// fragments and runs a chunked pipeline on three per-thread streams:
//
//   s_in : H2D of chunk i (DMA straight from the caller's buffer when it is page-locked, through
//          a ring of pinned bounce pieces otherwise)
//   s_k  : the checksum kernels of chunk i (the same launches as lampi_msg_csum) into a device
//          array of per-fragment results
//   s_out: (bcopy) D2H of chunk i's bytes -- the very bytes the kernel checksummed -- into the
//          caller's fragment slots: one 2D copy per chunk (slot pitch) when the slots are
//          page-locked, a pinned bounce and a CPU scatter otherwise
//
// with kBufs device chunks in flight, so chunk i+1 moves over PCIe while chunk i is checksummed
// and copied out.  The results come back in one D2H at the end.  There is no CPU checksum: the
// CPU only moves bytes between pageable memory and pinned staging.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "../../include/lampi_csum.h"
#include "host_internal.h"

namespace lampi {
namespace {

constexpr int kBufs = 3;                    // device chunks in flight
constexpr size_t kChunkTarget = 16u << 20;  // bytes per chunk (whole fragments; at least one)
constexpr int kInSlots = 4;                 // pageable sources: pinned bounce pieces ...
constexpr size_t kInPiece = 4u << 20;       // ... of this many bytes

// Everything a thread's pipeline holds; a plain aggregate, so release() can reset it.
struct PipeState {
    int dev = -1;
    hipStream_t s_in = nullptr, s_k = nullptr, s_out = nullptr;
    hipEvent_t in_done[kBufs] = {}, k_done[kBufs] = {}, out_done[kBufs] = {}, bin_free[kInSlots] = {};
    hipEvent_t bout_done[2] = {};
    uint8_t *dchunk = nullptr;  // kBufs chunks of chunk_bytes
    size_t chunk_bytes = 0;
    uint32_t *dres = nullptr;  // per-fragment results of the call
    size_t res_cap = 0;
    uint32_t *hres = nullptr;  // pinned copy of them (when the caller's array is pageable)
    size_t hres_cap = 0;
    uint8_t *bin = nullptr;    // pinned bounce pieces for pageable sources (kInSlots x kInPiece)
    uint32_t bin_next = 0;     // next bounce piece to fill
    uint8_t *bout = nullptr;   // pinned bounce for pageable slots: two chunks
    size_t bout_chunk = 0;
};

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
        if (p.dchunk) (void)hipFree(p.dchunk);
        if (p.dres) (void)hipFree(p.dres);
        pinned_free(p.hres, p.hres_cap * sizeof(uint32_t));
        pinned_free(p.bin, kInSlots * kInPiece);
        pinned_free(p.bout, 2 * p.bout_chunk);
        for (int b = 0; b < kBufs; ++b)
            for (hipEvent_t e : {p.in_done[b], p.k_done[b], p.out_done[b]})
                if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : p.bin_free)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : p.bout_done)
            if (e) (void)hipEventDestroy(e);
        for (hipStream_t s : {p.s_in, p.s_k, p.s_out})
            if (s) (void)hipStreamDestroy(s);
        if (have_cur && cur != p.dev) (void)hipSetDevice(cur);
        st = PipeState{};
    }
};

thread_local PipeCtx t_pipe;

#define TRY(call)                                   \
    do {                                            \
        const hipError_t e_ = (call);               \
        if (e_ != hipSuccess) return e_;            \
    } while (0)

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
        for (hipEvent_t &e : p.bin_free) TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (hipEvent_t &e : p.bout_done) TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    *out = &p;
    return hipSuccess;
}

// Capacity helpers: grow only (a device buffer is freed after the streams drained).
hipError_t ensure_chunks(PipeState &p, size_t chunk) {
    chunk = (chunk + 255) & ~(size_t)255;  // every chunk starts 256-byte aligned
    if (p.chunk_bytes >= chunk) return hipSuccess;
    if (p.dchunk) {
        for (hipStream_t s : {p.s_in, p.s_k, p.s_out}) TRY(hipStreamSynchronize(s));
        TRY(hipFree(p.dchunk));
        p.dchunk = nullptr;
        p.chunk_bytes = 0;
    }
    TRY(hipMalloc((void **)&p.dchunk, kBufs * chunk));
    p.chunk_bytes = chunk;
    return hipSuccess;
}

hipError_t ensure_results(PipeState &p, size_t n, bool host) {
    if (p.res_cap < n) {
        if (p.dres) {
            TRY(hipStreamSynchronize(p.s_k));
            TRY(hipFree(p.dres));
            p.dres = nullptr;
            p.res_cap = 0;
        }
        TRY(hipMalloc((void **)&p.dres, n * sizeof(uint32_t)));
        p.res_cap = n;
    }
    if (host && p.hres_cap < n) {
        pinned_free(p.hres, p.hres_cap * sizeof(uint32_t));
        p.hres = nullptr;
        p.hres_cap = 0;
        TRY(pinned_alloc((void **)&p.hres, n * sizeof(uint32_t), hipHostMallocDefault));
        p.hres_cap = n;
    }
    return hipSuccess;
}

// H2D of nb bytes at h into d on s_in: one DMA from page-locked memory, or bounce pieces.
hipError_t copy_in(PipeState &p, uint8_t *d, const uint8_t *h, size_t nb, bool pinned) {
    if (pinned) return hipMemcpyAsync(d, h, nb, hipMemcpyHostToDevice, p.s_in);
    if (!p.bin) TRY(pinned_alloc((void **)&p.bin, kInSlots * kInPiece, hipHostMallocDefault));
    for (size_t o = 0; o < nb; o += kInPiece) {
        const size_t n = std::min(kInPiece, nb - o);
        const uint32_t j = p.bin_next++ % kInSlots;
        uint8_t *slot = p.bin + (size_t)j * kInPiece;
        TRY(hipEventSynchronize(p.bin_free[j]));  // its previous DMA has read it
        std::memcpy(slot, h + o, n);
        TRY(hipMemcpyAsync(d + o, slot, n, hipMemcpyHostToDevice, p.s_in));
        TRY(hipEventRecord(p.bin_free[j], p.s_in));
    }
    return hipSuccess;
}

struct Range {
    size_t frag_len, nfrag, last;  // fragments of the call, bytes of its last fragment
};

// D2H of a chunk's fragments [f0, f0 + nf) (bytes d, packed frag_len apart; the last one
// possibly short) into slots h_ring + f*stride, on s_out.
hipError_t copy_out_pinned(PipeState &p, uint8_t *h_ring, size_t stride, const uint8_t *d, size_t f0, size_t nf,
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

// Pageable slots: the chunk goes to a pinned bounce half (s_out), the CPU scatters it later.
struct PendingScatter {
    bool live = false;
    int half = 0;
    size_t f0 = 0, nf = 0;
};

hipError_t scatter(PipeState &p, const PendingScatter &ps, uint8_t *h_ring, size_t stride, const Range &r) {
    if (!ps.live) return hipSuccess;
    TRY(hipEventSynchronize(p.bout_done[ps.half]));
    const uint8_t *b = p.bout + (size_t)ps.half * p.bout_chunk;
    for (size_t i = 0; i < ps.nf; ++i) {
        const size_t f = ps.f0 + i;
        const size_t n = f + 1 == r.nfrag ? r.last : r.frag_len;
        std::memcpy(h_ring + f * stride, b + i * r.frag_len, n);
    }
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
    const size_t fpc = std::max<size_t>(1, kChunkTarget / frag_len);  // fragments per chunk
    const size_t cb = fpc * frag_len;
    TRY(ensure_chunks(p, cb));
    const bool out_pinned = host_range_pinned(h_out, k_count * sizeof(uint32_t));
    TRY(ensure_results(p, k_count, !out_pinned));
    const bool src_pinned = host_range_pinned(h_msg + b0, b1 - b0);
    const bool copy = h_ring != nullptr;
    const bool ring_pinned = copy && host_range_pinned(h_ring, (k_count - 1) * stride + r.last);
    if (copy && !ring_pinned && p.bout_chunk < cb) {
        pinned_free(p.bout, 2 * p.bout_chunk);
        p.bout = nullptr;
        p.bout_chunk = 0;
        TRY(pinned_alloc((void **)&p.bout, 2 * cb, hipHostMallocDefault));
        p.bout_chunk = cb;
    }

    PendingScatter pending;
    const size_t nchunks = (k_count + fpc - 1) / fpc;
    for (size_t i = 0; i < nchunks; ++i) {
        const int b = (int)(i % kBufs);
        const size_t f0 = i * fpc, nf = std::min(fpc, k_count - f0);
        const size_t off = b0 + f0 * frag_len, nb = std::min(nf * frag_len, b1 - off);
        uint8_t *d = p.dchunk + (size_t)b * p.chunk_bytes;
        // chunk b is free once chunk i - kBufs was checksummed and copied out
        TRY(hipStreamWaitEvent(p.s_in, p.k_done[b], 0));
        if (copy) TRY(hipStreamWaitEvent(p.s_in, p.out_done[b], 0));
        TRY(copy_in(p, d, h_msg + off, nb, src_pinned));
        TRY(hipEventRecord(p.in_done[b], p.s_in));
        TRY(hipStreamWaitEvent(p.s_k, p.in_done[b], 0));
        TRY(launch_msg_csum(d, nb, frag_len, partial, p.dres + f0, mode, dev, img, p.s_k));
        TRY(hipEventRecord(p.k_done[b], p.s_k));
        if (!copy) continue;
        TRY(hipStreamWaitEvent(p.s_out, p.in_done[b], 0));
        if (ring_pinned) {
            TRY(copy_out_pinned(p, h_ring, stride, d, f0, nf, r));
        } else {
            const int half = (int)(i & 1);  // its previous chunk (i - 2) was scattered below
            TRY(hipMemcpyAsync(p.bout + (size_t)half * p.bout_chunk, d, nb, hipMemcpyDeviceToHost, p.s_out));
            TRY(hipEventRecord(p.bout_done[half], p.s_out));
        }
        TRY(hipEventRecord(p.out_done[b], p.s_out));
        if (!ring_pinned) {
            TRY(scatter(p, pending, h_ring, stride, r));  // chunk i - 1, while chunk i moves
            pending = {true, (int)(i & 1), f0, nf};
        }
    }
    if (copy && !ring_pinned) TRY(scatter(p, pending, h_ring, stride, r));
    uint32_t *res = out_pinned ? h_out : p.hres;
    TRY(hipMemcpyAsync(res, p.dres, k_count * sizeof(uint32_t), hipMemcpyDeviceToHost, p.s_k));
    TRY(hipStreamSynchronize(p.s_k));
    if (copy) TRY(hipStreamSynchronize(p.s_out));
    if (!out_pinned) std::memcpy(h_out, p.hres, k_count * sizeof(uint32_t));
    return hipSuccess;
}

// Argument checks shared by both entry points; fills the one empty fragment of an empty message.
int check_args(const void *h_msg, size_t msg_len, size_t frag_len, size_t k_first, size_t k_count,
               uint32_t *h_out, int mode, bool *done, uint32_t partial) {
    *done = false;
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32) return (int)hipErrorInvalidValue;
    if (frag_len == 0 || frag_len > 0xFFFFFFFFull) return (int)hipErrorInvalidValue;
    const size_t nfr = msg_len ? (msg_len - 1) / frag_len + 1 : 1;
    if (k_first > nfr || k_count > nfr - k_first) return (int)hipErrorInvalidValue;
    if (k_count == 0) {
        *done = true;
        return 0;
    }
    if (!h_out || (msg_len && !h_msg)) return (int)hipErrorInvalidValue;
    if (msg_len == 0) {  // one empty fragment: the register unchanged / an empty sum
        h_out[0] = mode == LAMPI_CSUM_CRC32 ? partial : 0u;
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
    const int rc = check_args(h_msg, msg_len, frag_len, k_first, k_count, h_out, mode, &done, partial);
    if (rc || done) return rc;
    if (!h_ring || slot_stride < frag_len) return (int)hipErrorInvalidValue;
    return (int)host_msg((const uint8_t *)h_msg, msg_len, frag_len, k_first, k_count, (uint8_t *)h_ring, slot_stride,
                         partial, h_out, mode);
}

}  // extern "C"
