// host_pipe.h -- the per-thread H2D || kernel || D2H pipeline behind the host-memory paths of
// liblampi_csum.so (internal): the send side (host_msg.cc: lampi_host_msg_csum / _bcopy) and the
// receive side (host_recv.cc: lampi_host_copy_to_app_batch, the host header checks).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace lampi {

constexpr int kBufs = 3;  // device chunks in flight
// Payload bytes per chunk.  A call's time is about (chunks + 1) pipeline stages: the first chunk's H2D
// and the last one's D2H run alone.  Checksum-only calls (H2D only): 64 MiB chunks, 51.2-51.7 GiB/s
// for 256 MiB messages against 49.1-50.7 at 32 MiB and 45-48 at 16 MiB; calls moving bytes both ways
// (host_msg bcopy, the receive path): 32 MiB, bcopy 36.3-37.7 -> 39.9-40.2 GiB/s and receive 34.8-37.1
// -> 36.8-39.4 against 64 MiB; 16 MiB about the same as 32 for bcopy, noisier for receive; 8 MiB
// receive 16 GiB/s (profiles/r04/chunk_ab.txt, one box).
constexpr size_t kChunkTarget = 64u << 20;
constexpr size_t kChunkDuplex = 32u << 20;
// The chunk size for a call (duplex: it also moves bytes back); LAMPI_HOST_CHUNK_BYTES overrides it
// for A/B runs.
size_t chunk_target(bool duplex);
// Largest fragment the host paths take (a chunk holds whole fragments, so kBufs x this is the most
// staging HBM a call can ask for: 3 GiB of the 288 GB).  The transports' fragments are at most
// 64 KiB (GM), 2 KiB (IB); larger ones are refused with hipErrorInvalidValue.
constexpr size_t kHostMaxFrag = (size_t)1 << 30;

// Everything a thread's pipeline holds; a plain aggregate, so release() can reset it.
struct PipeState {
    int dev = -1;
    hipStream_t s_in = nullptr, s_k = nullptr, s_out = nullptr;
    hipEvent_t in_done[kBufs] = {}, k_done[kBufs] = {}, out_done[kBufs] = {};
    uint8_t *dchunk = nullptr;  // kBufs input chunks of chunk_bytes
    size_t chunk_bytes = 0;
    uint8_t *dout = nullptr;  // kBufs output chunks of out_bytes (receive: the app-bound bytes)
    size_t out_bytes = 0;
    uint8_t *dmeta = nullptr;  // a call's descriptors and results on the device
    size_t dmeta_cap = 0;
    uint8_t *hmeta = nullptr;  // ... and their pinned host image
    size_t hmeta_cap = 0;
};

// The calling thread's pipeline on its current device (created on first use; a device switch
// releases the old one first).
hipError_t pipe_ctx(PipeState **out);
// Grow-only capacities (a device buffer is replaced only after the streams drained).
hipError_t ensure_chunks(PipeState &p, size_t chunk);
hipError_t ensure_out_chunks(PipeState &p, size_t chunk);
hipError_t ensure_meta(PipeState &p, size_t bytes);

// Drains the pipeline's streams when a call leaves early: every error exit after the first
// enqueue leaves no copy or kernel in flight, so the next call may reuse the chunks at once and no
// DMA writes the caller's memory after the error was returned.
struct PipeDrain {
    PipeState &p;
    bool armed = true;
    explicit PipeDrain(PipeState &ps) : p(ps) {}
    PipeDrain(const PipeDrain &) = delete;
    PipeDrain &operator=(const PipeDrain &) = delete;
    ~PipeDrain() {
        if (!armed) return;
        for (hipStream_t s : {p.s_in, p.s_k, p.s_out})
            if (s) (void)hipStreamSynchronize(s);
    }
};

#define LAMPI_TRY(call)                             \
    do {                                            \
        const hipError_t e_ = (call);               \
        if (e_ != hipSuccess) return e_;            \
    } while (0)

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace lampi
