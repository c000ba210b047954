// lampi_csum.cc -- C ABI of liblampi_csum.so (see include/lampi_csum.h).
//
// Device entry points validate their arguments, make sure the per-device table image
// exists, and launch the gfx950 kernels on the caller's stream.  Host entry points (the
// drop-ins for uicrc/bcopy_uicrc/uicsum/bcopy_uicsum) run the same kernels: the bytes go
// to the GPU, the GPU computes, the checksum (and, for bcopy, the copied bytes) comes back.
// There is no CPU checksum path in this library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/lampi_csum.h"
#include "crc_tables.h"
#include "frag_csum_kernels.h"
#include "host_internal.h"

namespace lampi {
namespace {

constexpr int kMaxDevices = 64;

struct DeviceTables {
    std::once_flag once;
    uint32_t *img = nullptr;
    hipError_t err = hipSuccess;
};
DeviceTables g_tables[kMaxDevices];


// The table image is built on the host (GF(2) algebra, crc_tables.cc) once per process and
// uploaded once per device; kernels stage it into LDS.
const std::vector<uint32_t> &host_image() {
    static const std::vector<uint32_t> img = build_table_image();
    return img;
}

std::atomic<int64_t> g_pinned_bytes{0};

}  // namespace

hipError_t current_device(int *dev) {
    hipError_t e = hipGetDevice(dev);
    if (e != hipSuccess) return e;
    if (*dev < 0 || *dev >= kMaxDevices) return hipErrorInvalidDevice;
    return hipSuccess;
}

hipError_t device_tables(int dev, const uint32_t **out) {
    DeviceTables &t = g_tables[dev];
    std::call_once(t.once, [&] {
        const std::vector<uint32_t> &h = host_image();
        uint32_t *p = nullptr;
        t.err = hipMalloc(&p, h.size() * sizeof(uint32_t));
        if (t.err == hipSuccess) t.err = hipMemcpy(p, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
        if (t.err == hipSuccess) t.img = p;
    });
    *out = t.img;
    return t.err;
}

hipError_t launch_msg_csum(const uint8_t *base, size_t msg_len, size_t frag_len, uint32_t partial, uint32_t *out,
                           int mode, int dev, const uint32_t *img, hipStream_t s) {
    const size_t n = msg_len ? (msg_len + frag_len - 1) / frag_len : 1;
    const int grid = crc_grid(dev);
    if (mode == LAMPI_CSUM_SUM32) return launch_sum_msg(base, msg_len, frag_len, n, out, img, grid, s);
    const bool regular = msg_len != 0 && frag_len % kRowBytes == 0 && msg_len % frag_len == 0 &&
                         regular_msg_frag(frag_len, false) && ((uintptr_t)base & 15u) == 0 &&
                         !crc_light_msg(frag_len, msg_len);
    if (regular) return launch_crc_regular(base, n, frag_len, partial, out, img, grid, s);
    return launch_crc_msg(base, msg_len, frag_len, partial, n, out, img, grid, s);
}

hipError_t pinned_alloc(void **p, size_t bytes, unsigned flags) {
    const hipError_t e = hipHostMalloc(p, bytes, flags);
    if (e == hipSuccess) g_pinned_bytes.fetch_add((int64_t)bytes, std::memory_order_relaxed);
    return e;
}

void pinned_free(void *p, size_t bytes) {
    if (!p) return;
    (void)hipHostFree(p);
    g_pinned_bytes.fetch_sub((int64_t)bytes, std::memory_order_relaxed);
}

[[noreturn]] void die(const char *what, hipError_t e) {
    std::fprintf(stderr, "liblampi_csum: %s failed: %s (%d); no CPU fallback exists\n", what,
                 hipGetErrorString(e), (int)e);
    std::abort();
}

namespace {

int to_int(hipError_t e) { return (int)e; }

// ------------------------------------------------------------------ host-path context

#define LAMPI_CHECK(call)                      \
    do {                                       \
        hipError_t e_ = (call);                \
        if (e_ != hipSuccess) die(#call, e_);  \
    } while (0)

// Per-thread staging for the synchronous host entry points: a stream, device buffers and a
// pinned host bounce buffer on the thread's current device.  Everything is released when the
// thread exits (thread_local destructor -- LA-MPI progress threads come and go), when the
// thread switches devices (the buffers belong to the old one), and on lampi_host_release().
constexpr size_t kBounceHalf = 4u << 20;  // pinned bounce buffer: two halves (ping-pong pieces)
// Calls of up to kZeroCopy bytes skip the DMA engines: the bytes are copied into a host-coherent
// pinned buffer the kernels read directly over PCIe, the descriptors are read from pinned memory
// too and the result is written straight to pinned memory -- one kernel launch (two for SUM or a
// CRC of more than one piece) and one synchronize per call instead of three DMA round trips.
constexpr size_t kZeroCopy = 256u << 10;
constexpr uint64_t kPieceMin = 64 * 1024;  // host path: bytes per fragment piece
constexpr uint32_t kMaxPieces = 16384;     // combine kernel capacity (LDS ping-pong)
constexpr size_t kResBytes = 8 * sizeof(uint64_t);
constexpr size_t kDescBytes = kMaxPieces * sizeof(lampi_frag_desc);
constexpr size_t kZpinBytes = kZeroCopy + 64;  // + slack: aligned word reads past a body (uicsum)

struct HostCtx {
    int dev = -1;
    hipStream_t stream = nullptr;
    hipEvent_t half_free[2] = {nullptr, nullptr};  // the last transfer through each bounce half
    uint8_t *pin = nullptr;                       // 2 x kBounceHalf pinned bytes (first call > kZeroCopy)
    uint64_t *pres = nullptr;                     // pinned, host-coherent result words (4 x u64) + signal word
    uint64_t seq = 0;                             // the last signal value asked for (wait_done)
    uint8_t *zpin = nullptr;                      // pinned, host-coherent staging of small calls
    uint8_t *zpin_d = nullptr;                    // ... and the device's view of it,
    uint64_t *pres_d = nullptr;                   //     of pres
    lampi_frag_desc *hdesc_d = nullptr;           //     and of hdesc
    uint8_t *dbuf = nullptr;
    size_t dcap = 0;
    uint32_t *dvals = nullptr;  // per-piece checksums + 4 result words
    size_t vcap = 0;
    lampi_frag_desc *ddesc = nullptr;
    size_t desccap = 0;
    uint64_t *dvals64 = nullptr;  // 64-bit csum: per-piece sums + 3 result words
    size_t v64cap = 0;
    lampi_frag_desc *hdesc = nullptr;             // pinned piece descriptors (kMaxPieces)
    std::map<uint64_t, uint32_t *> combine_tabs;  // piece size -> device nibble tables

    HostCtx() = default;
    HostCtx(const HostCtx &) = delete;
    HostCtx &operator=(const HostCtx &) = delete;
    ~HostCtx() { release(); }

    // Free every resource on the device it was made on; errors are ignored (this also runs at
    // thread exit, where there is nobody to report them to).
    void release() {
        if (dev < 0) return;
        int cur = -1;
        const bool have_cur = hipGetDevice(&cur) == hipSuccess;
        if (have_cur && cur != dev) (void)hipSetDevice(dev);
        if (stream) (void)hipStreamSynchronize(stream);
        if (dbuf) (void)hipFree(dbuf);
        if (dvals) (void)hipFree(dvals);
        if (ddesc) (void)hipFree(ddesc);
        if (dvals64) (void)hipFree(dvals64);
        for (auto &kv : combine_tabs) (void)hipFree(kv.second);
        pinned_free(pin, 2 * kBounceHalf);
        pinned_free(pres, kResBytes);
        pinned_free(hdesc, kDescBytes);
        pinned_free(zpin, kZpinBytes);
        for (hipEvent_t &e : half_free)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
        if (have_cur && cur != dev) (void)hipSetDevice(cur);
        dev = -1;
        seq = 0;
        stream = nullptr;
        half_free[0] = half_free[1] = nullptr;
        pin = nullptr;
        pres = nullptr;
        dbuf = nullptr;
        dvals = nullptr;
        ddesc = nullptr;
        dvals64 = nullptr;
        dcap = vcap = desccap = v64cap = 0;
        hdesc = nullptr;
        zpin = zpin_d = nullptr;
        pres_d = nullptr;
        hdesc_d = nullptr;
        combine_tabs.clear();
    }
};

thread_local HostCtx t_ctx;

constexpr int kSignalWord = 7;  // pres[7]: the sequence number wait_done polls for

HostCtx &host_ctx() {
    HostCtx &ctx = t_ctx;
    int dev = 0;
    LAMPI_CHECK(current_device(&dev));
    if (ctx.dev != dev) {
        ctx.release();  // device changed (or first use): the old buffers belong to the old device
        ctx.dev = dev;
        LAMPI_CHECK(hipStreamCreateWithFlags(&ctx.stream, hipStreamNonBlocking));
        for (hipEvent_t &e : ctx.half_free) LAMPI_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        // the 8 MiB bounce buffer waits for the first call above kZeroCopy (bounce()): threads
        // that only make small calls stay cheap to create and tear down
        constexpr unsigned kCoherent = hipHostMallocMapped | hipHostMallocCoherent;
        LAMPI_CHECK(pinned_alloc((void **)&ctx.pres, kResBytes, kCoherent));
        ctx.pres[kSignalWord] = ctx.seq = 0;
        LAMPI_CHECK(pinned_alloc((void **)&ctx.hdesc, kDescBytes, kCoherent));
        LAMPI_CHECK(pinned_alloc((void **)&ctx.zpin, kZpinBytes, kCoherent));
        LAMPI_CHECK(hipHostGetDevicePointer((void **)&ctx.zpin_d, ctx.zpin, 0));
        LAMPI_CHECK(hipHostGetDevicePointer((void **)&ctx.pres_d, ctx.pres, 0));
        LAMPI_CHECK(hipHostGetDevicePointer((void **)&ctx.hdesc_d, ctx.hdesc, 0));
    }
    return ctx;
}

template <class T>
void ensure(T *&p, size_t &cap, size_t n) {
    if (cap >= n) return;
    if (p) LAMPI_CHECK(hipFree(p));
    p = nullptr;
    size_t c = std::max(n, cap * 2);
    LAMPI_CHECK(hipMalloc(&p, c * sizeof(T)));
    cap = c;
}


uint64_t piece_size(uint64_t len) {
    uint64_t b = (len + kMaxPieces - 1) / kMaxPieces;
    b = (b + 4095) / 4096 * 4096;
    return std::max<uint64_t>(b, kPieceMin);
}

uint32_t next_pow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// normal-domain nibble tables of shift by B * 2^lvl, lvl = 0..13
uint32_t *combine_tables(HostCtx &c, uint64_t B) {
    auto it = c.combine_tabs.find(B);
    if (it != c.combine_tabs.end()) return it->second;
    std::vector<uint32_t> h(14 * 128);
    Gf2Mat m = shift_matrix(B);
    for (int lvl = 0; lvl < 14; ++lvl) {
        nibble_tables(m, &h[lvl * 128]);
        m = mat_mul(m, m);
    }
    uint32_t *d = nullptr;
    LAMPI_CHECK(hipMalloc(&d, h.size() * sizeof(uint32_t)));
    LAMPI_CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    c.combine_tabs[B] = d;
    return d;
}

// The staged bytes of a host call: small calls in the host-coherent pinned buffer (read by the
// kernels over PCIe), larger ones DMA'd into c.dbuf through the bounce buffer.
struct Staged {
    const uint8_t *base;  // device address of the bytes
    bool zero_copy;
};

// Piece descriptors for the kernels: zero-copy calls hand the kernels the pinned array itself.
const lampi_frag_desc *upload_descs(HostCtx &c, uint32_t n, bool zero_copy) {
    if (zero_copy) return c.hdesc_d;
    ensure(c.ddesc, c.desccap, std::max<uint32_t>(n, 1));
    LAMPI_CHECK(hipMemcpyAsync(c.ddesc, c.hdesc, n * sizeof(lampi_frag_desc), hipMemcpyHostToDevice, c.stream));
    return c.ddesc;
}

// Wait for the call's kernels.  A zero-copy call (at most 256 KiB, a few microseconds of device
// work) gets a sequence number that its last kernel stores into host-coherent pinned memory once
// the results are out (signal_host, system scope), and the host polls for it: a tiny kernel's
// round trip is 6.4 us that way against 10.9 us through hipStreamSynchronize's wake-up
// (tools/microbench/sync_latency.hip, profiles/r02_sync_latency.txt).  No signal within 5 ms, or
// a larger call (seq 0), waits in hipStreamSynchronize, which also reports errors.
uint64_t next_signal(HostCtx &c, const Staged &st) { return st.zero_copy ? ++c.seq : 0u; }
uint64_t *signal_word(HostCtx &c, uint64_t seq) { return seq ? c.pres_d + kSignalWord : nullptr; }

void wait_done(HostCtx &c, uint64_t seq) {
    if (seq) {
        const uint64_t *sig = c.pres + kSignalWord;
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t i = 0; __atomic_load_n(sig, __ATOMIC_ACQUIRE) != seq; ++i) {
            __builtin_ia32_pause();
            if ((i & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(5)) break;
        }
        if (__atomic_load_n(sig, __ATOMIC_ACQUIRE) == seq) return;
    }
    LAMPI_CHECK(hipStreamSynchronize(c.stream));
}

// CRC of the staged bytes [0, len) from register `partial`, computed on the GPU; the result is
// written by the last kernel straight into pinned host memory.
uint32_t device_crc(HostCtx &c, const Staged &st, uint64_t len, uint32_t partial) {
    const uint32_t *img = nullptr;
    LAMPI_CHECK(device_tables(c.dev, &img));
    const int grid = crc_grid(c.dev);
    // zero-copy calls above 8 KiB: 4 KiB pieces folded by the combine kernel (one piece per row:
    // the piece-stream kernel then joins no fragment across its chains, whose serial join of a
    // 64 KiB piece cost ~20 us); otherwise pieces of piece_size
    const uint64_t B = (st.zero_copy && len > 8192) ? 4096 : piece_size(len);
    const uint32_t n = (uint32_t)((len + B - 1) / B);
    // pieces of the front-padded message: piece 0 holds the first len - (n-1)*B bytes
    const uint64_t first = len - (uint64_t)(n - 1) * B;
    for (uint32_t k = 0; k < n; ++k) {
        const uint64_t off = k == 0 ? 0 : first + (uint64_t)(k - 1) * B;
        c.hdesc[k].addr = (uint64_t)(uintptr_t)(st.base + off);
        c.hdesc[k].length = (uint32_t)(k == 0 ? first : B);
        c.hdesc[k].partial = k == 0 ? partial : 0u;
    }
    uint32_t *res = (uint32_t *)c.pres_d;
    const uint64_t seq = next_signal(c, st);
    if (n == 1 && st.zero_copy) {  // the piece by value; its kernel signals
        LAMPI_CHECK(launch_host_one(st.base, (uint32_t)len, partial, res, LAMPI_CSUM_CRC32, img, c.stream,
                                    signal_word(c, seq), seq));
    } else if (n == 1) {
        LAMPI_CHECK(launch_crc_desc(upload_descs(c, 1, false), 1, res, img, grid, c.stream, false, 1u));
    } else {
        ensure(c.dvals, c.vcap, (size_t)n + 4);
        // (rows hint 1: pieces sized for the count split, not a small batch of unknown fragments)
        LAMPI_CHECK(launch_crc_desc(upload_descs(c, n, st.zero_copy), n, c.dvals, img, grid, c.stream, false, 1u));
        LAMPI_CHECK(launch_crc_combine(c.dvals, n, combine_tables(c, B), next_pow2(n), res, c.stream,
                                       signal_word(c, seq), seq));
    }
    wait_done(c, seq);
    return ((const volatile uint32_t *)c.pres)[0];
}

// uicsum of the staged bytes [0, len) with chaining state, computed on the GPU.
uint32_t device_sum(HostCtx &c, const Staged &st, uint64_t len, unsigned int *pint, unsigned int *plen) {
    const int grid = crc_grid(c.dev);
    const uint32_t k = *plen >= 4 ? 0u : *plen;
    const uint64_t head = k ? std::min<uint64_t>(4 - k, len) : 0;
    const uint64_t body = (len - head) & ~3ull;
    const uint64_t B = piece_size(body ? body : 1);
    const uint32_t n = (uint32_t)((body + B - 1) / B);
    for (uint32_t i = 0; i < n; ++i) {
        c.hdesc[i].addr = (uint64_t)(uintptr_t)(st.base + head + (uint64_t)i * B);
        c.hdesc[i].length = (uint32_t)std::min<uint64_t>(B, body - (uint64_t)i * B);
        c.hdesc[i].partial = 0;
    }
    ensure(c.dvals, c.vcap, (size_t)n + 4);
    uint32_t *out3 = (uint32_t *)c.pres_d;
    const uint64_t seq = next_signal(c, st);
    if (st.zero_copy) {  // one kernel sums the body, completes the state and signals
        LAMPI_CHECK(launch_sum_finish(nullptr, 0, st.base, len, *pint, *plen, out3, c.stream, signal_word(c, seq), seq));
        wait_done(c, seq);
        const volatile uint32_t *h = (const volatile uint32_t *)c.pres;
        *pint = h[1];
        *plen = h[2];
        return h[0];
    }
    if (n) {
        const lampi_frag_desc *d = upload_descs(c, n, st.zero_copy);
        LAMPI_CHECK(launch_sum_desc(d, n, c.dvals, nullptr, grid, c.stream, false, 1u));
    }
    LAMPI_CHECK(launch_sum_finish(c.dvals, n, st.base, len, *pint, *plen, out3, c.stream, signal_word(c, seq), seq));
    wait_done(c, seq);
    const volatile uint32_t *h = (const volatile uint32_t *)c.pres;
    *pint = h[1];
    *plen = h[2];
    return h[0];
}

// csum (64-bit words) of the staged bytes [0, len) with chaining state, computed on the GPU:
// every piece is summed at its byte phase in the caller's word grid, the finish kernel adds them
// up and forms the new trailing partial word.
uint64_t device_sum64(HostCtx &c, const Staged &st, uint64_t len, unsigned long *plong, unsigned long *plen) {
    const uint64_t k = *plen >= 8 ? 0u : *plen;
    const uint64_t B = piece_size(len);
    const uint32_t n = (uint32_t)((len + B - 1) / B);
    for (uint32_t i = 0; i < n; ++i) {
        c.hdesc[i].addr = (uint64_t)(uintptr_t)(st.base + (uint64_t)i * B);
        c.hdesc[i].length = (uint32_t)std::min<uint64_t>(B, len - (uint64_t)i * B);
        c.hdesc[i].partial = (uint32_t)((k + (uint64_t)i * B) & 7u);
    }
    ensure(c.dvals64, c.v64cap, (size_t)n + 3);
    const lampi_frag_desc *d = upload_descs(c, n, st.zero_copy);
    LAMPI_CHECK(launch_sum64_desc(d, n, c.dvals64, true, c.stream));
    uint64_t *out3 = c.pres_d;
    const uint64_t seq = next_signal(c, st);
    LAMPI_CHECK(launch_sum64_finish(c.dvals64, n, st.base, len, k ? (uint64_t)*plong : 0u, k, out3, c.stream,
                                    signal_word(c, seq), seq));
    wait_done(c, seq);
    const volatile uint64_t *h = (const volatile uint64_t *)c.pres;
    *plong = (unsigned long)h[1];
    *plen = (unsigned long)h[2];
    return h[0];
}

unsigned long empty_sum64(unsigned long *plong, unsigned long *plen) {
    if (*plen == 0 || *plen >= 8) {
        *plong = 0;
        *plen = 0;
    }
    return 0;
}

// The pinned bounce buffer, allocated on the thread's first call above kZeroCopy.
void bounce(HostCtx &c) {
    if (!c.pin) LAMPI_CHECK(pinned_alloc((void **)&c.pin, 2 * kBounceHalf, hipHostMallocDefault));
}

// host -> c.dbuf through the pinned bounce buffer: pieces of kBounceHalf bytes alternate between
// its two halves; a half is refilled once its previous DMA has completed (event), so the CPU
// copy of one piece overlaps the DMA of the other.
Staged stage_in(HostCtx &c, const void *src, uint64_t len) {
    if (len <= kZeroCopy) {
        std::memcpy(c.zpin, src, (size_t)len);
        return {c.zpin_d, true};
    }
    ensure(c.dbuf, c.dcap, (size_t)len);
    bounce(c);
    const uint8_t *s = (const uint8_t *)src;
    for (uint64_t off = 0, i = 0; off < len; off += kBounceHalf, ++i) {
        const size_t n = (size_t)std::min<uint64_t>(kBounceHalf, len - off);
        uint8_t *half = c.pin + (i & 1) * kBounceHalf;
        LAMPI_CHECK(hipEventSynchronize(c.half_free[i & 1]));
        std::memcpy(half, s + off, n);
        LAMPI_CHECK(hipMemcpyAsync(c.dbuf + off, half, n, hipMemcpyHostToDevice, c.stream));
        LAMPI_CHECK(hipEventRecord(c.half_free[i & 1], c.stream));
    }
    return {c.dbuf, false};
}

// c.dbuf -> host through the bounce buffer: the DMA of piece i+1 runs while piece i is copied out
// the copy half of a host bcopy: the bytes the GPU checksummed, from the staging buffer they sit
// in (the pinned buffer of a zero-copy call; c.dbuf, DMA'd back, otherwise)
void stage_out(HostCtx &c, const Staged &st, void *dst, uint64_t len) {
    if (!len) return;
    if (st.zero_copy) {
        std::memcpy(dst, c.zpin, (size_t)len);
        return;
    }
    bounce(c);
    uint8_t *d = (uint8_t *)dst;
    const uint64_t np = (len + kBounceHalf - 1) / kBounceHalf;
    auto issue = [&](uint64_t i) {
        const uint64_t off = i * kBounceHalf;
        const size_t n = (size_t)std::min<uint64_t>(kBounceHalf, len - off);
        LAMPI_CHECK(hipMemcpyAsync(c.pin + (i & 1) * kBounceHalf, c.dbuf + off, n, hipMemcpyDeviceToHost, c.stream));
        LAMPI_CHECK(hipEventRecord(c.half_free[i & 1], c.stream));
    };
    issue(0);
    for (uint64_t i = 0; i < np; ++i) {
        if (i + 1 < np) issue(i + 1);  // the other half: free, its last use was copied out below
        LAMPI_CHECK(hipEventSynchronize(c.half_free[i & 1]));
        const uint64_t off = i * kBounceHalf;
        std::memcpy(d + off, c.pin + (i & 1) * kBounceHalf, (size_t)std::min<uint64_t>(kBounceHalf, len - off));
    }
}

// zero-length uicsum: no bytes, only the state convention of the reference
// (MemFunctions.cc:1073-1222: an aligned state is reset to (0,0), a partial one is kept)
uint32_t empty_sum(unsigned int *pint, unsigned int *plen) {
    if (*plen == 0 || *plen >= 4) {
        *pint = 0;
        *plen = 0;
    }
    return 0;
}

}  // namespace
}  // namespace lampi

using namespace lampi;

extern "C" {

unsigned int lampi_uicrc(const void *src, unsigned long crclen, unsigned int partial_crc) {
    if (crclen == 0) return partial_crc;  // no bytes: the register is unchanged
    HostCtx &c = host_ctx();
    const Staged st = stage_in(c, src, crclen);
    return device_crc(c, st, crclen, partial_crc);
}

unsigned int lampi_bcopy_uicrc(const void *src, void *dst, unsigned long copylen, unsigned long crclen,
                               unsigned int partial_crc) {
    const uint64_t n = std::max<uint64_t>(copylen, crclen);
    if (n == 0) return partial_crc;
    HostCtx &c = host_ctx();
    const Staged st = stage_in(c, src, n);
    const uint32_t r = device_crc(c, st, n, partial_crc);
    stage_out(c, st, dst, copylen);
    return r;
}

unsigned int lampi_uicsum(const void *src, unsigned long csumlen, unsigned int *pint, unsigned int *plen) {
    if (csumlen == 0) return empty_sum(pint, plen);
    HostCtx &c = host_ctx();
    const Staged st = stage_in(c, src, csumlen);
    return device_sum(c, st, csumlen, pint, plen);
}

unsigned int lampi_bcopy_uicsum(const void *src, void *dst, unsigned long copylen, unsigned long csumlen,
                                unsigned int *pint, unsigned int *plen) {
    const uint64_t n = std::max<uint64_t>(copylen, csumlen);
    if (n == 0) return empty_sum(pint, plen);
    HostCtx &c = host_ctx();
    const Staged st = stage_in(c, src, n);
    const uint32_t r = device_sum(c, st, n, pint, plen);
    stage_out(c, st, dst, copylen);
    return r;
}

unsigned long lampi_csum(const void *src, unsigned long csumlen, unsigned long *plong, unsigned long *plen) {
    if (csumlen == 0) return empty_sum64(plong, plen);
    HostCtx &c = host_ctx();
    const Staged st = stage_in(c, src, csumlen);
    return device_sum64(c, st, csumlen, plong, plen);
}

unsigned long lampi_bcopy_csum(const void *src, void *dst, unsigned long copylen, unsigned long csumlen,
                               unsigned long *plong, unsigned long *plen) {
    const uint64_t n = std::max<uint64_t>(copylen, csumlen);
    if (n == 0) return empty_sum64(plong, plen);
    HostCtx &c = host_ctx();
    const Staged st = stage_in(c, src, n);
    const uint64_t r = device_sum64(c, st, n, plong, plen);
    stage_out(c, st, dst, copylen);
    return r;
}

int lampi_frag_csum64_batch(const lampi_frag_desc *d_descs, size_t n, uint64_t *d_out, void *stream) {
    if (n == 0) return 0;
    if (!d_descs || !d_out) return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_sum64_desc(d_descs, n, d_out, false, (hipStream_t)stream));
}

int lampi_frag_csum_batch(const lampi_frag_desc *d_descs, size_t n, uint32_t *d_out, int mode, void *stream) {
    const bool by_bytes = (mode & LAMPI_CSUM_BY_BYTES) != 0;
    // (0: no hint -- small batches then run as row groups; 1: the caller's one-row hint keeps the count split)
    const uint32_t rows_hint = LAMPI_CSUM_ROWS_HINT_OF(mode);
    mode &= ~(LAMPI_CSUM_BY_BYTES | LAMPI_CSUM_ROWS_HINT_MASK);
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32) return to_int(hipErrorInvalidValue);
    if (n == 0) return 0;
    if (!d_descs || !d_out) return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    if (mode == LAMPI_CSUM_SUM32)
        return to_int(launch_sum_desc(d_descs, n, d_out, img, crc_grid(dev), s, by_bytes, rows_hint));
    return to_int(launch_crc_desc(d_descs, n, d_out, img, crc_grid(dev), s, by_bytes, rows_hint));
}

// Internal diagnostic (not in include/lampi_csum.h): the read-only CRC piece-stream kernel's timeline,
// 8 u64 per workgroup into d_stamps (tools/microbench/stream_timeline.py).  Returns the workgroup count
// or a negative hipError_t.
int lampi_diag_stream_timeline(const lampi_frag_desc *d_descs, size_t n, uint32_t *d_out, uint64_t *d_stamps,
                               void *stream) {
    if (n == 0 || !d_descs || !d_out || !d_stamps) return -to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return -to_int(e);
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return -to_int(e);
    uint32_t nwg = 0;
    e = diag_stream_timeline(d_descs, n, d_out, img, d_stamps, (hipStream_t)stream, &nwg);
    return e != hipSuccess ? -to_int(e) : (int)nwg;
}

// Internal diagnostic (not in include/lampi_csum.h): config B's kernel's timeline on a read-only CRC message of n 4 KiB
// fragments at d_base (n even), 16 u64 per workgroup into d_stamps (tools/microbench/regular_timeline.py).  Returns
// the workgroup count or a negative hipError_t.
int lampi_diag_regular_timeline(const void *d_base, size_t n, uint32_t *d_out, uint64_t *d_stamps, void *stream) {
    if (n == 0 || !d_base || !d_out || !d_stamps) return -to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return -to_int(e);
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return -to_int(e);
    uint32_t nwg = 0;
    e = diag_regular_timeline((const uint8_t *)d_base, n, d_out, img, d_stamps, (hipStream_t)stream, &nwg);
    return e != hipSuccess ? -to_int(e) : (int)nwg;
}

// Internal diagnostic (retired from include/lampi_csum.h in round 5): lampi_frag_csum_batch's
// results on the north_star's baseline schedule, one wavefront walking each fragment's 4 KiB rows
// (crc_rows_kernel / sum_rows_kernel) -- kept for bench.py's config C comparison and the parity tests only.
int lampi_diag_frag_csum_batch_per_wave(const lampi_frag_desc *d_descs, size_t n, uint32_t *d_out, int mode,
                                        void *stream) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32) return to_int(hipErrorInvalidValue);
    if (n == 0) return 0;
    if (!d_descs || !d_out) return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_desc_per_wave(d_descs, n, d_out, mode, img, (hipStream_t)stream));
}

}  // extern "C"

namespace {
// A strided output (d_out 4-byte aligned, out_stride a multiple of 4 and >= 4) is valid for n words.
bool strided_ok(const void *d_out, size_t out_stride, size_t n) {
    return d_out && !((uintptr_t)d_out & 3u) && !(out_stride & 3u) && out_stride >= 4 && n <= 0xFFFFFFFFull;
}

// Runs batch(vals) -- a launch writing n checksum words to vals -- and puts word i at d_out + i*out_stride:
// straight into d_out when out_stride is 4, otherwise into stream-ordered scratch and then one 4-byte scatter
// (the send side's dataChecksum @64 of each 72-byte gmHeaderData record: d_out = hdrs + 64, out_stride = the
// buffer size).  d_out == nullptr: the words are discarded (the copies with checksumming off).
template <class F>
int with_out(size_t n, void *d_out, size_t out_stride, hipStream_t s, F &&batch) {
    if (d_out && out_stride == 4) return batch((uint32_t *)d_out);
    uint32_t *vals = nullptr;
    hipError_t e = hipMallocAsync((void **)&vals, std::max<size_t>(n, 1) * sizeof(uint32_t), s);
    if (e != hipSuccess) return to_int(e);
    int r = batch(vals);
    if (r == 0 && d_out) r = to_int(launch_scatter_u32(vals, n, (uint8_t *)d_out, out_stride, s));
    const hipError_t f = hipFreeAsync(vals, s);
    return r != 0 ? r : to_int(f);
}
}  // namespace

extern "C" {

int lampi_frag_csum_batch_strided(const lampi_frag_desc *d_descs, size_t n, void *d_out, size_t out_stride, int mode,
                                  void *stream) {
    const int base_mode = mode & ~(LAMPI_CSUM_BY_BYTES | LAMPI_CSUM_ROWS_HINT_MASK);
    if (base_mode != LAMPI_CSUM_CRC32 && base_mode != LAMPI_CSUM_SUM32) return to_int(hipErrorInvalidValue);
    if (n == 0) return 0;
    if (!d_descs || !strided_ok(d_out, out_stride, n)) return to_int(hipErrorInvalidValue);
    return with_out(n, d_out, out_stride, (hipStream_t)stream,
                    [&](uint32_t *vals) { return lampi_frag_csum_batch(d_descs, n, vals, mode, stream); });
}

int lampi_frag_bcopy_batch_strided(const lampi_copy_desc *d_descs, size_t n, void *d_out, size_t out_stride, int mode,
                                   void *stream) {
    const uint32_t rows_hint = std::max(1u, LAMPI_CSUM_ROWS_HINT_OF(mode));
    const int base_mode = mode & ~LAMPI_CSUM_ROWS_HINT_MASK;
    if (base_mode != LAMPI_CSUM_CRC32 && base_mode != LAMPI_CSUM_SUM32 && base_mode != LAMPI_CSUM_NONE)
        return to_int(hipErrorInvalidValue);
    const bool none = base_mode == LAMPI_CSUM_NONE;  // (d_out unused: may be NULL)
    if (n == 0) return 0;
    if (!d_descs || (!none && !strided_ok(d_out, out_stride, n)) || n > 0xFFFFFFFFull)
        return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;  // CRC: the tables
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    hipStream_t s = (hipStream_t)stream;
    return with_out(n, none ? nullptr : d_out, out_stride, s, [&](uint32_t *vals) {
        return to_int(launch_bcopy_desc(d_descs, n, vals, base_mode, img, s, rows_hint));
    });
}

int lampi_frag_bcopy_batch(const lampi_copy_desc *d_descs, size_t n, uint32_t *d_out, int mode, void *stream) {
    return lampi_frag_bcopy_batch_strided(d_descs, n, d_out, sizeof(uint32_t), mode, stream);
}

int lampi_copy_to_app_batch(const lampi_recv_desc *d_descs, size_t n, const void *d_expected, size_t expected_stride,
                            int64_t *d_copied, uint32_t *d_csum, uint32_t *d_mask, uint32_t *d_nbad, int mode,
                            void *stream) {
    const uint32_t rows_hint = std::max(1u, LAMPI_CSUM_ROWS_HINT_OF(mode));
    mode &= ~LAMPI_CSUM_ROWS_HINT_MASK;
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32 && mode != LAMPI_CSUM_NONE)
        return to_int(hipErrorInvalidValue);
    const bool check = mode != LAMPI_CSUM_NONE;  // (checksumming off: no expected values read)
    if (!d_nbad || (n && (!d_descs || (check && !d_expected) || !d_copied || !d_csum || !d_mask)) ||
        ((uintptr_t)d_expected & 3u) || (expected_stride & 3u) || n > 0xFFFFFFFFull)
        return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;  // CRC: the tables
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_copy_to_app(d_descs, n, (const uint8_t *)d_expected, expected_stride, d_copied, d_csum, d_mask,
                                     d_nbad, mode, img, (hipStream_t)stream, rows_hint));
}

int lampi_msg_csum(const void *d_msg, size_t msg_len, size_t frag_len, uint32_t partial, uint32_t *d_out, int mode,
                   void *stream) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32) return to_int(hipErrorInvalidValue);
    if (frag_len == 0 || frag_len > 0xFFFFFFFFull || !d_out || (msg_len && !d_msg))
        return to_int(hipErrorInvalidValue);
    // a zero-length message is one empty fragment (the path layer still sends a header)
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_msg_csum((const uint8_t *)d_msg, msg_len, frag_len, partial, d_out, mode, dev, img,
                                  (hipStream_t)stream));
}

int lampi_msg_bcopy_strided(const void *d_msg, size_t msg_len, size_t frag_len, void *d_dst, size_t dst_stride,
                            uint32_t partial, void *d_out, size_t out_stride, int mode, void *stream) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32 && mode != LAMPI_CSUM_NONE)
        return to_int(hipErrorInvalidValue);
    const bool none = mode == LAMPI_CSUM_NONE;  // (d_out unused: may be NULL)
    const size_t n = frag_len && msg_len ? (msg_len + frag_len - 1) / frag_len : 1;
    if (frag_len == 0 || frag_len > 0xFFFFFFFFull || dst_stride < frag_len || (!none && !strided_ok(d_out, out_stride, n)) ||
        (msg_len && (!d_msg || !d_dst)))
        return to_int(hipErrorInvalidValue);
    if (none && msg_len == 0) return 0;  // (nothing to copy, no checksum)
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;  // CRC: the tables
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    hipStream_t s = (hipStream_t)stream;
    // checksumming off: the SUM copy schedules (every byte copied is read once; the sums are discarded)
    return with_out(n, none ? nullptr : d_out, out_stride, s, [&](uint32_t *vals) {
        return to_int(launch_msg_bcopy((const uint8_t *)d_msg, msg_len, frag_len, partial, (uint8_t *)d_dst, dst_stride,
                                       n, vals, none ? LAMPI_CSUM_SUM32 : mode, img, s));
    });
}

int lampi_msg_bcopy(const void *d_msg, size_t msg_len, size_t frag_len, void *d_dst, size_t dst_stride,
                    uint32_t partial, uint32_t *d_out, int mode, void *stream) {
    return lampi_msg_bcopy_strided(d_msg, msg_len, frag_len, d_dst, dst_stride, partial, d_out, sizeof(uint32_t), mode,
                                   stream);
}

int lampi_chain_csum_batch_strided(const lampi_copy_desc *d_pieces, size_t npieces, const uint32_t *d_first,
                                   size_t nfrags, void *d_out, size_t out_stride, int mode, void *stream) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32 && mode != LAMPI_CSUM_NONE)
        return to_int(hipErrorInvalidValue);
    const bool none = mode == LAMPI_CSUM_NONE;  // (d_out unused: may be NULL)
    if (nfrags == 0) return 0;
    if (!d_first || (!none && !strided_ok(d_out, out_stride, nfrags)) || (npieces && !d_pieces) ||
        npieces > 0xFFFFFFFFull || nfrags > 0xFFFFFFFFull)
        return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    hipStream_t s = (hipStream_t)stream;
    uint32_t *scratch = nullptr;
    if (npieces) {
        e = hipMallocAsync((void **)&scratch, 2 * npieces * sizeof(uint32_t), s);
        if (e != hipSuccess) return to_int(e);
    }
    // (checksumming off: launch_chain copies and writes zeros, here into discarded scratch)
    int r = with_out(nfrags, none ? nullptr : d_out, out_stride, s, [&](uint32_t *vals) {
        return to_int(launch_chain(d_pieces, npieces, d_first, nfrags, vals, mode, img, scratch,
                                   scratch ? scratch + npieces : nullptr, s));
    });
    if (scratch) {
        const int f = to_int(hipFreeAsync(scratch, s));
        if (r == 0) r = f;
    }
    return r;
}

int lampi_chain_csum_batch(const lampi_copy_desc *d_pieces, size_t npieces, const uint32_t *d_first, size_t nfrags,
                           uint32_t *d_out, int mode, void *stream) {
    return lampi_chain_csum_batch_strided(d_pieces, npieces, d_first, nfrags, d_out, sizeof(uint32_t), mode, stream);
}

int lampi_chain_copy_to_app_batch(const lampi_copy_desc *d_pieces, size_t npieces, const uint32_t *d_first,
                                  size_t nfrags, const void *d_expected, size_t expected_stride, int64_t *d_copied,
                                  uint32_t *d_csum, uint32_t *d_mask, uint32_t *d_nbad, int mode, void *stream) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32 && mode != LAMPI_CSUM_NONE)
        return to_int(hipErrorInvalidValue);
    const bool check = mode != LAMPI_CSUM_NONE;
    if (!d_nbad) return to_int(hipErrorInvalidValue);
    hipStream_t s = (hipStream_t)stream;
    if (nfrags == 0) return to_int(hipMemsetAsync(d_nbad, 0, sizeof(uint32_t), s));
    if (!d_first || !d_copied || !d_csum || !d_mask || (check && !d_expected) || (npieces && !d_pieces) ||
        ((uintptr_t)d_expected & 3u) || (expected_stride & 3u) || npieces > 0xFFFFFFFFull || nfrags > 0xFFFFFFFFull)
        return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    uint32_t *scratch = nullptr;
    if (npieces) {
        e = hipMallocAsync((void **)&scratch, 2 * npieces * sizeof(uint32_t), s);
        if (e != hipSuccess) return to_int(e);
    }
    ChainVerdict v;
    v.expected = (const uint8_t *)d_expected;
    v.exp_stride = expected_stride;
    v.copied = d_copied;
    v.mask = d_mask;
    v.nbad = d_nbad;
    v.init = 1;  // nonContigCopyFunction's first call starts from CRC_INITIAL_REGISTER
    e = launch_chain(d_pieces, npieces, d_first, nfrags, d_csum, mode, img, scratch,
                     scratch ? scratch + npieces : nullptr, s, &v);
    if (scratch) {
        const hipError_t f = hipFreeAsync(scratch, s);
        if (e == hipSuccess) e = f;
    }
    return to_int(e);
}

int lampi_header_csum_batch_strided(const void *d_hdrs, size_t n, size_t stride, uint32_t crclen, uint32_t word_count,
                                    void *d_out, size_t out_stride, int mode, void *stream) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32 && mode != LAMPI_CSUM_NONE)
        return to_int(hipErrorInvalidValue);
    if (mode == LAMPI_CSUM_NONE) return 0;  // no header checksum with checksumming off (gm/sendFrag.cc:219-225)
    if (n == 0) return 0;
    if (!d_hdrs || !strided_ok(d_out, out_stride, n) || ((uintptr_t)d_hdrs & 3u) || (stride & 3u))
        return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_header_csum((const uint8_t *)d_hdrs, n, stride, crclen, word_count, mode, img,
                                     (uint8_t *)d_out, out_stride, (hipStream_t)stream));
}

int lampi_header_csum_batch(const void *d_hdrs, size_t n, size_t stride, uint32_t crclen, uint32_t word_count,
                            uint32_t *d_out, int mode, void *stream) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32) return to_int(hipErrorInvalidValue);
    return lampi_header_csum_batch_strided(d_hdrs, n, stride, crclen, word_count, d_out, sizeof(uint32_t), mode,
                                           stream);
}

int lampi_header_check_batch(const void *d_hdrs, size_t n, size_t stride, uint32_t hdr_bytes, uint32_t word_count,
                             uint32_t csum_offset, uint32_t *d_mask, uint32_t *d_nbad, int mode, void *stream) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32) return to_int(hipErrorInvalidValue);
    if (!d_nbad || (n && (!d_hdrs || !d_mask)) || ((uintptr_t)d_hdrs & 3u) || (stride & 3u) || (csum_offset & 3u) ||
        n > 0xFFFFFFFFull)
        return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_header_check((const uint8_t *)d_hdrs, n, stride, hdr_bytes, word_count, csum_offset, mode,
                                      img, d_mask, d_nbad, (hipStream_t)stream));
}

int lampi_header_compare_batch(const void *d_hdrs, size_t n, size_t stride, uint32_t crclen, uint32_t csum_offset,
                               uint32_t *d_mask, uint32_t *d_nbad, int mode, void *stream) {
    if (mode != LAMPI_CSUM_CRC32 && mode != LAMPI_CSUM_SUM32) return to_int(hipErrorInvalidValue);
    if (!d_nbad || (n && (!d_hdrs || !d_mask)) || ((uintptr_t)d_hdrs & 3u) || (stride & 3u) || (csum_offset & 3u) ||
        n > 0xFFFFFFFFull)
        return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    const uint32_t *img = nullptr;
    e = device_tables(dev, &img);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_header_compare((const uint8_t *)d_hdrs, n, stride, crclen, csum_offset, mode, img, d_mask,
                                        d_nbad, (hipStream_t)stream));
}

int lampi_check_data_batch(const uint32_t *d_calc, const void *d_expected, size_t expected_stride,
                           const void *d_lengths, size_t lengths_stride, size_t n, uint32_t *d_mask, uint32_t *d_nbad,
                           void *stream) {
    if (!d_nbad || (n && (!d_calc || !d_expected || !d_mask)) || ((uintptr_t)d_expected & 3u) ||
        (expected_stride & 3u) || ((uintptr_t)d_lengths & 3u) || (lengths_stride & 3u) || n > 0xFFFFFFFFull)
        return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_check_data(d_calc, (const uint8_t *)d_expected, expected_stride, (const uint8_t *)d_lengths,
                                    lengths_stride, n, d_mask, d_nbad, (hipStream_t)stream));
}

int lampi_fill_stream(void *d_dst, size_t nbytes, uint64_t seed, uint64_t byte_off, void *stream) {
    if (nbytes == 0) return 0;
    if (!d_dst) return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_fill_stream((uint8_t *)d_dst, nbytes, seed, byte_off, crc_grid(dev), (hipStream_t)stream));
}

int lampi_fill_stream_frags(void *d_dst, size_t n, size_t frag_len, uint64_t seed, uint64_t k0, uint64_t kstep,
                            void *stream) {
    if (n == 0) return 0;
    if (!d_dst || frag_len == 0 || frag_len % 8 != 0 || ((uintptr_t)d_dst & 7u)) return to_int(hipErrorInvalidValue);
    int dev = 0;
    hipError_t e = current_device(&dev);
    if (e != hipSuccess) return to_int(e);
    return to_int(launch_fill_frags((uint64_t *)d_dst, n, frag_len / 8, seed, k0, kstep, crc_grid(dev),
                                    (hipStream_t)stream));
}

void lampi_host_release(void) {
    t_ctx.release();
    release_pipeline();
    release_thread_scratch();
}

int64_t lampi_host_pinned_bytes(void) { return g_pinned_bytes.load(std::memory_order_relaxed); }

int64_t lampi_device_scratch_bytes(void) { return device_scratch_bytes(); }

int lampi_host_register(void *h_ptr, size_t len) {
    if (!h_ptr || !len) return to_int(hipErrorInvalidValue);
    return to_int(hipHostRegister(h_ptr, len, hipHostRegisterDefault));
}

int lampi_host_unregister(void *h_ptr) {
    if (!h_ptr) return to_int(hipErrorInvalidValue);
    return to_int(hipHostUnregister(h_ptr));
}

const char *lampi_csum_version(void) { return "lampi-frag-csum 0.1 (gfx950, CDNA4)"; }

}  // extern "C"
