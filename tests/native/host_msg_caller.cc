// host_msg_caller.cc -- a native C++ caller of the host-memory message path
// (lampi_host_msg_csum / lampi_host_msg_bcopy, include/lampi_csum.h) in the shapes LA-MPI's send
// loop has (ref src/path/gm/path.cc:98-176, gm/sendFrag.cc:147-155; IB 1,976-byte payloads,
// src/path/ib/header.h:75; Quadrics checksum-only sends, src/path/quadrics/sendFrag.h:861-872):
// GM 65,456-byte payloads into 64 KiB buffers behind a 72-byte header, 4 KiB / 16 KiB fragments,
// a fragment larger than the pipeline's chunk, short last fragments, sub-ranges of fragments (the
// clear-to-send gating of gm/path.cc:104-118), page-locked and pageable sources and rings, both
// checksum modes, on two threads at once and then on the main thread after lampi_host_release().
//
// Every fragment's checksum is compared with the oracle (oracle/libcsum_ref.so, the
// reference-pinned CPU restatement -- test infrastructure), every slot's bytes with the source,
// and the bytes around the slots must keep their sentinel.  Prints one line per call and "done";
// exits 1 on any mismatch.  Build: make -C tests/native (after oracle/ and lampi_amd/).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "lampi_csum.h"
#include "../../oracle/csum_ref.h"

static std::mutex g_out;
static int g_bad = 0;

struct Shape {
    size_t frag_len, msg_len, gap;  // gap: ring bytes between payloads (header room), 0 = packed
};

static void report(const std::string &line, bool ok) {
    std::lock_guard<std::mutex> g(g_out);
    std::printf("%s %s\n", line.c_str(), ok ? "ok" : "BAD");
    if (!ok) ++g_bad;
}

static std::vector<uint32_t> expected(const uint8_t *msg, const Shape &s, int mode, uint32_t partial) {
    const size_t n = s.msg_len ? (s.msg_len - 1) / s.frag_len + 1 : 1;
    std::vector<uint32_t> v(n);
    for (size_t k = 0; k < n; ++k) {
        const size_t off = k * s.frag_len, len = std::min(s.frag_len, s.msg_len - off);
        if (mode == LAMPI_CSUM_CRC32) {
            v[k] = oracle_uicrc(msg + off, len, partial);
        } else {
            uint32_t pi = 0, pl = 0;
            v[k] = oracle_uicsum(msg + off, len, &pi, &pl);
        }
    }
    return v;
}

// One message, every mode / range / pinning combination.
static void run_shape(int tid, const Shape &s, uint8_t *msg_pageable, uint8_t *msg_pinned) {
    const size_t nfr = s.msg_len ? (s.msg_len - 1) / s.frag_len + 1 : 1;
    const size_t stride = s.frag_len + s.gap;
    std::vector<uint8_t> ring_pageable(nfr * stride + 64);
    std::vector<uint8_t> ring_store(nfr * stride + 64 + 4096);
    uint8_t *ring_pinned = ring_store.data() + (4096 - ((uintptr_t)ring_store.data() & 4095));
    const int reg = lampi_host_register(ring_pinned, nfr * stride + 64);
    if (reg) report("register ring rc " + std::to_string(reg), false);
    const size_t ranges[][2] = {{0, nfr}, {0, 1}, {nfr / 3, (nfr + 2) / 3}, {nfr > 3 ? nfr - 3 : 0, nfr > 3 ? 3 : nfr}};
    for (int mode : {LAMPI_CSUM_CRC32, LAMPI_CSUM_SUM32}) {
        const uint32_t partial = mode == LAMPI_CSUM_CRC32 ? (tid & 1 ? 0x1234ABCDu : LAMPI_CRC_INITIAL_REGISTER) : 0u;
        const std::vector<uint32_t> want = expected(msg_pageable, s, mode, partial);
        for (int src_pin = 0; src_pin < 2; ++src_pin) {
            const uint8_t *msg = src_pin ? msg_pinned : msg_pageable;
            for (const auto &rg : ranges) {
                const size_t k0 = rg[0], kc = rg[1];
                char tag[256];
                std::snprintf(tag, sizeof tag, "t%d L %zu msg %zu gap %zu mode %d src_pin %d k0 %zu kc %zu", tid,
                              s.frag_len, s.msg_len, s.gap, mode, src_pin, k0, kc);
                // checksum only
                std::vector<uint32_t> out(kc + 1, 0xDEADBEEFu);
                int rc = lampi_host_msg_csum(msg, s.msg_len, s.frag_len, k0, kc, partial, out.data(), mode);
                bool ok = rc == 0 && out[kc] == 0xDEADBEEFu;
                for (size_t i = 0; ok && i < kc; ++i) ok = out[i] == want[k0 + i];
                report(std::string("csum ") + tag, ok);
                // fused copy into both kinds of ring
                for (int ring_pin = 0; ring_pin < 2; ++ring_pin) {
                    uint8_t *ring = ring_pin ? ring_pinned : ring_pageable.data();
                    const size_t ring_bytes = nfr * stride + 64;
                    std::memset(ring, 0xA5, ring_bytes);
                    std::fill(out.begin(), out.end(), 0xDEADBEEFu);
                    rc = lampi_host_msg_bcopy(msg, s.msg_len, s.frag_len, k0, kc, ring, stride, partial, out.data(),
                                              mode);
                    ok = rc == 0 && out[kc] == 0xDEADBEEFu;
                    for (size_t i = 0; ok && i < kc; ++i) ok = out[i] == want[k0 + i];
                    // slot i holds fragment k0+i; every other ring byte keeps the sentinel
                    size_t pos = 0;
                    for (size_t i = 0; ok && i < kc; ++i) {
                        const size_t k = k0 + i, len = std::min(s.frag_len, s.msg_len - k * s.frag_len);
                        const uint8_t *slot = ring + i * stride;
                        for (; ok && pos < i * stride; ++pos) ok = ring[pos] == 0xA5;
                        ok = ok && std::memcmp(slot, msg_pageable + k * s.frag_len, len) == 0;
                        pos = i * stride + len;
                    }
                    for (; ok && pos < ring_bytes; ++pos) ok = ring[pos] == 0xA5;
                    report(std::string(ring_pin ? "bcopy_pinned_ring " : "bcopy_pageable_ring ") + tag, ok);
                }
            }
        }
    }
    if (!reg) lampi_host_unregister(ring_pinned);
}

static void run_suite(int tid, const std::vector<Shape> &shapes, uint8_t *msg_pageable, uint8_t *msg_pinned) {
    for (const Shape &s : shapes) run_shape(tid, s, msg_pageable, msg_pinned);
}

int main(int argc, char **argv) {
    const uint64_t seed = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 6;
    const int nthreads = argc > 2 ? std::atoi(argv[2]) : 2;
    const size_t kMsg = (150u << 20) + 12345;  // three 64 MiB pipeline chunks, ragged end
    std::vector<uint8_t> pageable(kMsg + 1);
    oracle_fill_stream(pageable.data(), seed, 0, kMsg);
    uint8_t *pinned = nullptr;
    std::vector<uint8_t> pin_store(kMsg + 4096 + 8);
    pinned = pin_store.data() + (4096 - ((uintptr_t)pin_store.data() & 4095)) + 8;  // a payload 8 bytes in
    std::memcpy(pinned, pageable.data(), kMsg);
    if (lampi_host_register(pinned, kMsg) != 0) {
        std::printf("lampi_host_register failed\n");
        return 1;
    }
    const std::vector<Shape> shapes = {
        {65456, kMsg, 72 + 8},            // GM: 65,456-byte payloads in 64 KiB buffers after the header
        {4096, (64u << 20) + 4096 * 5, 0},  // 4 KiB, one chunk + a few fragments, packed slots
        {16384, kMsg, 80},                // 16 KiB
        {1976, 3u << 20, 72},             // IB: 1,976-byte payloads
        {(70u << 20) + 3, kMsg, 16},      // fragments larger than a pipeline chunk
        {4096, 4095, 0},                  // one short fragment
        {4096, 0, 0},                     // empty message: one empty fragment
    };
    // invalid arguments are refused and write nothing
    uint32_t sentinel = 0xCAFEF00Du;
    const bool refused = lampi_host_msg_csum(pageable.data(), kMsg, 0, 0, 1, 0, &sentinel, 0) != 0 &&
                         lampi_host_msg_csum(pageable.data(), 4096, 4096, 1, 1, 0, &sentinel, 0) != 0 &&
                         lampi_host_msg_bcopy(pageable.data(), 8192, 4096, 0, 2, pinned, 4095, 0, &sentinel, 1) != 0 &&
                         lampi_host_msg_csum(pageable.data(), 4096, 4096, 0, 1, 0, &sentinel, 7) != 0 &&
                         sentinel == 0xCAFEF00Du;
    report("invalid_arguments_refused", refused);
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(run_suite, t + 1, std::cref(shapes), pageable.data(), pinned);
    for (auto &t : th) t.join();
    lampi_host_release();
    run_suite(0, shapes, pageable.data(), pinned);
    lampi_host_release();
    lampi_host_unregister(pinned);
    std::printf("pinned_after_release %lld\n", (long long)lampi_host_pinned_bytes());
    std::printf("bad %d done\n", g_bad);
    return g_bad != 0;
}
