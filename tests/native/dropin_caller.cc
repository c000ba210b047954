// dropin_caller.cc -- a native C++ program written against the reference's MemFunctions.h
// overloads (ref src/util/MemFunctions.h:43-65), compiled against include/lampi/MemFunctions.h
// and linked to liblampi_csum.so: the drop-in path a maintainer takes.
// It runs the call shapes of src/path on the SURVEY.md 8(d) stream and prints one line per
// call; tests/test_gpu_native.py recomputes every line with the oracle.
//   line: <op> <src_off> <dst_off> <copylen> <csumlen> <partial_in> <pint_in> <plen_in> ->
//         <result> <pint_out> <plen_out> <copy_ok>
// Threads: the same suite runs on T worker threads (each thread exits afterwards: the
// thread-exit release of the host staging), then again on the main thread after
// lampi_host_release().
// Build: make -C tests/native
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "lampi/MemFunctions.h"

static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static std::vector<unsigned char> stream_bytes(uint64_t seed, size_t n) {
    std::vector<unsigned char> b(n + 8);
    for (size_t i = 0; i < (n + 7) / 8; ++i) {
        uint64_t w = mix(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
        std::memcpy(&b[8 * i], &w, 8);
    }
    b.resize(n);
    return b;
}

struct Case {
    size_t off, doff, copylen, csumlen;
    unsigned partial, pint, plen;
};

static std::mutex g_out;

static void run_suite(const std::vector<unsigned char> &buf, const std::vector<Case> &cases, int tid) {
    std::vector<unsigned char> dst(buf.size() + 64);
    std::vector<std::string> lines;
    char line[256];
    auto emit = [&](const char *op, const Case &c, unsigned long r, unsigned long pi, unsigned long pl, int ok) {
        std::snprintf(line, sizeof line, "%d %s %zu %zu %zu %zu %u %u %u -> %lu %lu %lu %d", tid, op, c.off, c.doff,
                      c.copylen, c.csumlen, c.partial, c.pint, c.plen, r, pi, pl, ok);
        lines.push_back(line);
    };
    for (const Case &c : cases) {
        const unsigned char *s = buf.data() + c.off;
        // send: uicrc over a DMA source (quadrics/sendFrag.h:861-872), header-style default register
        emit("uicrc", c, uicrc(s, c.csumlen), 0, 0, 1);
        emit("uicrc_p", c, uicrc(s, c.csumlen, c.partial), 0, 0, 1);
        // send/receive copies: bcopy_uicrc (gm/sendFrag.cc:149, gm/recvFrag.h:174 copylen < crclen)
        std::memset(dst.data(), 0xEE, dst.size());
        unsigned r = bcopy_uicrc(s, dst.data() + c.doff, c.copylen, c.csumlen);
        int ok = std::memcmp(dst.data() + c.doff, s, c.copylen) == 0 && dst[c.doff + c.copylen] == 0xEE &&
                 (c.doff == 0 || dst[c.doff - 1] == 0xEE);
        emit("bcopy_uicrc", c, r, 0, 0, ok);
        std::memset(dst.data(), 0xEE, dst.size());
        r = bcopy_uicrc(s, dst.data() + c.doff, c.copylen, c.csumlen, c.partial);
        ok = std::memcmp(dst.data() + c.doff, s, c.copylen) == 0 && dst[c.doff + c.copylen] == 0xEE;
        emit("bcopy_uicrc_p", c, r, 0, 0, ok);
        // additive: fresh and chained partial-word state (gm/sendFrag.cc:202-204: csum += ...)
        emit("uicsum", c, uicsum(s, c.csumlen), 0, 0, 1);
        unsigned pi = c.pint, pl = c.plen;
        r = uicsum(s, c.csumlen, &pi, &pl);
        emit("uicsum_s", c, r, pi, pl, 1);
        std::memset(dst.data(), 0xEE, dst.size());
        r = bcopy_uicsum(s, dst.data() + c.doff, c.copylen, c.csumlen);
        ok = std::memcmp(dst.data() + c.doff, s, c.copylen) == 0 && dst[c.doff + c.copylen] == 0xEE;
        emit("bcopy_uicsum", c, r, 0, 0, ok);
        pi = c.pint;
        pl = c.plen;
        std::memset(dst.data(), 0xEE, dst.size());
        r = bcopy_uicsum(s, dst.data() + c.doff, c.copylen, c.csumlen, &pi, &pl);
        ok = std::memcmp(dst.data() + c.doff, s, c.copylen) == 0 && dst[c.doff + c.copylen] == 0xEE;
        emit("bcopy_uicsum_s", c, r, pi, pl, ok);
        // 64-bit (MemFunctions.h:43-50)
        emit("csum", c, csum(s, c.csumlen), 0, 0, 1);
        std::memset(dst.data(), 0xEE, dst.size());
        unsigned long r64 = bcopy_csum(s, dst.data() + c.doff, c.copylen, c.csumlen);
        ok = std::memcmp(dst.data() + c.doff, s, c.copylen) == 0 && dst[c.doff + c.copylen] == 0xEE;
        emit("bcopy_csum", c, r64, 0, 0, ok);
    }
    std::lock_guard<std::mutex> g(g_out);
    for (auto &l : lines) std::puts(l.c_str());
}

int main(int argc, char **argv) {
    const uint64_t seed = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 11;
    const int nthreads = argc > 2 ? std::atoi(argv[2]) : 4;
    const size_t N = 3 << 20;
    std::vector<unsigned char> buf = stream_bytes(seed, N);
    std::vector<Case> cases;
    uint64_t z = seed * 977 + 5;
    const size_t lens[] = {0, 1, 3, 4, 5, 63, 64, 72, 1976, 4095, 4096, 4097, 16384, 65456, 65536, 1 << 20};
    for (size_t L : lens) {
        z = mix(z);
        Case c;
        c.off = z % 61;
        c.doff = (z >> 8) % 13;
        c.csumlen = L;
        c.copylen = (z >> 16) % 3 == 0 && L ? L - 1 - (z >> 20) % L : L;  // copylen < csumlen sometimes
        c.partial = (unsigned)(z >> 32);
        c.plen = (unsigned)((z >> 24) % 4);
        c.pint = c.plen ? (unsigned)(z >> 40) & ((1u << (8 * c.plen)) - 1) : 0u;
        cases.push_back(c);
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(run_suite, std::cref(buf), std::cref(cases), t + 1);
    for (auto &t : th) t.join();
    lampi_host_release();
    run_suite(buf, cases, 0);
    lampi_host_release();
    run_suite(buf, cases, 0);  // a released thread allocates its staging again
    std::printf("seed %llu cases %zu threads %d done\n", (unsigned long long)seed, cases.size(), nthreads);
    return 0;
}
