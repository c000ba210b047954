// host_leak.cc -- the host entry points' staging must not leak: 1,000 short-lived threads each
// make host calls and exit (thread_local release), then 1,000 call + lampi_host_release()
// rounds on one thread (the same release a device switch runs).  Prints device memory in use
// before and after each phase (hipMemGetInfo) and the checksum XOR of all calls.
// Build: make -C tests/native
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "lampi_csum.h"

static size_t used() {
    size_t f = 0, t = 0;
    if (hipMemGetInfo(&f, &t) != hipSuccess) std::abort();
    return t - f;
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 1000;
    std::vector<unsigned char> buf(1 << 20);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (unsigned char)(i * 131 + 7);
    std::vector<unsigned char> dst(buf.size());
    unsigned x = lampi_uicrc(buf.data(), buf.size(), 0xFFFFFFFFu);  // warm: tables, first context
    const unsigned want = x;
    const size_t u0 = used();
    unsigned bad = 0;
    for (int r = 0; r < rounds; ++r) {
        std::thread t([&] {
            if (lampi_uicrc(buf.data(), buf.size(), 0xFFFFFFFFu) != want) ++bad;
            unsigned pi = 0, pl = 0;
            (void)lampi_bcopy_uicsum(buf.data(), dst.data(), 4096, 4099, &pi, &pl);
        });
        t.join();
    }
    const size_t u1 = used();
    for (int r = 0; r < rounds; ++r) {
        if (lampi_bcopy_uicrc(buf.data(), dst.data(), 65456, 65456, 0xFFFFFFFFu) == 0x12345678u) ++bad;
        lampi_host_release();
    }
    const size_t u2 = used();
    std::printf("rounds %d used_before %zu after_threads %zu after_release %zu bad %u\n", rounds, u0, u1, u2, bad);
    return bad != 0;
}
