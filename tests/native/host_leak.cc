// host_leak.cc -- the host entry points' staging must not leak: 1,000 short-lived threads each
// make host calls and exit (thread_local release), then 1,000 call + lampi_host_release()
// rounds on one thread (the same release a device switch runs).  Prints device memory in use
// before and after each phase (hipMemGetInfo) and the page-locked host memory the library holds
// (lampi_host_pinned_bytes: bounce buffers, result words, staging -- invisible to hipMemGetInfo).
// The calls include the host-message pipeline (lampi_host_msg_csum / _bcopy), the receive path
// (lampi_host_copy_to_app_batch on GM-sized fragments, whose row groups take per-thread device scratch,
// lampi_device_scratch_bytes) and calls above the zero-copy limit, so every kind of staging is
// allocated and must be released.
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
    std::vector<uint32_t> frag(buf.size() / 4096);
    unsigned x = lampi_uicrc(buf.data(), buf.size(), 0xFFFFFFFFu);  // warm: tables, first context
    const unsigned want = x;
    if (lampi_host_msg_csum(buf.data(), buf.size(), 4096, 0, frag.size(), 0xFFFFFFFFu, frag.data(), 0) != 0) return 2;
    const uint32_t want0 = frag[0];
    // 16 GM-sized fragments delivered from buf into dst (row groups: device scratch on the pipeline's stream)
    std::vector<lampi_host_recv_frag> rf(16);
    for (size_t i = 0; i < rf.size(); ++i) rf[i] = {i * 65456, dst.data() + i * 65456, 65456, 65456, 0u};
    auto recv = [&]() {
        std::vector<int64_t> copied(rf.size());
        std::vector<uint32_t> cs(rf.size());
        uint32_t mask = 0, nbad = 0;
        return lampi_host_copy_to_app_batch(buf.data(), buf.size(), rf.data(), rf.size(), copied.data(), cs.data(),
                                            &mask, &nbad, 0) == 0 &&
               nbad == rf.size() && copied[0] == -1;  // expected 0: every fragment reads as corrupt
    };
    const size_t u0 = used();
    const long long p0 = (long long)lampi_host_pinned_bytes();
    unsigned bad = 0;
    for (int r = 0; r < rounds; ++r) {
        std::thread t([&] {
            if (lampi_uicrc(buf.data(), buf.size(), 0xFFFFFFFFu) != want) ++bad;
            unsigned pi = 0, pl = 0;
            (void)lampi_bcopy_uicsum(buf.data(), dst.data(), 4096, 4099, &pi, &pl);
            std::vector<uint32_t> f(frag.size());
            if (r % 4 == 0) {  // the pipeline, pageable source and ring: every bounce buffer
                if (lampi_host_msg_bcopy(buf.data(), buf.size(), 4096, 0, f.size(), dst.data(), 4096, 0xFFFFFFFFu,
                                         f.data(), 0) != 0 || f[0] != want0)
                    ++bad;
            }
            if (r % 4 == 1 && !recv()) ++bad;
        });
        t.join();
    }
    const size_t u1 = used();
    const long long p1 = (long long)lampi_host_pinned_bytes();
    const long long s1 = (long long)lampi_device_scratch_bytes();
    for (int r = 0; r < rounds; ++r) {
        if (lampi_bcopy_uicrc(buf.data(), dst.data(), 65456, 65456, 0xFFFFFFFFu) == 0x12345678u) ++bad;
        if (r % 8 == 0 && lampi_host_msg_csum(buf.data(), buf.size(), 4096, 0, frag.size(), 0xFFFFFFFFu, frag.data(),
                                              0) != 0)
            ++bad;
        if (r % 8 == 1 && !recv()) ++bad;
        lampi_host_release();
    }
    const size_t u2 = used();
    const long long p2 = (long long)lampi_host_pinned_bytes();
    const long long s2 = (long long)lampi_device_scratch_bytes();
    std::printf("rounds %d used_before %zu after_threads %zu after_release %zu pinned_before %lld "
                "pinned_after_threads %lld pinned_after_release %lld scratch_after_threads %lld "
                "scratch_after_release %lld bad %u\n",
                rounds, u0, u1, u2, p0, p1, p2, s1, s2, bad);
    return bad != 0;
}
