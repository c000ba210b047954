// host_recv_caller.cc -- a native C++ caller of the host-memory receive path
// (lampi_host_header_check_batch / lampi_host_header_compare_batch / lampi_host_copy_to_app_batch,
// include/lampi_csum.h) in the shapes LA-MPI's receive loops have:
//   * GM: a ring of 64 KiB receive buffers, each a 72-byte gmHeader (dataLength @20, dataChecksum @64,
//     header checksum @68, ref src/path/gm/header.h:56-70) followed by up to 65,456 payload bytes;
//     the receiver checks the header residue (gm/path.cc:364-393), then CopyToApp
//     (common/BaseDesc.cc:288-342) with CopyFunction / CheckData (gm/recvFrag.h:165-257);
//   * GM buffers holding 4 KiB payloads (a 64 KiB slot pitch with wide gaps: one 2D DMA);
//   * IB: 2,048-byte ibData2KMsg_t buffers behind a 40-byte GRH (ib/init.cc:404-514), header checksum
//     uicrc/uicsum over 68 bytes compared with the stored word (ib/path.cc:652-680), 1,976 payload bytes
//     (ib/header.h:75-80), dataChecksum @64.
// Every shape runs in both checksum modes from page-locked and pageable rings, on two threads at once
// and then on the main thread after lampi_host_release().  Per batch: ~1% of the headers corrupted
// (the reference's `checksum |= 0xA4A4`, or a flipped header byte), ~2% of the data checksums
// corrupted (`dataChecksum |= 0xA4A4`, recvFrag.h:215-228) and ~1% of the payloads hit by a flipped
// byte after the sender stamped them; AppBufferLen <= 0 / < / = / > the fragment length; ragged and
// empty fragments; fragments delivered in ring order into one application buffer (runs of contiguous
// deliveries) and a shuffled batch delivered to scattered places.
//
// Every header verdict, every copied count, checksum and mask bit is compared with the oracle
// (oracle/libcsum_ref.so, the reference-pinned restatement -- test infrastructure), every byte of the
// application buffers with what CopyToApp would have delivered (sentinel elsewhere).  Prints one line
// per call and "bad N done"; exits 1 on any mismatch.  Build: make -C tests/native.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "lampi_csum.h"
#include "../../oracle/csum_ref.h"

static std::mutex g_out;
static int g_bad = 0;

static void report(const std::string &line, bool ok) {
    std::lock_guard<std::mutex> g(g_out);
    std::printf("%s %s\n", line.c_str(), ok ? "ok" : "BAD");
    if (!ok) ++g_bad;
}

static uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
static void wr32(uint8_t *p, uint32_t v) { std::memcpy(p, &v, 4); }
static uint32_t corrupt_a4(uint32_t w) { return (w | 0xA4A4u) != w ? (w | 0xA4A4u) : (w ^ 0xA4A4u); }

struct Shape {
    const char *name;
    size_t L;       // payload bytes of a full fragment
    size_t S;       // slot pitch
    size_t hdr_at;  // header offset in the slot (IB: after the 40-byte GRH)
    size_t nslots;
    bool ib;        // IB header check (recompute and compare) instead of GM's residue
};
constexpr size_t kHdr = 72, kDataLenOff = 20, kDataCsumOff = 64, kHdrCsumOff = 68;

static uint32_t data_csum(const uint8_t *p, size_t len, int mode) {
    if (mode == LAMPI_CSUM_CRC32) return oracle_uicrc(p, len, ORACLE_CRC_INIT);
    uint32_t pi = 0, pl = 0;
    return oracle_uicsum(p, len, &pi, &pl);
}

// Sender side of one slot: header fields, data checksum, header checksum (GM: headerChecksum over
// 68 bytes / 18 words, gm/sendFrag.cc:218-225; IB: uicrc/uicsum over 68 bytes, ib/sendFrag.cc:306-314).
static void stamp(uint8_t *slot, const Shape &s, uint32_t len, int mode) {
    uint8_t *h = slot + s.hdr_at;
    wr32(h + kDataLenOff, len);
    wr32(h + kDataCsumOff, data_csum(h + kHdr, len, mode));
    wr32(h + kHdrCsumOff, 0);
    uint32_t hc;
    if (!s.ib) {
        hc = oracle_header_checksum(h, kHdr - 4, 18, mode == LAMPI_CSUM_CRC32);
    } else {
        hc = data_csum(h, kHdr - 4, mode);
    }
    wr32(h + kHdrCsumOff, hc);
}

// The receiver's header verdict, restated from the reference's rules with the oracle.
static bool header_bad(const uint8_t *h, const Shape &s, int mode) {
    if (s.ib) return data_csum(h, kHdr - 4, mode) != rd32(h + kHdrCsumOff);
    if (mode == LAMPI_CSUM_CRC32) return oracle_uicrc(h, kHdr, ORACLE_CRC_INIT) != 0;
    uint32_t v = 0;
    for (int w = 0; w < 18; ++w) v += rd32(h + 4 * w);
    return v != 2 * rd32(h + kHdrCsumOff);
}

struct Want {
    int64_t copied;
    uint32_t csum;
    bool bad;
};
// RecvDesc_t::CopyToApp with the GM / IB hooks, on the oracle (the test's own composition of the pinned
// bcopy_uicrc / bcopy_uicsum, BaseDesc.cc:288-342, recvFrag.h:165-257).
static Want copy_to_app(const uint8_t *frag, uint32_t length, int64_t app_len, uint32_t expected, int mode,
                        std::vector<uint8_t> &tmp) {
    const uint32_t c = app_len <= 0 ? 0u : (app_len < (int64_t)length ? (uint32_t)app_len : length);
    // checksumming off: CopyFunction copies and returns 0 (gm/recvFrag.h:178-181), CheckData passes (:231-232)
    if (mode == LAMPI_CSUM_NONE) return {(int64_t)c, 0u, false};
    if (c == 0) return {0, mode == LAMPI_CSUM_CRC32 ? ORACLE_CRC_INIT : 0u, false};
    tmp.resize(std::max<size_t>(c, 1));
    uint32_t v;
    if (mode == LAMPI_CSUM_CRC32) {
        v = oracle_bcopy_uicrc(frag, tmp.data(), c, length, ORACLE_CRC_INIT);
    } else {
        uint32_t pi = 0, pl = 0;
        v = oracle_bcopy_uicsum(frag, tmp.data(), c, length, &pi, &pl);
    }
    return {v == expected ? (int64_t)c : -1, v, v != expected};
}

static bool bit(const std::vector<uint32_t> &m, size_t i) { return (m[i / 32] >> (i % 32)) & 1u; }

struct Ring {
    std::vector<uint8_t> store;
    uint8_t *p = nullptr;
    size_t bytes = 0;
    bool pinned = false;
    Ring(size_t n, bool pin) : store(n + 8192), bytes(n), pinned(pin) {
        p = store.data() + (4096 - ((uintptr_t)store.data() & 4095));
        if (pin && lampi_host_register(p, n) != 0) {
            report("register ring", false);
            pinned = false;
        }
    }
    ~Ring() {
        if (pinned) lampi_host_unregister(p);
    }
};

// One batch: build and stamp the ring, corrupt some of it, check the headers, deliver the fragments
// whose headers pass, compare everything with the oracle.
// dmode: the delivery's mode (LAMPI_CSUM_NONE: checksumming off; the headers are still checked in `mode`)
static void run_batch(int tid, const Shape &s, int mode, bool pin, bool shuffled, uint64_t seed, int dmode = -1) {
    if (dmode < 0) dmode = mode;
    char tag[200];
    std::snprintf(tag, sizeof tag, "t%d %s mode %d/%d ring_%s %s", tid, s.name, mode, dmode, pin ? "pinned" : "pageable",
                  shuffled ? "shuffled" : "ring_order");
    const size_t n = shuffled ? std::min<size_t>(s.nslots, 300) : s.nslots;
    Ring ring(n * s.S, pin);
    oracle_fill_stream(ring.p, seed, 0, ring.bytes);
    std::mt19937_64 rng(seed * 7 + 3);
    std::vector<uint32_t> len(n);
    for (size_t j = 0; j < n; ++j) {
        const uint64_t r = rng() % 100;
        len[j] = r < 2 ? 0u : r < 12 ? (uint32_t)(1 + rng() % s.L) : (uint32_t)s.L;
        stamp(ring.p + j * s.S, s, len[j], mode);
    }
    // corruption after stamping: headers, payload bytes; and the data checksums CheckData reads after the
    // header passed (the reference corrupts gmHeader_m->data.dataChecksum there, recvFrag.h:215-228)
    std::vector<char> bad_expected(n, 0);
    for (size_t j = 0; j < n; ++j) {
        uint8_t *h = ring.p + j * s.S + s.hdr_at;
        const uint64_t r = rng() % 1000;
        if (r < 4) wr32(h + kHdrCsumOff, corrupt_a4(rd32(h + kHdrCsumOff)));
        else if (r < 10) h[rng() % (kHdr - 4)] ^= (uint8_t)(1 + rng() % 255);
        else if (r < 30) bad_expected[j] = 1;
        else if (r < 40 && len[j]) h[kHdr + rng() % len[j]] ^= (uint8_t)(1 + rng() % 255);
    }

    // 1. the header checks over every slot
    std::vector<uint64_t> hoffs(n);
    for (size_t j = 0; j < n; ++j) hoffs[j] = j * s.S + s.hdr_at;
    std::vector<uint32_t> hmask((n + 31) / 32 + 1, 0xDEADBEEFu);
    uint32_t hnbad = 0xDEADBEEFu;
    int rc = s.ib ? lampi_host_header_compare_batch(ring.p, ring.bytes, hoffs.data(), n, kHdr - 4, kHdrCsumOff,
                                                    hmask.data(), &hnbad, mode)
                  : lampi_host_header_check_batch(ring.p, ring.bytes, hoffs.data(), n, kHdr, 18, kHdrCsumOff,
                                                  hmask.data(), &hnbad, mode);
    bool ok = rc == 0 && hmask.back() == 0xDEADBEEFu;
    std::vector<size_t> good;
    uint32_t want_nbad = 0;
    for (size_t j = 0; ok && j < n; ++j) {
        const bool b = header_bad(ring.p + hoffs[j], s, mode);
        want_nbad += b;
        ok = bit(hmask, j) == b;
        if (!b) good.push_back(j);
    }
    ok = ok && hnbad == want_nbad;
    for (size_t i = n; ok && i < ((n + 31) / 32) * 32; ++i) ok = !bit(hmask, i);
    report(std::string("headers ") + tag + " nbad " + std::to_string(want_nbad), ok);

    // 2. CopyToApp for the fragments whose headers passed, AppBufferLen cases by index
    if (shuffled) std::shuffle(good.begin(), good.end(), rng);
    const size_t m = good.size();
    std::vector<lampi_host_recv_frag> fr(m);
    const size_t slot_app = s.L + 64;  // shuffled batches: scattered deliveries, one app slot each
    std::vector<uint8_t> app(shuffled ? m * slot_app + 64 : n * s.L + 64, 0x5A);
    for (size_t i = 0; i < m; ++i) {
        const size_t j = good[i];
        const uint8_t *h = ring.p + hoffs[j];
        lampi_host_recv_frag &x = fr[i];
        x.frag_off = hoffs[j] + kHdr;
        x.length = len[j];
        x.expected = bad_expected[j] ? corrupt_a4(rd32(h + kDataCsumOff)) : rd32(h + kDataCsumOff);
        // ring order: fragment j lands at j * L of one message buffer; shuffled: its own app slot
        x.app = shuffled ? app.data() + (m - 1 - i) * slot_app + (i % 7) : app.data() + j * s.L;
        const int64_t L = len[j];
        switch (j % 13) {
            case 1: x.app_len = L - (int64_t)(j % 300) - 1; break;  // < (may be <= 0)
            case 2: x.app_len = 0; break;
            case 3: x.app_len = -7; break;
            case 4: x.app_len = L + 1000; break;  // >
            default: x.app_len = L; break;        // =
        }
    }
    std::vector<int64_t> copied(m + 1, 0x7777);
    std::vector<uint32_t> csum(m + 1, 0xDEADBEEFu), mask((m + 31) / 32 + 1, 0xDEADBEEFu);
    uint32_t nbad = 0xDEADBEEFu;
    rc = lampi_host_copy_to_app_batch(ring.p, ring.bytes, fr.data(), m, copied.data(), csum.data(), mask.data(), &nbad,
                                      dmode);
    ok = rc == 0 && copied[m] == 0x7777 && csum[m] == 0xDEADBEEFu && mask.back() == 0xDEADBEEFu;
    std::vector<uint8_t> want_app(app.size(), 0x5A), tmp;
    uint32_t wbad = 0;
    for (size_t i = 0; ok && i < m; ++i) {
        const lampi_host_recv_frag &x = fr[i];
        const uint8_t *frag = ring.p + x.frag_off;
        const Want w = copy_to_app(frag, x.length, x.app_len, x.expected, dmode, tmp);
        ok = copied[i] == w.copied && csum[i] == w.csum && bit(mask, i) == w.bad;
        wbad += w.bad;
        const uint32_t c = x.app_len <= 0 ? 0u : (uint32_t)std::min<int64_t>(x.app_len, x.length);
        if (c) std::memcpy(want_app.data() + ((uint8_t *)x.app - app.data()), frag, c);
        if (!ok)
            std::printf("  frag %zu (slot %zu) len %u app_len %lld: copied %lld/%lld csum %08x/%08x bad %d/%d\n", i,
                        good[i], x.length, (long long)x.app_len, (long long)copied[i], (long long)w.copied, csum[i],
                        w.csum, (int)bit(mask, i), (int)w.bad);
    }
    ok = ok && nbad == wbad && app == want_app;
    for (size_t i = m; ok && i < ((m + 31) / 32) * 32; ++i) ok = !bit(mask, i);
    report(std::string("copy_to_app ") + tag + " frags " + std::to_string(m) + " nbad " + std::to_string(wbad), ok);
}

static void run_suite(int tid, const std::vector<Shape> &shapes) {
    uint64_t seed = 1000 + 97 * (uint64_t)tid;
    for (const Shape &s : shapes)
        for (int mode : {LAMPI_CSUM_CRC32, LAMPI_CSUM_SUM32, LAMPI_CSUM_NONE})
            for (int pin = 0; pin < 2; ++pin)
                for (int shuf = 0; shuf < 2; ++shuf)
                    if (mode == LAMPI_CSUM_NONE)  // checksumming off: headers CRC-checked, delivery copy only
                        run_batch(tid, s, LAMPI_CSUM_CRC32, pin != 0, shuf != 0, ++seed, LAMPI_CSUM_NONE);
                    else
                        run_batch(tid, s, mode, pin != 0, shuf != 0, ++seed);
}

// Edge cases of one small batch: invalid arguments write nothing, an empty batch, only empty deliveries.
static void run_edges() {
    std::vector<uint8_t> ring(1 << 16, 0x11), app(1 << 16, 0x5A);
    lampi_host_recv_frag x{};
    x.frag_off = 100;
    x.length = 4096;
    x.app = app.data();
    x.app_len = 4096;
    x.expected = 0;
    int64_t copied = 0x7777;
    uint32_t csum = 0xDEADBEEFu, mask = 0xDEADBEEFu, nbad = 0xDEADBEEFu;
    bool ok = lampi_host_copy_to_app_batch(ring.data(), 4000, &x, 1, &copied, &csum, &mask, &nbad, 0) != 0 &&
              lampi_host_copy_to_app_batch(ring.data(), ring.size(), &x, 1, &copied, &csum, &mask, nullptr, 0) != 0 &&
              lampi_host_copy_to_app_batch(ring.data(), ring.size(), &x, 1, &copied, &csum, &mask, &nbad, 7) != 0 &&
              lampi_host_copy_to_app_batch(nullptr, ring.size(), &x, 1, &copied, &csum, &mask, &nbad, 0) != 0;
    uint64_t off = ring.size() - 10;
    ok = ok && lampi_host_header_check_batch(ring.data(), ring.size(), &off, 1, 72, 18, 68, &mask, &nbad, 0) != 0 &&
         lampi_host_header_compare_batch(ring.data(), ring.size(), &off, 1, 68, 66, &mask, &nbad, 0) != 0;
    ok = ok && copied == 0x7777 && csum == 0xDEADBEEFu && mask == 0xDEADBEEFu && nbad == 0xDEADBEEFu;
    report("invalid_arguments_refused", ok);
    ok = lampi_host_copy_to_app_batch(nullptr, 0, nullptr, 0, nullptr, nullptr, nullptr, &nbad, 0) == 0 && nbad == 0;
    report("empty_batch", ok);
    // nothing to deliver (AppBufferLen <= 0, zero length): nothing read -- the ring pointer may be null
    lampi_host_recv_frag e[3] = {x, x, x};
    e[0].app_len = 0;
    e[1].app_len = -1;
    e[2].length = 0;
    e[2].frag_off = (uint64_t)1 << 40;
    int64_t c3[3];
    uint32_t s3[3];
    for (int mode : {0, 1}) {
        mask = nbad = 0xDEADBEEFu;
        ok = lampi_host_copy_to_app_batch(nullptr, 0, e, 3, c3, s3, &mask, &nbad, mode) == 0 && nbad == 0 &&
             mask == 0 && c3[0] == 0 && c3[1] == 0 && c3[2] == 0;
        for (int i = 0; i < 3; ++i) ok = ok && s3[i] == (mode == 0 ? ORACLE_CRC_INIT : 0u);
        report("nothing_to_deliver mode " + std::to_string(mode), ok && app[0] == 0x5A);
    }
}

int main(int argc, char **argv) {
    const int nthreads = argc > 1 ? std::atoi(argv[1]) : 2;
    const std::vector<Shape> shapes = {
        {"gm65456", 65456, 65536, 0, 1100, false},   // 72 MB of payload: two pipeline chunks
        {"gm4k_in_64k", 4096, 65536, 0, 1100, false},  // constant pitch, wide gaps: 2D DMA
        {"ib1976", 1976, 2088, 40, 36000, true},      // 71 MB: two chunks of dense runs
    };
    run_edges();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(run_suite, t + 1, std::cref(shapes));
    for (auto &t : th) t.join();
    lampi_host_release();
    run_suite(0, shapes);
    lampi_host_release();
    std::printf("pinned_after_release %lld scratch_after_release %lld\n", (long long)lampi_host_pinned_bytes(),
                (long long)lampi_device_scratch_bytes());
    std::printf("bad %d done\n", g_bad);
    return g_bad != 0;
}
