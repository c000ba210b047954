// host_chain_caller.cc -- a native C++ caller of lampi_host_chain_csum_batch (include/lampi_csum.h):
// chained checksums over typemap pieces in host memory, the send side's gather into the payload
// (ref src/path/gm/sendFrag.cc:157-217, ib/sendFrag.cc:140-203) and the receive side's scatter into
// the application buffer (non_contiguous_copy, src/path/common/BaseDesc.cc:72-163).
//
//   * the reference's own chain fixtures (argv[1]: a text file tests/test_gpu_native.py writes from
//     tests/golden/fixtures.json `chain` -- "seed off len crc sum ncuts cut..." per case, the values
//     computed by the compiled reference MemFunctions.cc): every case one fragment of one batch,
//     pieces gathered into a gapped destination;
//   * strided-vector typemaps (MPI_Type_vector-like: E-byte elements at stride S) gathered into packed
//     payloads and scattered back, K elements per fragment, checked against the oracle's checksum of the
//     packed bytes (chained == contiguous, the identity the partial state guarantees);
//   * random typemaps: misaligned pieces of 1 B .. 20 KB, checksum-only pieces (dst NULL), pieces
//     whose csumlen exceeds copylen, CRC starting registers, empty fragments -- against the oracle's
//     piece-by-piece chain (oracle/libcsum_ref.so, reference-pinned; test infrastructure);
// both modes, pageable and page-locked buffers, on two threads at once and then on the main thread.
// Every checksum and every destination byte is checked (sentinels around the copies).  Prints one
// line per batch and "bad N done"; exits 1 on any mismatch.  Build: make -C tests/native.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <random>
#include <sstream>
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

static uint32_t contiguous(const uint8_t *p, size_t len, int mode, uint32_t partial = ORACLE_CRC_INIT) {
    if (mode == LAMPI_CSUM_CRC32) return oracle_uicrc(p, len, partial);
    uint32_t pi = 0, pl = 0;
    return oracle_uicsum(p, len, &pi, &pl);
}

struct Buf {  // a host buffer, optionally page-locked through the library
    std::vector<uint8_t> store;
    uint8_t *p;
    size_t n;
    bool pinned;
    Buf(size_t bytes, bool pin, uint8_t fill) : store(bytes + 8192, fill), n(bytes), pinned(pin) {
        p = store.data() + (4096 - ((uintptr_t)store.data() & 4095));
        if (pin && lampi_host_register(p, bytes + 64) != 0) {
            report("register", false);
            pinned = false;
        }
    }
    ~Buf() {
        if (pinned) lampi_host_unregister(p);
    }
};

struct Case {
    uint64_t seed, off, len;
    uint32_t crc, sum;
    std::vector<uint64_t> cuts;
};

// The reference's chain fixtures: one batch of every case, pieces gathered into a gapped destination.
static void run_fixtures(int tid, const std::vector<Case> &cases) {
    size_t total = 0;
    for (const Case &c : cases) total += c.len + 16;
    for (int pin = 0; pin < 2; ++pin) {
        Buf src(total, pin, 0), dst(total * 2 + 64, pin, 0x5A);
        std::vector<lampi_host_piece> pcs;
        std::vector<uint32_t> first{0};
        std::vector<uint8_t> want(dst.n, 0x5A);
        size_t so = 0, dpos = 0;
        for (const Case &c : cases) {
            oracle_fill_stream(src.p + so, c.seed, c.off, c.len);
            std::vector<uint64_t> b{0};
            b.insert(b.end(), c.cuts.begin(), c.cuts.end());
            b.push_back(c.len);
            for (size_t i = 0; i + 1 < b.size(); ++i) {
                const uint32_t n = (uint32_t)(b[i + 1] - b[i]);
                pcs.push_back({src.p + so + b[i], dst.p + dpos, n, n, ORACLE_CRC_INIT, 0u});
                std::memcpy(want.data() + dpos, src.p + so + b[i], n);
                dpos += n + 5;  // receive-side scatter with gaps
            }
            first.push_back((uint32_t)pcs.size());
            so += c.len + 16;
        }
        for (int mode : {LAMPI_CSUM_CRC32, LAMPI_CSUM_SUM32}) {
            std::memset(dst.p, 0x5A, dst.n);
            std::vector<uint32_t> out(cases.size() + 1, 0xDEADBEEFu);
            const int rc = lampi_host_chain_csum_batch(pcs.data(), pcs.size(), first.data(), cases.size(), out.data(),
                                                       mode);
            bool ok = rc == 0 && out[cases.size()] == 0xDEADBEEFu;
            for (size_t i = 0; ok && i < cases.size(); ++i) ok = out[i] == (mode == 0 ? cases[i].crc : cases[i].sum);
            ok = ok && std::memcmp(dst.p, want.data(), dst.n) == 0;
            report("fixtures t" + std::to_string(tid) + " cases " + std::to_string(cases.size()) + " mode " +
                       std::to_string(mode) + (pin ? " pinned" : " pageable"),
                   ok);
        }
    }
}

// Strided vectors: gather (send) and scatter (receive) of E-byte elements at stride S, K per fragment.
static void run_vectors(int tid, uint64_t seed) {
    const size_t shapes[][4] = {{8, 16, 512, 8192},  {24, 40, 1000, 9000}, {100, 128, 333, 5000},
                                {1024, 1536, 64, 2000}, {4096, 8192, 16, 600}, {1976, 2088, 1, 3000}};
    for (const auto &sh : shapes) {
        const size_t E = sh[0], S = sh[1], K = sh[2], M = sh[3], nf = (M + K - 1) / K;
        for (int pin = 0; pin < 2; ++pin) {
            Buf app(M * S, pin, 0x5A), packed(M * E, pin, 0x5A);
            oracle_fill_stream(app.p, seed + E, 0, M * S);
            std::vector<uint8_t> want_packed(M * E);
            for (size_t i = 0; i < M; ++i) std::memcpy(want_packed.data() + i * E, app.p + i * S, E);
            std::vector<lampi_host_piece> g(M), s(M);
            std::vector<uint32_t> first(nf + 1);
            for (size_t f = 0; f <= nf; ++f) first[f] = (uint32_t)std::min(M, f * K);
            for (size_t i = 0; i < M; ++i) {
                g[i] = {app.p + i * S, packed.p + i * E, (uint32_t)E, (uint32_t)E, ORACLE_CRC_INIT, 0u};
                s[i] = {packed.p + i * E, app.p + i * S, (uint32_t)E, (uint32_t)E, ORACLE_CRC_INIT, 0u};
            }
            for (int mode : {LAMPI_CSUM_CRC32, LAMPI_CSUM_SUM32}) {
                char tag[160];
                std::snprintf(tag, sizeof tag, "t%d E %zu S %zu K %zu frags %zu mode %d %s", tid, E, S, K, nf, mode,
                              pin ? "pinned" : "pageable");
                std::vector<uint32_t> want(nf);
                for (size_t f = 0; f < nf; ++f)
                    want[f] = contiguous(want_packed.data() + first[f] * E, (first[f + 1] - first[f]) * E, mode);
                // gather: the packed payloads and their checksums
                std::memset(packed.p, 0x5A, packed.n);
                std::vector<uint32_t> out(nf, 0xDEADBEEFu);
                int rc = lampi_host_chain_csum_batch(g.data(), M, first.data(), nf, out.data(), mode);
                bool ok = rc == 0 && out == want && std::memcmp(packed.p, want_packed.data(), packed.n) == 0;
                report(std::string("vector_gather ") + tag, ok);
                // scatter: the packed payloads back into a wiped application buffer, same checksums
                std::vector<uint8_t> keep(app.p, app.p + app.n);
                std::memset(app.p, 0x33, app.n);
                std::fill(out.begin(), out.end(), 0xDEADBEEFu);
                rc = lampi_host_chain_csum_batch(s.data(), M, first.data(), nf, out.data(), mode);
                ok = rc == 0 && out == want;
                for (size_t i = 0; ok && i < M; ++i) {
                    ok = std::memcmp(app.p + i * S, keep.data() + i * S, E) == 0;
                    for (size_t b = E; ok && b < S; ++b) ok = app.p[i * S + b] == 0x33;  // the gaps untouched
                }
                std::memcpy(app.p, keep.data(), app.n);
                report(std::string("vector_scatter ") + tag, ok);
            }
        }
    }
}

// Random typemaps against the oracle's piece-by-piece chain.
static void run_random(int tid, uint64_t seed) {
    std::mt19937_64 rng(seed);
    for (int rep = 0; rep < 6; ++rep) {
        const size_t nf = 1 + rng() % 600;
        const size_t src_bytes = 24u << 20;
        Buf src(src_bytes, rep & 1, 0), dst(src_bytes, rep & 1, 0x5A);
        oracle_fill_stream(src.p, seed + rep, 0, src_bytes);
        std::vector<lampi_host_piece> pcs;
        std::vector<uint32_t> first{0};
        std::vector<std::vector<size_t>> frag_pieces;
        size_t dpos = 0;
        for (size_t f = 0; f < nf; ++f) {
            const size_t np = rng() % 13 == 0 ? 0 : 1 + rng() % 40;
            const uint32_t partial = (uint32_t)rng();
            for (size_t i = 0; i < np; ++i) {
                const uint32_t len = rng() % 4 ? 1 + rng() % 64 : 200 + rng() % 20000;
                const size_t so = rng() % (src_bytes - len);
                const int kind = (int)(rng() % 10);  // 0: checksum only, 1: csumlen > copylen, else plain
                lampi_host_piece x{src.p + so, nullptr, 0u, len, i == 0 ? partial : 0u, 0u};
                if (kind != 0 && dpos + len + 8 < dst.n) {
                    x.dst = dst.p + dpos;
                    x.copylen = kind == 1 ? len / 2 : len;
                    dpos += x.copylen + rng() % 3;
                }
                pcs.push_back(x);
            }
            first.push_back((uint32_t)pcs.size());
        }
        for (int mode : {LAMPI_CSUM_CRC32, LAMPI_CSUM_SUM32}) {
            std::memset(dst.p, 0x5A, dst.n);
            std::vector<uint8_t> want_dst(dst.n, 0x5A);
            std::vector<uint32_t> want(nf);
            for (size_t f = 0; f < nf; ++f) {
                uint32_t crc = first[f] < first[f + 1] ? pcs[first[f]].partial : ORACLE_CRC_INIT, sum = 0, pi = 0, pl = 0;
                for (size_t j = first[f]; j < first[f + 1]; ++j) {
                    const lampi_host_piece &x = pcs[j];
                    const size_t n = std::max(x.copylen, x.csumlen);
                    if (mode == LAMPI_CSUM_CRC32) crc = oracle_uicrc(x.src, n, crc);
                    else sum += oracle_uicsum(x.src, n, &pi, &pl);
                    if (x.dst) std::memcpy(want_dst.data() + ((uint8_t *)x.dst - dst.p), x.src, x.copylen);
                }
                want[f] = mode == LAMPI_CSUM_CRC32 ? crc : sum;
            }
            std::vector<uint32_t> out(nf, 0xDEADBEEFu);
            const int rc = lampi_host_chain_csum_batch(pcs.data(), pcs.size(), first.data(), nf, out.data(), mode);
            const bool ok = rc == 0 && out == want && std::memcmp(dst.p, want_dst.data(), dst.n) == 0;
            report("random t" + std::to_string(tid) + " rep " + std::to_string(rep) + " frags " + std::to_string(nf) +
                       " pieces " + std::to_string(pcs.size()) + " mode " + std::to_string(mode),
                   ok);
        }
    }
}

// The non-contiguous CopyToApp (lampi_host_chain_copy_to_app_batch): random typemaps of received fragments
// scattered into an application buffer, ~25% of the expected checksums corrupted (|= 0xA4A4), the pieces'
// partial garbage (the batch starts CRC from the initial register), fragments with no pieces (AppBufferLen
// <= 0); every verdict, checksum and delivered byte against the oracle's piece-by-piece chain
// (ref src/path/common/BaseDesc.cc:72-163, :326-340; src/path/gm/recvFrag.h:186-257), all three modes.
static void run_deliver(int tid, uint64_t seed) {
    std::mt19937_64 rng(seed);
    for (int rep = 0; rep < 4; ++rep) {
        const size_t nf = 1 + rng() % 500;
        const size_t src_bytes = 16u << 20;
        Buf src(src_bytes, rep & 1, 0), dst(src_bytes, rep & 1, 0x5A);
        oracle_fill_stream(src.p, seed + 31 * rep, 0, src_bytes);
        std::vector<lampi_host_piece> pcs;
        std::vector<uint32_t> first{0};
        size_t dpos = 0;
        for (size_t f = 0; f < nf; ++f) {
            const size_t np = rng() % 11 == 0 ? 0 : 1 + rng() % 30;
            for (size_t i = 0; i < np && dpos + 21000 < dst.n; ++i) {
                const uint32_t len = rng() % 9 == 0 ? 0u : rng() % 4 ? 1 + rng() % 64 : 200 + rng() % 20000;
                const size_t so = rng() % (src_bytes - len);
                pcs.push_back(lampi_host_piece{src.p + so, dst.p + dpos, len, len, (uint32_t)rng(), 0u});
                dpos += len + rng() % 5;
            }
            first.push_back((uint32_t)pcs.size());
        }
        for (int mode : {LAMPI_CSUM_CRC32, LAMPI_CSUM_SUM32, LAMPI_CSUM_NONE}) {
            std::memset(dst.p, 0x5A, dst.n);
            std::vector<uint8_t> want_dst(dst.n, 0x5A);
            std::vector<uint32_t> expected(nf), want_csum(nf);
            std::vector<int64_t> want_copied(nf);
            std::vector<uint32_t> want_mask((nf + 31) / 32, 0u);
            uint32_t want_nbad = 0;
            for (size_t f = 0; f < nf; ++f) {
                uint32_t crc = ORACLE_CRC_INIT, sum = 0, pi = 0, pl = 0;
                int64_t copied = 0;
                for (size_t j = first[f]; j < first[f + 1]; ++j) {
                    const lampi_host_piece &x = pcs[j];
                    if (mode == LAMPI_CSUM_CRC32) crc = oracle_uicrc(x.src, x.copylen, crc);
                    if (mode == LAMPI_CSUM_SUM32) sum += oracle_uicsum(x.src, x.copylen, &pi, &pl);
                    std::memcpy(want_dst.data() + ((uint8_t *)x.dst - dst.p), x.src, x.copylen);
                    copied += x.copylen;
                }
                const uint32_t c = mode == LAMPI_CSUM_CRC32 ? crc : mode == LAMPI_CSUM_SUM32 ? sum : 0u;
                expected[f] = rng() % 4 == 0 ? (c | 0xA4A4u) : c;
                const bool bad = mode != LAMPI_CSUM_NONE && copied != 0 && c != expected[f];
                want_csum[f] = c;
                want_copied[f] = bad ? -1 : copied;
                if (bad) {
                    want_mask[f / 32] |= 1u << (f % 32);
                    ++want_nbad;
                }
            }
            std::vector<int64_t> copied(nf, 77);
            std::vector<uint32_t> csum(nf, 0xDEADBEEFu), mask((nf + 31) / 32, 0xFFFFFFFFu);
            uint32_t nbad = 12345;
            const int rc = lampi_host_chain_copy_to_app_batch(pcs.data(), pcs.size(), first.data(), nf, expected.data(),
                                                              copied.data(), csum.data(), mask.data(), &nbad, mode);
            const bool ok = rc == 0 && copied == want_copied && csum == want_csum && mask == want_mask &&
                            nbad == want_nbad && std::memcmp(dst.p, want_dst.data(), dst.n) == 0;
            report("deliver t" + std::to_string(tid) + " rep " + std::to_string(rep) + " frags " + std::to_string(nf) +
                       " pieces " + std::to_string(pcs.size()) + " mode " + std::to_string(mode) + " bad " +
                       std::to_string(want_nbad),
                   ok);
        }
    }
}

static void run_edges() {
    std::vector<uint8_t> a(4096, 1), b(4096, 0x5A);
    lampi_host_piece x{a.data(), b.data(), 100, 100, ORACLE_CRC_INIT, 0u};
    const uint32_t f_ok[2] = {0, 1}, f_bad[2] = {1, 0}, f_over[2] = {0, 2};
    uint32_t out[2] = {0xDEADBEEFu, 0xDEADBEEFu};
    lampi_host_piece nul = x;
    nul.src = nullptr;
    bool ok = lampi_host_chain_csum_batch(&x, 1, f_bad, 1, out, 0) != 0 &&
              lampi_host_chain_csum_batch(&x, 1, f_over, 1, out, 0) != 0 &&
              lampi_host_chain_csum_batch(&nul, 1, f_ok, 1, out, 0) != 0 &&
              lampi_host_chain_csum_batch(&x, 1, f_ok, 1, out, 9) != 0 && out[0] == 0xDEADBEEFu && b[0] == 0x5A;
    report("invalid_arguments_refused", ok);
    // fragments without pieces: CRC the initial register, SUM 0
    const uint32_t f_empty[4] = {0, 0, 0, 0};
    uint32_t o3[3];
    ok = lampi_host_chain_csum_batch(nullptr, 0, f_empty, 3, o3, 0) == 0 && o3[0] == ORACLE_CRC_INIT &&
         o3[2] == ORACLE_CRC_INIT && lampi_host_chain_csum_batch(nullptr, 0, f_empty, 3, o3, 1) == 0 && o3[1] == 0;
    report("fragments_without_pieces", ok);
    // the delivery batch: bad arguments refused before anything is written; no pieces = DataOK whatever expected
    int64_t cp[3] = {7, 7, 7};
    uint32_t cs[3] = {1, 1, 1}, mk[1] = {0xFFFFFFFFu}, nb = 9, ex[3] = {1, 2, 3};
    ok = lampi_host_chain_copy_to_app_batch(&x, 1, f_bad, 1, ex, cp, cs, mk, &nb, 0) != 0 &&
         lampi_host_chain_copy_to_app_batch(&x, 1, f_ok, 1, nullptr, cp, cs, mk, &nb, 0) != 0 &&
         lampi_host_chain_copy_to_app_batch(&x, 1, f_ok, 1, ex, cp, cs, mk, &nb, 9) != 0 && cp[0] == 7 && nb == 9;
    ok = ok && lampi_host_chain_copy_to_app_batch(nullptr, 0, f_empty, 3, ex, cp, cs, mk, &nb, 0) == 0 && nb == 0 &&
         mk[0] == 0 && cp[0] == 0 && cp[2] == 0 && cs[1] == ORACLE_CRC_INIT &&
         lampi_host_chain_copy_to_app_batch(nullptr, 0, f_empty, 3, nullptr, cp, cs, mk, &nb, LAMPI_CSUM_NONE) == 0 &&
         nb == 0 && cs[0] == 0;
    report("deliver_edges", ok);
}

static void suite(int tid, const std::vector<Case> *cases) {
    if (cases && !cases->empty()) run_fixtures(tid, *cases);
    run_vectors(tid, 500 + tid);
    run_random(tid, 900 + 17 * tid);
    run_deliver(tid, 1300 + 7 * tid);
}

int main(int argc, char **argv) {
    std::vector<Case> cases;
    if (argc > 1) {
        std::ifstream in(argv[1]);
        std::string line;
        while (std::getline(in, line)) {
            std::istringstream ss(line);
            Case c;
            size_t ncut = 0;
            if (!(ss >> c.seed >> c.off >> c.len >> c.crc >> c.sum >> ncut)) continue;
            c.cuts.resize(ncut);
            for (auto &v : c.cuts) ss >> v;
            cases.push_back(c);
        }
        std::printf("fixture_cases %zu\n", cases.size());
    }
    const int nthreads = argc > 2 ? std::atoi(argv[2]) : 2;
    run_edges();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(suite, t + 1, &cases);
    for (auto &t : th) t.join();
    lampi_host_release();
    suite(0, &cases);
    lampi_host_release();
    std::printf("pinned_after_release %lld scratch_after_release %lld\n", (long long)lampi_host_pinned_bytes(),
                (long long)lampi_device_scratch_bytes());
    std::printf("bad %d done\n", g_bad);
    return g_bad != 0;
}
