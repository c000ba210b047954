// plan_check.cc -- CPU check of the host paths' DMA planner (lampi_amd/csrc/host_plan.h), no GPU.
//
// Random batches of items (NIC-ring fragments with the ring rules; typemap pieces with the strict
// rules, including strided vectors and fragment boundaries) are planned chunk by chunk, and the plan
// is executed on the CPU: every H2D transfer is a memcpy (2D row by row) from the source into a host
// stand-in of the chunk's input buffer, every item's `copy` bytes are moved from its input offset to
// its output offset (the kernel's part), and every D2H transfer is a memcpy into the destinations.
// Checked: each item's source bytes arrive at its input offset; the destinations end up holding the
// sources' bytes and nothing else is written (sentinels); no transfer reads outside the items' own
// bytes (strict rules) or outside the ring (ring rules); chunks stay within the planner's announced
// capacities and start only where boundary() allows; transfers are coalesced where the layout allows
// (one H2D and one D2H for a dense ring batch, one 2D transfer per direction for a strided vector).
// Prints "bad N done"; exits 1 on any failure.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../lampi_amd/csrc/host_plan.h"

using namespace lampi;

static int g_bad = 0;
static void report(const std::string &what, bool ok) {
    std::printf("%s %s\n", what.c_str(), ok ? "ok" : "BAD");
    if (!ok) ++g_bad;
}

struct Item {
    uint64_t src, len;
    uint64_t dst, copy;  // dst: offset into the destination arena
    bool start;          // a chunk may start here
};

struct Items {
    const std::vector<Item> *v;
    uint8_t *dst_base;
    size_t size() const { return v->size(); }
    PlanItem get(size_t j) const {
        const Item &x = (*v)[j];
        return PlanItem{x.src, x.len, x.copy ? dst_base + x.dst : nullptr, x.copy};
    }
    bool boundary(size_t j) const { return (*v)[j].start; }
};

// Plan and execute one batch; src arena [0, src_bytes) (ring: all of it readable).
static void run(const std::string &name, const std::vector<Item> &items, size_t src_bytes, bool ring, size_t cap,
                size_t want_in_xfers = 0, size_t want_out_xfers = 0) {
    std::vector<uint8_t> src(src_bytes);
    for (size_t i = 0; i < src_bytes; ++i) src[i] = (uint8_t)(i * 131 + (i >> 9) * 7 + 1);
    size_t dst_bytes = 64;
    for (const Item &x : items) dst_bytes = std::max<size_t>(dst_bytes, x.dst + x.copy + 64);
    std::vector<uint8_t> dst(dst_bytes, 0xA5), want(dst_bytes, 0xA5);
    std::vector<uint8_t> readable(src_bytes, ring ? 1 : 0);
    for (const Item &x : items) {
        if (!ring)
            for (uint64_t i = 0; i < x.len; ++i) readable[x.src + i] = 1;
        if (x.copy) std::memcpy(want.data() + x.dst, src.data() + x.src, x.copy);
    }
    PlanRules R;
    R.ring = ring;
    R.ring_bytes = src_bytes;
    std::vector<size_t> din(items.size()), dout(items.size());
    const Items view{&items, dst.data()};
    StreamPlanner<Items> pl(view, R, cap, din.data(), dout.data());
    std::vector<uint8_t> dev_in(pl.in_need()), dev_out(pl.out_need());
    ChunkPlan c;
    std::vector<InXfer> in;
    std::vector<OutXfer> out;
    bool ok = true;
    size_t nin = 0, nout = 0, nchunks = 0, next_j = 0;
    while (ok && pl.next(c, in, out)) {
        ++nchunks;
        ok = c.j0 == next_j && c.j1 >= c.j0 && c.in_used <= pl.in_need() && c.out_used <= pl.out_need() &&
             (c.j0 == 0 || c.j0 >= items.size() || items[c.j0].start);
        next_j = c.j1;
        std::fill(dev_in.begin(), dev_in.end(), 0xEE);
        for (const InXfer &t : in) {
            ++nin;
            for (size_t r = 0; ok && r < t.rows; ++r) {
                const size_t h = t.hoff + r * t.hpitch, d = t.doff + r * t.dpitch;
                ok = h + t.width <= src_bytes && d + t.width <= dev_in.size();
                for (size_t i = 0; ok && i < t.width; ++i) ok = readable[h + i] != 0;
                if (ok) std::memcpy(dev_in.data() + d, src.data() + h, t.width);
            }
        }
        std::fill(dev_out.begin(), dev_out.end(), 0xDD);
        for (size_t j = c.j0; ok && j < c.j1; ++j) {
            const Item &x = items[j];
            if (x.len) ok = din[j] + x.len <= dev_in.size() && !std::memcmp(dev_in.data() + din[j], src.data() + x.src, x.len);
            if (ok && x.copy) {
                ok = dout[j] + x.copy <= dev_out.size();
                if (ok) std::memcpy(dev_out.data() + dout[j], dev_in.data() + din[j], x.copy);
            }
        }
        for (const OutXfer &t : out) {
            ++nout;
            for (size_t r = 0; ok && r < t.rows; ++r) {
                uint8_t *h = t.h + r * t.hpitch;
                const size_t d = t.doff + r * t.dpitch;
                ok = h >= dst.data() && h + t.width <= dst.data() + dst.size() && d + t.width <= dev_out.size();
                if (ok) std::memcpy(h, dev_out.data() + d, t.width);
            }
        }
    }
    ok = ok && next_j == items.size() && dst == want;
    if (ok && want_in_xfers) ok = nin == want_in_xfers;
    if (ok && want_out_xfers) ok = nout == want_out_xfers;
    char tail[160];
    std::snprintf(tail, sizeof tail, " items %zu chunks %zu h2d %zu d2h %zu", items.size(), nchunks, nin, nout);
    report(name + tail, ok);
}

int main() {
    std::mt19937_64 rng(12345);
    // GM ring: 65,456-byte payloads 80 bytes apart in 64 KiB slots, delivered in order: one dense H2D
    // and one contiguous D2H per chunk
    {
        std::vector<Item> v;
        const size_t n = 300;
        for (size_t j = 0; j < n; ++j) v.push_back({72 + j * 65536, 65456, j * 65456, 65456, true});
        run("ring_gm_dense", v, n * 65536, true, 64u << 20, 1, 1);
        run("ring_gm_dense_small_chunks", v, n * 65536, true, 4u << 20);
    }
    // 4 KiB payloads in 64 KiB slots: one 2D H2D
    {
        std::vector<Item> v;
        for (size_t j = 0; j < 200; ++j) v.push_back({72 + j * 65536, 4096, j * 4096, 4096, true});
        run("ring_4k_pitch", v, 200 * 65536, true, 64u << 20, 1, 1);
    }
    // short payloads then long ones at one constant slot pitch: a 2D run must never widen its
    // rows past what the planner charged for its members (64 x 100 B then 65,456 B at a 64 KiB pitch once
    // made a 65-row run of 64 KiB rows in a ~426 KB chunk)
    {
        std::vector<Item> v;
        for (size_t j = 0; j < 64; ++j) v.push_back({72 + j * 65536, 100, j * 100, 100, true});
        v.push_back({72 + 64 * 65536, 65456, 6400, 65456, true});
        run("ring_pitch_short_then_long", v, 66 * 65536, true, 32u << 20);
        for (int rep = 0; rep < 20; ++rep) {
            std::vector<Item> w;
            const size_t n = 20 + rng() % 400;
            size_t apos = 0;
            for (size_t j = 0; j < n; ++j) {
                const uint64_t len = rng() % 3 ? 1 + rng() % 300 : 60000 + rng() % 5457;
                w.push_back({72 + j * 65536, len, apos, len, true});
                apos += len;
            }
            run("ring_pitch_mixed_" + std::to_string(rep), w, (n + 1) * 65536, true, (size_t)(1 + rng() % 32) << 20);
        }
    }
    // IB-shaped ring with ragged lengths, truncated copies (AppBufferLen <), skipped fragments
    for (int rep = 0; rep < 20; ++rep) {
        std::vector<Item> v;
        const size_t n = 50 + rng() % 3000, S = 2088;
        size_t apos = 0;
        for (size_t j = 0; j < n; ++j) {
            const uint64_t len = rng() % 10 == 0 ? rng() % 1977 : 1976;
            uint64_t copy = rng() % 7 == 0 ? rng() % (len + 1) : len;
            if (rng() % 13 == 0) copy = 0;
            const uint64_t l = copy ? len : (rng() % 2 ? len : 0);  // nothing to copy: nothing read either
            v.push_back({112 + j * S, copy ? l : 0, apos, copy, true});
            apos += copy + (rng() % 5 == 0 ? rng() % 100 : 0);
        }
        run("ring_ib_ragged_" + std::to_string(rep), v, n * S, true, (size_t)(1 + rng() % 4) << 20);
    }
    // shuffled ring fragments scattered anywhere
    for (int rep = 0; rep < 10; ++rep) {
        std::vector<Item> v;
        const size_t n = 400, S = 9000;
        std::vector<size_t> perm(n);
        for (size_t j = 0; j < n; ++j) perm[j] = j;
        std::shuffle(perm.begin(), perm.end(), rng);
        for (size_t j = 0; j < n; ++j) {
            const uint64_t len = 1 + rng() % 8900;
            v.push_back({perm[j] * S + rng() % (S - len), len, perm[n - 1 - j] * 9000, len, true});
        }
        run("ring_shuffled_" + std::to_string(rep), v, n * S, true, (size_t)(1 + rng() % 2) << 20);
    }
    // typemaps (strict rules): a strided vector of E-byte elements at stride S gathered into a packed
    // payload (send) and scattered back (receive); fragments of K elements, chunks only at fragment starts
    const size_t shapes[][3] = {{8, 16, 64}, {24, 40, 1000}, {100, 128, 333}, {1024, 1536, 64}, {4096, 8192, 16}};
    for (const auto &sh : shapes) {
        const size_t E = sh[0], S = sh[1], K = sh[2], n = 4000;
        std::vector<Item> g, s;
        for (size_t j = 0; j < n; ++j) {
            g.push_back({j * S, E, j * E, E, j % K == 0});  // gather: strided source, packed destination
            s.push_back({j * E, E, j * S, E, j % K == 0});  // scatter: packed source, strided destination
        }
        const std::string tag = "E" + std::to_string(E) + "_S" + std::to_string(S);
        run("vector_gather_" + tag, g, n * S, false, 64u << 20, 1, 1);
        run("vector_scatter_" + tag, s, n * E, false, 64u << 20, 1, 1);
        run("vector_gather_small_chunks_" + tag, g, n * S, false, 64u << 10);
    }
    // random typemaps: misaligned pieces of 1 B .. 20 KB in random places, checksum-only pieces
    for (int rep = 0; rep < 20; ++rep) {
        std::vector<Item> v;
        const size_t n = 1 + rng() % 2000;
        size_t pos = 0, dpos = 0;
        for (size_t j = 0; j < n; ++j) {
            const uint64_t len = rng() % 4 ? 1 + rng() % 64 : 200 + rng() % 20000;
            pos += rng() % 3 ? 0 : rng() % 50;  // touching or not
            const bool cp = rng() % 9 != 0;
            v.push_back({pos, len, dpos, cp ? len : 0, rng() % 17 == 0});
            pos += len;
            dpos += cp ? len + (rng() % 4 == 0 ? 3 : 0) : 0;
        }
        v[0].start = true;
        run("typemap_random_" + std::to_string(rep), v, pos + 64, false, (size_t)(16 + rng() % 512) << 10);
    }
    std::printf("bad %d done\n", g_bad);
    return g_bad != 0;
}
