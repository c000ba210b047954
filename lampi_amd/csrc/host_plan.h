// host_plan.h -- DMA planning for the host-memory batch paths of liblampi_csum.so (internal): the
// receive path (host_recv.cc, fragments in a NIC ring delivered to application buffers) and the
// typemap path (host_chain.cc, pieces of non-contiguous datatypes gathered / scattered with their
// chained checksums).
//
// A batch is a list of items, each reading `len` source bytes (checksummed) and writing `copy` of
// them to a host destination.  The planner walks the items in order and cuts them into pipeline
// chunks; inside a chunk it coalesces
//   * the source ranges into H2D transfers: touching or nearly touching ranges (when the source may
//     be read between items, i.e. inside one NIC ring) become one 1D copy, ranges at a constant pitch
//     one 2D copy, anything else a copy each;
//   * the destination ranges into D2H transfers: touching ranges one 1D copy, equal ranges at a
//     constant pitch one 2D copy, anything else a copy each;
// and gives every item its offsets in the chunk's device input and output buffers.  It runs one
// chunk ahead of the pipeline, so the first chunk's DMA starts while later chunks are planned.
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

#include "host_pipe.h"

namespace lampi {

// A DMA transfer: host (base + hoff) -> chunk (rows == 1: 1D of width bytes), or chunk -> host h.
struct InXfer {
    size_t hoff;    // source offset from the batch's base (the ring; 0 for absolute addresses)
    size_t width;   // bytes per row
    size_t rows;
    size_t hpitch;  // host bytes between rows (2D)
    size_t doff;    // offset in the input chunk
    size_t dpitch;
};
struct OutXfer {
    uint8_t *h;
    size_t width, rows, hpitch;
    size_t doff, dpitch;  // offset in the output chunk, device bytes between rows
};
struct ChunkPlan {
    size_t j0 = 0, j1 = 0;  // items [j0, j1)
    size_t in_used = 0, out_used = 0;
    uint64_t payload = 0;   // source bytes read (checksummed)
    size_t nread = 0;       // items with source bytes
    size_t ncopy = 0;       // items with bytes to write
};

// One item as the planner sees it.
struct PlanItem {
    uint64_t src;   // source offset from the base
    uint64_t len;   // source bytes read (0: none)
    uint8_t *dst;   // destination of the first `copy` bytes
    uint64_t copy;  // bytes written (0: none)
};

// What the source may be read as.  ring: inside one readable range of `ring_bytes` (a NIC ring), so a
// transfer may read between and past items; otherwise only the items' own bytes are read.
struct PlanRules {
    bool ring = false;
    size_t ring_bytes = 0;
    size_t pad_in() const;  // chunk bytes the planner charges per source item beyond its length
};

// Dense 1D runs may carry gaps of at most this many bytes each and 1/16 of their payload in all.
constexpr size_t kDenseGap = 4096;
// a 2D row's padding to 16 bytes and a run's 256-byte alignment fit in 272; a ring's dense gap on top
inline size_t PlanRules::pad_in() const { return 272 + (ring ? kDenseGap : 0); }

// The open run of source bytes being coalesced into one H2D transfer.
struct InRun {
    enum Kind { kNone, kOne, kDense, kPitch } kind = kNone;
    size_t lo = 0, end = 0;        // source range [lo, end) (1D kinds)
    size_t last = 0, pitch = 0;    // the last member's offset, the row pitch (kPitch)
    size_t width = 0;              // the widest member (kPitch rows)
    size_t gaps = 0, payload = 0;  // gap and payload bytes (kDense)
    size_t rows = 0;               // members
    size_t charge = 0;             // what the planner's capacity bound charged for the members
    size_t size() const {          // device bytes it needs
        if (kind == kNone) return 0;
        if (kind == kPitch) return rows * align_up(width, 16);
        return end - lo;
    }
    // The run with the range [o, o + len) appended, or kind kNone if it cannot take it.
    InRun extended(size_t o, size_t len, const PlanRules &R) const {
        InRun r = *this;
        r.charge += len + R.pad_in();
        const size_t maxgap = R.ring ? kDenseGap : 0;
        switch (kind) {
            case kNone:
                break;
            case kOne:
            case kDense:
                if (o >= end && o - end <= maxgap && (gaps + o - end) * 16 <= payload + len) {
                    r.kind = kDense;
                    r.gaps += o - end;
                    r.payload += len;
                    r.end = o + len;
                    r.last = o;
                    ++r.rows;
                    return r;
                }
                if (kind == kOne && o > last) {
                    // rows of the widest member's bytes: in a ring any row may read past its item;
                    // elsewhere only rows of one length
                    const size_t w = std::max(width, len);
                    const bool fits = R.ring ? o + w <= R.ring_bytes : len == width;
                    // rows widened to w must stay within the members' charge (short
                    // fragments then a long one at one slot pitch overran the chunk buffer)
                    if (fits && o - last >= w && 2 * align_up(w, 16) <= r.charge) {
                        r.kind = kPitch;
                        r.pitch = o - last;
                        r.width = w;
                        r.last = o;
                        r.rows = 2;
                        return r;
                    }
                }
                break;
            case kPitch: {
                const size_t w = std::max(width, len);
                const bool fits = R.ring ? o + w <= R.ring_bytes && len <= pitch : len == width;
                if (o > last && o - last == pitch && fits && (rows + 1) * align_up(w, 16) <= r.charge) {
                    r.width = w;
                    r.last = o;
                    ++r.rows;
                    return r;
                }
                break;
            }
        }
        r.kind = kNone;
        return r;
    }
    static InRun single(size_t o, size_t len, const PlanRules &R) {
        InRun r;
        r.kind = kOne;
        r.charge = len + R.pad_in();
        r.lo = r.last = o;
        r.end = o + len;
        r.width = r.payload = len;
        r.rows = 1;
        return r;
    }
};

// The open run of destination bytes being coalesced into one D2H transfer.
struct OutRun {
    enum Kind { kNone, kOne, kContig, kPitch } kind = kNone;
    uint8_t *start = nullptr, *end = nullptr;  // [start, end) (1D kinds)
    uint8_t *last = nullptr;                   // the last member's destination
    size_t pitch = 0, width = 0, rows = 0;
    size_t size() const {
        if (kind == kNone) return 0;
        if (kind == kPitch) return rows * align_up(width, 16);
        return (size_t)(end - start);
    }
    // the device offset of row r / address d within the run, relative to its start
    size_t offset_of(size_t r, const uint8_t *d) const {
        return kind == kPitch ? r * align_up(width, 16) : (size_t)(d - start);
    }
    OutRun extended(uint8_t *d, size_t c) const {
        OutRun r = *this;
        switch (kind) {
            case kNone:
                break;
            case kOne:
            case kContig:
                if (d == end) {
                    r.kind = kContig;
                    r.end = d + c;
                    r.last = d;
                    ++r.rows;
                    return r;
                }
                if (kind == kOne && d > last && c == width && (size_t)(d - last) >= c) {
                    r.kind = kPitch;
                    r.pitch = (size_t)(d - last);
                    r.last = d;
                    r.rows = 2;
                    return r;
                }
                break;
            case kPitch:
                if (d > last && (size_t)(d - last) == pitch && c == width) {
                    r.last = d;
                    ++r.rows;
                    return r;
                }
                break;
        }
        r.kind = kNone;
        return r;
    }
    static OutRun single(uint8_t *d, size_t c) {
        OutRun r;
        r.kind = kOne;
        r.start = r.last = d;
        r.end = d + c;
        r.width = c;
        r.rows = 1;
        return r;
    }
};

// Items: size(), get(j) -> PlanItem, boundary(j) -> a chunk may start at item j.
template <class Items>
class StreamPlanner {
  public:
    StreamPlanner(const Items &items, const PlanRules &rules, size_t cap, size_t *din, size_t *dout)
        : it_(items), R_(rules), cap_(cap), din_(din), dout_(dout), n_(items.size()) {
        // capacity bounds: a chunk closes once it would pass cap_ at an item where a chunk may start,
        // so it holds at most cap_ plus one indivisible group (each item adding at most its bytes, a
        // dense gap, a 2D row's padding and an alignment)
        uint64_t in_total = 0, out_total = 0, gin = 0, gout = 0, gin_max = 0, gout_max = 0;
        const uint64_t pad_in = R_.pad_in();
        for (size_t j = 0; j < n_; ++j) {
            if (it_.boundary(j)) gin = gout = 0;
            const PlanItem x = it_.get(j);
            const uint64_t a = x.len ? x.len + pad_in : 0, b = x.copy ? x.copy + 272 : 0;
            in_total += a;
            out_total += b;
            gin += a;
            gout += b;
            gin_max = std::max(gin_max, gin);
            gout_max = std::max(gout_max, gout);
        }
        in_need_ = std::max<uint64_t>(256, std::min<uint64_t>(cap_, in_total) + gin_max);
        out_need_ = std::max<uint64_t>(256, std::min<uint64_t>(cap_, out_total) + gout_max);
    }
    size_t in_need() const { return in_need_; }
    size_t out_need() const { return out_need_; }

    // The next chunk (items [c.j0, c.j1), its transfers), or false after the last one.  A batch
    // with nothing to move still has one chunk (no transfers).
    bool next(ChunkPlan &c, std::vector<InXfer> &in, std::vector<OutXfer> &out) {
        if (done_) return false;
        in.clear();
        out.clear();
        in_ = &in;
        out_ = &out;
        c = ChunkPlan{};
        c.j0 = j_;
        for (; j_ < n_; ++j_) {
            const size_t j = j_;
            const PlanItem x = it_.get(j);
            if (x.len == 0 && x.copy == 0) continue;
            InRun iext;
            if (x.len) iext = run_.extended(x.src, x.len, R_);
            const bool in_ext = iext.kind != InRun::kNone;
            const size_t in_total = !x.len ? in_base_ + run_.size()
                                    : in_ext ? in_base_ + iext.size()
                                             : align_up(in_base_ + run_.size(), 256) + x.len;
            OutRun oext;
            if (x.copy) oext = orun_.extended(x.dst, x.copy);
            const bool out_ext = oext.kind != OutRun::kNone;
            const size_t out_total = !x.copy ? out_base_ + orun_.size()
                                     : out_ext ? out_base_ + oext.size()
                                               : align_up(out_base_ + orun_.size(), 256) + x.copy;
            if (c.nread + c.ncopy > 0 && it_.boundary(j) && (in_total > cap_ || out_total > cap_)) {
                close_chunk(c, j);  // j opens the next chunk
                return true;
            }
            if (x.len) {
                if (in_ext) {
                    run_ = iext;
                } else {
                    close_in();
                    in_base_ = align_up(in_base_, 256);
                    run_ = InRun::single(x.src, x.len, R_);
                }
                members_.push_back(j);
                c.payload += x.len;
                ++c.nread;
            }
            if (x.copy) {
                if (out_ext) {
                    orun_ = oext;
                } else {
                    close_out();
                    out_base_ = align_up(out_base_, 256);
                    orun_ = OutRun::single(x.dst, x.copy);
                }
                omembers_.push_back(j);
                ++c.ncopy;
            }
        }
        close_chunk(c, n_);
        done_ = true;
        return true;
    }

  private:
    // the open input run becomes a transfer; its members get their chunk offsets
    void close_in() {
        if (run_.kind == InRun::kNone) return;
        InXfer x{};
        x.doff = in_base_;
        x.hoff = run_.lo;
        if (run_.kind == InRun::kPitch) {
            x.width = run_.width;
            x.rows = run_.rows;
            x.hpitch = run_.pitch;
            x.dpitch = align_up(run_.width, 16);
            for (size_t r = 0; r < members_.size(); ++r) din_[members_[r]] = x.doff + r * x.dpitch;
        } else {
            x.width = run_.end - run_.lo;
            x.rows = 1;
            x.hpitch = x.dpitch = x.width;
            for (size_t m : members_) din_[m] = x.doff + (it_.get(m).src - run_.lo);
        }
        in_->push_back(x);
        in_base_ += run_.size();
        run_ = InRun{};
        members_.clear();
    }
    void close_out() {
        if (orun_.kind == OutRun::kNone) return;
        OutXfer x{};
        x.h = orun_.start;
        x.doff = out_base_;
        if (orun_.kind == OutRun::kPitch) {
            x.width = orun_.width;
            x.rows = orun_.rows;
            x.hpitch = orun_.pitch;
            x.dpitch = align_up(orun_.width, 16);
        } else {
            x.width = (size_t)(orun_.end - orun_.start);
            x.rows = 1;
            x.hpitch = x.dpitch = x.width;
        }
        for (size_t r = 0; r < omembers_.size(); ++r)
            dout_[omembers_[r]] = out_base_ + orun_.offset_of(r, it_.get(omembers_[r]).dst);
        out_->push_back(x);
        out_base_ += orun_.size();
        orun_ = OutRun{};
        omembers_.clear();
    }
    void close_chunk(ChunkPlan &c, size_t j1) {
        close_in();
        close_out();
        c.j1 = j1;
        c.in_used = in_base_;
        c.out_used = out_base_;
        in_base_ = out_base_ = 0;
    }

    const Items &it_;
    PlanRules R_;
    size_t cap_;
    size_t *din_, *dout_;
    size_t n_;
    size_t in_need_ = 0, out_need_ = 0;
    size_t j_ = 0;
    bool done_ = false;
    std::vector<InXfer> *in_ = nullptr;
    std::vector<OutXfer> *out_ = nullptr;
    InRun run_;
    OutRun orun_;
    std::vector<size_t> members_, omembers_;
    size_t in_base_ = 0, out_base_ = 0;  // chunk bytes used before the open runs
};

// Issue a chunk's transfers.
inline hipError_t issue_in(const std::vector<InXfer> &v, const uint8_t *base, uint8_t *din, hipStream_t s) {
    for (const InXfer &t : v) {
        const uint8_t *h = (const uint8_t *)((uintptr_t)base + t.hoff);  // base 0: absolute addresses
        const hipError_t e = t.rows == 1
                                 ? hipMemcpyAsync(din + t.doff, h, t.width, hipMemcpyHostToDevice, s)
                                 : hipMemcpy2DAsync(din + t.doff, t.dpitch, h, t.hpitch, t.width, t.rows,
                                                    hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
inline hipError_t issue_out(const std::vector<OutXfer> &v, const uint8_t *dout, hipStream_t s) {
    for (const OutXfer &t : v) {
        const hipError_t e = t.rows == 1
                                 ? hipMemcpyAsync(t.h, dout + t.doff, t.width, hipMemcpyDeviceToHost, s)
                                 : hipMemcpy2DAsync(t.h, t.hpitch, dout + t.doff, t.dpitch, t.width, t.rows,
                                                    hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace lampi
