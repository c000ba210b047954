// frag_csum.hip -- gfx950 kernels for LA-MPI's per-fragment checksums.
//
// CRC mode (uicrc, ref src/util/MemFunctions.cc:1331-1367) -- one wavefront per fragment:
//   * The fragment is right-aligned in a frame of R rows of 4096 bytes (R = ceil(L/4096));
//     the P = 4096R - L leading frame bytes are zeros.  Leading zeros do not change a CRC
//     computed from a zero register, so every lane runs the same code.
//   * The caller's starting register (`partial`, 0xFFFFFFFF fresh) is XORed into the
//     first four message bytes (crc(s, B) = crc(0, B ^ bytes_BE(s)), |B| >= 4; the
//     |B| < 4 remainder s << 8|B| is added at the end).
//   * Lane l owns bytes [64l, 64l+64) of each row: 4 x dwordx4 loads (lane-contiguous,
//     measured as fast as fully coalesced rows on MI355X), slicing-by-4 CRC from a zero
//     register, table lookups in LDS addressed by one v_perm each.
//   * Between rows a lane's register jumps 4032 zero bytes (nibble-table shift, Horner).
//   * At the end lane l applies its own shift by 64*(63-l) bytes (per-lane nibble
//     tables, conflict-free) and the 64 registers are XOR-reduced across the wave (DPP).
//
// Scheduling (measured, tools/microbench/readocc.hip, readdyn.hip, crc_sched.hip): HBM reads
// run fastest when the chip sweeps memory as one compact window in address order.  So the
// grid is NOT persistent: 256-thread workgroups (4 waves) each own 4*fpw consecutive
// fragments and wave w takes fragments w, w+4, w+8, ...; the hardware dispatcher keeps the
// window compact and balances the load.  Persistent grids (static or atomic work queues)
// and 512/1024-thread workgroups measured 3-10% slower on raw reads.
//
// LDS (66048 B per workgroup -> two workgroups per CU), tables built per workgroup from a
// 12 KiB basis image (crc_tables.cc):
//   row e = 0..255 at e*256:
//     [0,128)    slicing tables, entry e of S_j, copy c = 0..7 at j*32 + 4c.  Lane octet g
//                (lanes 8g..8g+7 of a 32-lane ds_read_b32 group) reads table q^g in
//                instruction q -> 32 distinct banks, conflict-free; one v_perm forms the
//                address (byte0 = j*32+4c, byte1 = byte j of X).
//     [128,256)  per-lane combine tables: (p*16 + v)*2 + (l >> 5) is the row, lane l & 31
//                the word -> bank l % 32, conflict-free.
//   [65536, 66048)  Horner nibble tables (shift by 4032 bytes), p*64 + 4v (broadcast reads).
//
// SUM mode (uicsum, ref MemFunctions.cc:1073-1222): left-aligned rows, lane-contiguous
// 64-byte pieces, funnel-shifted to the fragment's own word grid, zero-padded tail,
// 32-bit adds reduced across the wave.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "crc_const.h"
#include "crc_tables.h"
#include "frag_csum_kernels.h"

// A/B knobs (tools/ab/*.sh): the schedule switches measured against each other are read from the environment
// only in the A/B build of the library (make AB=1: liblampi_csum_ab.so, -DLAMPI_AB_KNOBS=1, loaded by the A/B
// scripts through LAMPI_CSUM_LIB).  The default library compiles each to its measured default and reads only
// the documented switches (LAMPI_CSUM_NO_SHAPES here, LAMPI_HOST_CHUNK_BYTES in host_msg.cc); the knob names
// do not appear in it (tests/test_abi.py).
#if LAMPI_AB_KNOBS
#define LAMPI_AB_ENV(name) std::getenv(name)
#else
#define LAMPI_AB_ENV(name) (static_cast<const char *>(nullptr))
#endif

namespace lampi {

// per-stream device scratch (defined with the launchers)
static hipError_t stream_scratch(hipStream_t s, size_t bytes, void **out, bool *pooled);
static hipError_t scratch_done(hipStream_t s, void *p, bool pooled, hipError_t e);
static hipError_t pair_counters(hipStream_t s, uint32_t **cur, uint32_t **next);
static void reset_pair_counters(hipStream_t s);
static hipError_t scratch_done(hipStream_t s, void *p, bool pooled, hipError_t e);

namespace {

constexpr uint32_t kLdsHorner = 65536;
constexpr uint32_t kLdsBytes = 65536 + 512;
constexpr int kBlock = 256;
constexpr uint32_t kMaxWgGrid = 1u << 22;  // workgroups of a one-workgroup-per-item grid (x 256 threads < 2^32)
constexpr int kWaves = kBlock / 64;  // waves per workgroup

// Global-address-space byte pointer: keeps loads as global_load_* (flat loads would force
// vmcnt(0) + lgkmcnt(0) waits and defeat the prefetch).
typedef __attribute__((address_space(1))) const uint8_t gbyte;
typedef __attribute__((address_space(1))) uint8_t gbyte_w;  // global byte stores (not flat: a flat store
                                                            // pending makes every LDS wait lgkmcnt(0))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
typedef __attribute__((address_space(1))) const uint32_t guint;

typedef __attribute__((address_space(1))) uint8_t gwbyte;
typedef __attribute__((address_space(1))) uint32_t gwuint;
typedef __attribute__((address_space(1))) u32x4 gwu32x4;
// 16-byte stores to destinations that are only dword-aligned (GM ring slots after a 72-byte
// header): the type says 4-byte alignment, so the compiler assumes nothing more than the host
// gates guarantee; global_store_dwordx4 at a dword-aligned address runs at the aligned rate
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
typedef u32x4 u32x4_a1 __attribute__((aligned(1)));
typedef __attribute__((address_space(1))) const u32x4_a1 gu32x4_a1;  // unaligned 16-byte loads
typedef __attribute__((address_space(1))) u32x4_a4 gwu32x4_a4;

// Copy destinations are written with non-temporal stores (the `nt` bit: streamed past the caches
// the payload is not re-read from): +1.3 to +2 points of read + write bandwidth in the copy shapes
// measured (tools/microbench/copy5.hip, profiles/r02_copy5.txt).
// (The asm-issued row loads stay cached: with the nt bit, read-only CRC fell from 80.6% to 42.3%
// and config C from 73.6% to 44.1%; profiles/r02_sumcopy/ab_ntal/.)
#define LAMPI_ST_NT " nt"
__device__ __forceinline__ void st16(gwu32x4_a4 *p, const u32x4 &v) { __builtin_nontemporal_store(v, p); }
// source loads of the SUM copy kernels: non-temporal (read once; same-box A/B, profiles/r02_sumcopy/
// ab_ntl/: descriptors +1 to +2.5 points, messages, slots and +1 destinations +0.5 to +1.4)
__device__ __forceinline__ u32x4 ld16u(gu32x4_a1 *p) { return __builtin_nontemporal_load(p); }
// coalesced row loads of crc_rows_kernel (fused CRC copies of descriptors, the receive step,
// ragged messages): non-temporal, same-box A/B (profiles/r02_sumcopy/ab_cntl/) descriptors, +1
// destinations, the receive step and GM 65,456-byte slots +0.5 to +1 point.  The same bit on
// crc_regular_kernel<copy>'s asm loads cost 1.6-2.2 points there (not used).
__device__ __forceinline__ u32x4 ld16c(gu32x4_a1 *p) { return __builtin_nontemporal_load(p); }
typedef __attribute__((address_space(1))) u32x4_a1 gwu32x4_a1;  // unaligned 16-byte stores
__device__ __forceinline__ void st16u(gwu32x4_a1 *p, const u32x4 &v) { __builtin_nontemporal_store(v, p); }

struct FragInfo {
    gbyte *addr;
    uint32_t len;      // bytes checksummed
    uint32_t partial;
    uint8_t *dst;      // copy sources only: destination of the first copylen bytes
    uint32_t copylen;
    uint32_t aux = 0;  // receive sources: the expected checksum, loaded with the descriptor so its
                       // latency hides under the fragment's rows (emit compares against it)
};

// ---- fragment sources (wave-uniform) ----------------------------------------------
struct DescSource {
    static constexpr bool kCopy = false;
    static constexpr bool kPhase = false;  // SUM: partial & 3 is the byte phase (PieceSource only)
    const lampi_frag_desc *d;
    __device__ FragInfo get(size_t f) const {
        const lampi_frag_desc x = d[f];
        return {(gbyte *)(uintptr_t)x.addr, x.length, x.partial, nullptr, 0u};
    }
};

// bcopy_uicrc / bcopy_uicsum (ref MemFunctions.cc:1263-1321, 518-875): copy copylen bytes and
// checksum max(copylen, csumlen) bytes of the source (the residue is checksummed, not copied)
struct CopySource {
    static constexpr bool kCopy = true;
    static constexpr bool kPhase = false;
    const lampi_copy_desc *d;
    __device__ FragInfo get(size_t f) const {
        const lampi_copy_desc x = d[f];
        const uint32_t len = x.copylen > x.csumlen ? x.copylen : x.csumlen;
        return {(gbyte *)(uintptr_t)x.src, len, x.partial, (uint8_t *)(uintptr_t)x.dst, x.copylen};
    }
};

// A fused send copy with checksumming off (LAMPI_CSUM_NONE: doChecksum == false, ref
// src/path/gm/sendFrag.cc:153-155, :185-187, :206-208 -- MEMCOPY_FUNC instead of bcopy_uicrc / bcopy_uicsum):
// only the copylen bytes are read and copied; the SUM copy kernels run it and their sums go to scratch.
struct CopyOnlySource {
    static constexpr bool kCopy = true;
    static constexpr bool kPhase = false;
    const lampi_copy_desc *d;
    __device__ FragInfo get(size_t f) const {
        const lampi_copy_desc x = d[f];
        return {(gbyte *)(uintptr_t)x.src, x.copylen, 0u, (uint8_t *)(uintptr_t)x.dst, x.copylen};
    }
};

// host-path pieces of one chained 64-bit csum: partial = the piece's byte phase (0..7)
struct PhaseDescSource {
    static constexpr bool kCopy = false;
    static constexpr bool kPhase = true;
    const lampi_frag_desc *d;
    __device__ FragInfo get(size_t f) const {
        const lampi_frag_desc x = d[f];
        return {(gbyte *)(uintptr_t)x.addr, x.length, x.partial, nullptr, 0u};
    }
};

struct MsgSource {
    static constexpr bool kCopy = false;
    static constexpr bool kPhase = false;
    const uint8_t *base;
    size_t msg_len;
    size_t frag_len;
    uint32_t partial;
    __device__ FragInfo get(size_t f) const {
        size_t off = f * frag_len;
        size_t rem = msg_len - off;
        return {(gbyte *)(base + off), (uint32_t)(rem < frag_len ? rem : frag_len), partial, nullptr, 0u};
    }
};

// fragment k of a contiguous message copied to dst + k*dst_stride (bcopy of every fragment)
struct MsgCopySource {
    static constexpr bool kCopy = true;
    static constexpr bool kPhase = false;
    const uint8_t *base;
    size_t msg_len;
    size_t frag_len;
    uint32_t partial;
    uint8_t *dst;
    size_t dst_stride;
    __device__ FragInfo get(size_t f) const {
        size_t off = f * frag_len;
        size_t rem = msg_len - off;
        const uint32_t len = (uint32_t)(rem < frag_len ? rem : frag_len);
        return {(gbyte *)(base + off), len, partial, dst + f * dst_stride, len};
    }
};

// The 4 KiB rows of a message's fragments as items (SUM fused copies of fragments longer than a
// row, launch_msg_bcopy): item v is row v % rpf of fragment v / rpf, one short-lived workgroup
// each (sum_copy_wg_kernel: the textbook copy shape).  A row starts at a multiple
// of 4096 bytes into its fragment, on the fragment's word grid, so the fragment's uicsum is the
// sum of its rows' sums: emit adds them into out (zeroed first).  Rows past a short last
// fragment are empty.
struct MsgRowCopySource {
    static constexpr bool kCopy = true;
    static constexpr bool kPhase = false;
    const uint8_t *base;
    size_t msg_len;
    size_t frag_len;
    uint8_t *dst;
    size_t dst_stride;
    uint32_t rpf;  // rows per fragment, ceil(frag_len / 4096)
    __device__ FragInfo get(size_t v) const {
        const size_t f = v / rpf, r = v - f * rpf;
        const size_t off = f * frag_len + r * kRowBytes;
        const size_t fend = min(msg_len, (f + 1) * frag_len);
        const uint32_t len = off < fend ? (uint32_t)min((size_t)kRowBytes, fend - off) : 0u;
        return {(gbyte *)(base + off), len, 0u, dst + f * dst_stride + r * kRowBytes, len};
    }
};

// Row group g of fragment f (item v = f * W + g; LAMPI_CSUM_ROWS_HINT, SUM copies): the fragment's bytes
// [g k 4096, min((g + 1) k 4096, len)) with k = ceil(ceil(len / 4096) / W) -- every group starts on the
// fragment's word grid -- and the part of the copy inside them; groups past the fragment are empty.
// The kernel stores each group's sum at out[v] (scratch); sum_group_join_kernel adds them and emits.
template <class Src>
struct GroupSource {
    static constexpr bool kCopy = Src::kCopy;
    static constexpr bool kPhase = false;
    Src src;
    uint32_t W;
    __device__ FragInfo get(size_t v) const {
        const size_t f = v / W;
        const uint32_t g = (uint32_t)(v - f * W);
        FragInfo fi = src.get(f);
        const uint64_t R = ((uint64_t)fi.len + kRowBytes - 1) / kRowBytes, k = (R + W - 1) / W;
        const uint64_t a = min((uint64_t)g * k * kRowBytes, (uint64_t)fi.len);
        const uint64_t e = min(a + k * kRowBytes, (uint64_t)fi.len);
        const uint64_t ce = min(e, (uint64_t)fi.copylen);
        fi.addr += a;
        fi.len = (uint32_t)(e - a);
        fi.dst += a;
        fi.copylen = ce > a ? (uint32_t)(ce - a) : 0u;
        return fi;
    }
};

// One piece of a host call (lampi_uicrc / lampi_uicsum on at most kZeroCopy bytes) by value, so
// no descriptor is read back over PCIe; its result is followed by the host signal (emit).
struct HostOneSource {
    static constexpr bool kCopy = false;
    static constexpr bool kPhase = false;
    uint64_t addr;
    uint32_t len, partial;
    uint64_t *sig;  // host-coherent word the host polls (HostCtx::wait_done); seq is stored there
    uint64_t seq;
    __device__ FragInfo get(size_t) const { return {(gbyte *)(uintptr_t)addr, len, partial, nullptr, 0u}; }
};

// Tell a polling host that this kernel's results (already stored) are complete: a system-scope
// fence, then the sequence number with a system-scope release store (vector store).
__device__ __forceinline__ void signal_host(uint64_t *sig, uint64_t seq) {
    if (sig == nullptr) return;
    __threadfence_system();
    __hip_atomic_store(sig, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Typemap pieces of chained checksums (lampi_chain_csum_batch): pieces longer than `small`
// bytes; the others read as empty here and are done one thread per piece.  CRC values start
// from a zero register (the chain fold threads the caller's register); SUM values are taken at
// the piece's byte phase in its fragment's word grid (phase[k], partial-word chaining).
struct PieceSource {
    static constexpr bool kCopy = true;
    static constexpr bool kPhase = true;
    const lampi_copy_desc *d;
    const uint32_t *phase;  // SUM only (nullptr for CRC)
    uint32_t small;
    __device__ FragInfo get(size_t f) const {
        const lampi_copy_desc x = d[f];
        const uint32_t len = x.copylen > x.csumlen ? x.copylen : x.csumlen;
        if (len <= small) return {(gbyte *)(uintptr_t)x.src, 0u, 0u, nullptr, 0u};
        return {(gbyte *)(uintptr_t)x.src, len, phase ? phase[f] : 0u, (uint8_t *)(uintptr_t)x.dst, x.copylen};
    }
};

// RecvDesc_t::CopyToApp (ref src/path/common/BaseDesc.cc:288-342): copy lengthToCopy =
// min(length_m, AppBufferLen) bytes (none when AppBufferLen <= 0), checksum all length_m bytes
// (CopyFunction, gm/recvFrag.h:165-182: bcopy with copylen < csumlen), and -- where the kernel
// stores the checksum (emit) -- apply CheckData (gm/recvFrag.h:213-257) against the expected
// value.  A fragment with nothing to copy is not checksummed: CopyFunction returns the CRC
// initial register (or 0) for length 0 and CheckData passes it.
struct RecvSource {
    static constexpr bool kCopy = true;
    static constexpr bool kPhase = false;
    const lampi_recv_desc *d;
    uint32_t empty;            // CopyFunction of 0 bytes: 0xFFFFFFFF (CRC) or 0 (SUM)
    const uint8_t *expected;   // expected checksum of fragment f at expected + f * exp_stride
    size_t exp_stride;
    int64_t *copied;           // CopyToApp's return: lengthToCopy, or -1 when corrupt
    uint32_t *mask;            // bit f set when corrupt (zeroed by zero_verdicts_kernel first)
    uint32_t *nbad;
    __device__ static uint32_t to_copy(const lampi_recv_desc &x) {
        return x.app_len <= 0 ? 0u : (x.app_len < (int64_t)x.length ? (uint32_t)x.app_len : x.length);
    }
    __device__ FragInfo get(size_t f) const {
        // the expected value is read whatever the descriptor says (its record exists for every f),
        // so its load does not wait for the descriptor's
        const uint32_t e0 = *(const guint *)(expected + f * exp_stride);
        const lampi_recv_desc x = d[f];
        const uint32_t c = to_copy(x);
        const uint32_t e = c ? e0 : 0u;
        return {(gbyte *)(uintptr_t)x.frag, c ? x.length : 0u, empty, (uint8_t *)(uintptr_t)x.app, c, e};
    }
    __device__ void verdict(size_t f, uint32_t v, const FragInfo &fi) const {
        const uint32_t c = fi.copylen;
        const bool bad = c != 0u && v != fi.aux;
        copied[f] = bad ? -1ll : (int64_t)c;
        if (bad) {  // rare: one atomic per corrupt fragment
            atomicOr(mask + (f >> 5), 1u << (f & 31u));
            atomicAdd(nbad, 1u);
        }
    }
};

// CopyToApp with checksumming off (LAMPI_CSUM_NONE: the network's doChecksum == false, mpirun -mf/-if/-qf
// nochecksum, ref src/run/Input.cc:1986-2067): CopyFunction only copies and returns 0
// (src/path/gm/recvFrag.h:178-181), CheckData passes every fragment (:231-232).  Same copy as RecvSource, no
// expected value read; d_csum[f] = 0 and d_copied[f] = lengthToCopy (emit).
struct RecvCopyOnlySource : RecvSource {
    __device__ FragInfo get(size_t f) const {
        const lampi_recv_desc x = d[f];
        const uint32_t c = to_copy(x);
        return {(gbyte *)(uintptr_t)x.frag, c, 0u, (uint8_t *)(uintptr_t)x.app, c, 0u};
    }
    __device__ void verdict(size_t f, uint32_t, const FragInfo &fi) const { copied[f] = (int64_t)fi.copylen; }
};

// Read-only CRC descriptor batches of moderate size without a row-count hint run in two launches by
// size class (launch_crc_desc): fragments of 8-16 rows (GM's 65,456-byte payloads) on the table-light
// kernel, one wave each -- its best shape, 80% with the hint -- (SplitDescSource<true>), the rest on the
// piece streams (SplitDescSource<false>).  Each source reads a fragment of the other class as not its own
// (aux = 1): the light kernel's wave exits, the piece streams skip it and leave its out[] word alone.
__device__ __forceinline__ bool split_large(uint32_t len) { return len > 7u * kRowBytes && len <= 16u * kRowBytes; }
template <bool kLarge>
struct SplitDescSource {
    static constexpr bool kCopy = false;
    static constexpr bool kPhase = false;
    const lampi_frag_desc *d;
    __device__ FragInfo get(size_t f) const {
        const lampi_frag_desc x = d[f];
        if (split_large(x.length) != kLarge) return {(gbyte *)(uintptr_t)x.addr, 0u, 0u, nullptr, 0u, 1u};
        return {(gbyte *)(uintptr_t)x.addr, x.length, x.partial, nullptr, 0u};
    }
};
template <class S>
struct IsSplit : std::false_type {};
template <bool B>
struct IsSplit<SplitDescSource<B>> : std::true_type {};

// Small read-only CRC batches without a hint (launch_crc_desc): every fragment as W row groups, most of
// them empty for short fragments -- a workgroup whose four waves hold no rows leaves before staging tables.
struct SparseDescSource : DescSource {};
template <class S>
struct IsSparse : std::false_type {};
template <>
struct IsSparse<SparseDescSource> : std::true_type {};

template <class S>
struct IsRecv : std::false_type {};
template <>
struct IsRecv<RecvSource> : std::true_type {};
template <>
struct IsRecv<RecvCopyOnlySource> : std::true_type {};

// The receive step's verdicts zeroed by the launch before the one that gives them (row groups: the first
// launch, whose waves of group 0 zero the mask word of fragments f = 32i and f = 0 the count), instead of
// a kernel of its own (zero_verdicts_kernel, ~5 us in the stream).
__device__ __forceinline__ void zero_verdict_words(const RecvSource &src, size_t f) {
    if ((f & 31u) == 0) src.mask[f >> 5] = 0u;
    if (f == 0) *src.nbad = 0u;
}
template <class S>
struct IsGroupRecv : std::false_type {};
template <>
struct IsGroupRecv<GroupSource<RecvSource>> : std::true_type {};

// Byte-balanced descriptor batches (launch_crc_desc / launch_sum_desc for n <= kPlanMax): plan_kernel
// cuts every fragment longer than the plan's window B into segments of at most B bytes and groups the
// segments into workgroups by bytes, not by count.  A segment is checksummed like a fragment of its
// own -- CRC from the fragment's register (its first segment) or from 0 (the others), SUM from a fresh
// state -- and the kernel joins the parts of a split fragment: crc(s, A||B) = shift_|B|(crc(s, A)) ^
// crc(0, B), so each part is shifted past the rest of its fragment and XORed into out[f] (zeroed by
// the plan); sums simply add.  CRC segments are cut from the fragment's end (every shift is a whole
// number of 4 KiB rows), SUM segments from its start (every segment on the fragment's word grid).
struct SegDesc {
    uint32_t frag;  // the descriptor it belongs to
    uint32_t off;   // its first byte in the fragment (0: the fragment's first segment, which takes its register)
    uint32_t len;
    uint32_t rows;  // bit 31: the fragment is split; bits 0..30: 4 KiB rows of it after this segment (CRC)
};
static_assert(sizeof(SegDesc) == 16, "plan layout");
constexpr uint32_t kSegSplit = 1u << 31;

// (the plan reads only the lengths; address and register come from the descriptor itself)
struct SegSource {
    static constexpr bool kCopy = false;
    static constexpr bool kPhase = false;
    const SegDesc *s;
    const lampi_frag_desc *d;
    __device__ SegDesc segment(size_t j) const { return s[j]; }
    __device__ FragInfo get(size_t j) const {
        const SegDesc x = s[j];
        const lampi_frag_desc D = d[x.frag];
        return {(gbyte *)(uintptr_t)(D.addr + x.off), x.len, x.off == 0u ? D.partial : 0u, nullptr, 0u};
    }
};

template <class S>
struct IsSeg : std::false_type {};
template <>
struct IsSeg<SegSource> : std::true_type {};

// Row segments (LAMPI_CSUM_ROWS_HINT on lampi_frag_csum_batch): item v = f W + g is segment g of fragment f,
// its frame rows [g k, min((g + 1) k, R)) with R = ceil(L / 4096), k = ceil(R / W) -- CRC cut from the
// fragment's end (every segment but the first on a frame row boundary), SUM from its start -- computed on
// the device from the descriptor, no plan launch.  The launcher zeroes out; split fragments XOR (add) their
// shifted parts into it as the plan's segments do; items past a fragment's last segment are skipped.
constexpr uint32_t kSegSkip = 0xFFFFFFFFu;
struct RowSegSource {
    static constexpr bool kCopy = false;
    static constexpr bool kPhase = false;
    const lampi_frag_desc *d;
    uint32_t W;
    int sum;
    __device__ SegDesc segment(size_t v) const {
        const size_t f = v / W;
        const uint32_t g = (uint32_t)(v - f * W);
        const uint64_t L = d[f].length;
        const uint64_t R = (L + kRowBytes - 1) / kRowBytes;
        const uint64_t k = R ? (R + W - 1) / W : 1u, ng = R ? (R + k - 1) / k : 1u;
        if (g >= ng) return SegDesc{(uint32_t)f, 0u, 0u, kSegSkip};
        const uint64_t r1 = min((uint64_t)(g + 1) * k, R);
        uint64_t a, e;
        if (sum) {
            a = min((uint64_t)g * k * kRowBytes, L);
            e = min(r1 * kRowBytes, L);
        } else {
            const uint64_t P = R * kRowBytes - L;
            a = g ? (uint64_t)g * k * kRowBytes - P : 0u;
            e = r1 * kRowBytes - P;
        }
        const uint32_t rows = sum ? 0u : (uint32_t)(R - r1);
        return SegDesc{(uint32_t)f, (uint32_t)a, (uint32_t)(e - a), rows | (ng > 1 ? kSegSplit : 0u)};
    }
    __device__ FragInfo get(size_t v) const {
        const SegDesc x = segment(v);
        const lampi_frag_desc D = d[x.frag];
        return {(gbyte *)(uintptr_t)(D.addr + x.off), x.len, x.off == 0u ? D.partial : 0u, nullptr, 0u};
    }
};
// sources whose items are segments of fragments (the epilogue stores or joins by SegDesc)
template <class S>
struct HasSegments : IsSeg<S> {};
template <>
struct HasSegments<RowSegSource> : std::true_type {};

// every kernel stores a fragment's checksum through this: receive sources also decide it
template <class Src, class Acc>
__device__ __forceinline__ void emit(const Src &src, Acc *out, size_t f, Acc v, const FragInfo &fi) {
    if constexpr (std::is_same<Src, HostOneSource>::value) {  // the host call's one result, then the signal
        out[f] = v;
        signal_host(src.sig, src.seq);
        return;
    }
    if constexpr (std::is_same<Src, MsgRowCopySource>::value) {  // a row's part of its fragment's sum
        if (v != 0) atomicAdd(out + f / src.rpf, v);
        return;
    }
    if constexpr (IsSplit<Src>::value)
        if (fi.aux) return;  // the other launch's fragment
    if constexpr (std::is_same<Src, RecvCopyOnlySource>::value) v = 0;  // no checksum with checksumming off
    out[f] = v;
    if constexpr (IsRecv<Src>::value) src.verdict(f, v, fi);
}

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t lds_u32(const uint32_t *lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(lds) + byte_addr);
}

// ---- asm-issued loads ----------------------------------------------------------------
// Hot-loop loads are issued by inline asm and waited for by an explicit s_waitcnt that
// threads the destination registers through as in/out operands, so no use can be
// scheduled above the wait.  hipcc's waitcnt pass merges loop-carried load state
// conservatively (it waited for two rows where one was needed) and cannot see asm loads;
// the loads the compiler emits itself are older than or independent of these, and a
// younger compiler store only makes a wait stricter, never unsafe.
struct Row {
    u32x4 q[4];
};

// the lane's four 16-byte chunks at p, p + kS, p + 2kS, p + 3kS (kS = 16: one contiguous
// 64-byte piece; kS = 1024: the coalesced layout, every instruction covers 1 KiB of the row)
template <int kS = 16>
__device__ __forceinline__ void issue_row(gbyte *p, Row &r) {
    asm volatile(
        "global_load_dwordx4 %0, %4, off\n\t"
        "global_load_dwordx4 %1, %4, off offset:%5\n\t"
        "global_load_dwordx4 %2, %4, off offset:%6\n\t"
        "global_load_dwordx4 %3, %4, off offset:%7"
        : "=&v"(r.q[0]), "=&v"(r.q[1]), "=&v"(r.q[2]), "=&v"(r.q[3])
        : "v"(p), "n"(kS), "n"(2 * kS), "n"(3 * kS)
        : "memory");
}

template <int N>
__device__ __forceinline__ void wait_row(Row &r) {
    asm volatile("s_waitcnt vmcnt(%4) ; lampi-wait %0 %1 %2 %3" : "+v"(r.q[0]), "+v"(r.q[1]), "+v"(r.q[2]), "+v"(r.q[3]) : "n"(N) : "memory");
}

__device__ __forceinline__ u32x4 issue_b128(gbyte *p) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(v) : "v"(p) : "memory");  // the L2-resident basis
    return v;
}

__device__ __forceinline__ void row_words(const Row &r, uint32_t d[16]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        d[4 * k + 0] = r.q[k].x;
        d[4 * k + 1] = r.q[k].y;
        d[4 * k + 2] = r.q[k].z;
        d[4 * k + 3] = r.q[k].w;
    }
}

// 4 x dwordx4 stores of a lane's 64-byte piece.  Stores count in vmcnt in issue order with
// the loads (MI355X_MICROARCH.md, s_waitcnt), so the ring's wait counts include them.  The
// trailing s_nop covers the store-data read hazard before the registers are rewritten.
template <int kS = 16>
__device__ __forceinline__ void store_row(gwbyte *p, const Row &r) {
    asm volatile(
        "global_store_dwordx4 %0, %1, off" LAMPI_ST_NT "\n\t"
        "global_store_dwordx4 %0, %2, off offset:%5" LAMPI_ST_NT "\n\t"
        "global_store_dwordx4 %0, %3, off offset:%6" LAMPI_ST_NT "\n\t"
        "global_store_dwordx4 %0, %4, off offset:%7" LAMPI_ST_NT "\n\t"
        "s_nop 1"
        :
        : "v"(p), "v"(r.q[0]), "v"(r.q[1]), "v"(r.q[2]), "v"(r.q[3]), "n"(kS), "n"(2 * kS), "n"(3 * kS)
        : "memory");
}

// ---- LDS table staging --------------------------------------------------------------
// The slicing and Horner tables are built from compile-time constants (crc_const.h): no
// memory wait.  Only the per-lane combine tables come from the basis image (64 lanes x 32
// columns, 8 KiB, L2-resident): two dwordx4 loads per thread, issued before anything else so
// their latency overlaps the rows the workgroup issues next (`pre`) and the constant builds.
// kParts: bit 0 slicing, bit 1 combine, bit 2 Horner tables (the piece streams need no Horner
// tables).
constexpr cx::SliceBasis kSliceBasis = cx::slice_basis();
constexpr cx::Mat kHornerMat = cx::swapped(cx::shift(kRowBytes - kLaneBytes));  // 4032 bytes
constexpr cx::Mat kHorner16Mat = cx::swapped(cx::shift(kChunkStep));           // 1008 bytes

__device__ __forceinline__ uint32_t sel4(uint32_t s, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return (s & 2u) ? ((s & 1u) ? d : c) : ((s & 1u) ? b : a);
}

struct CombineBasis {
    u32x4 a, b;  // columns 4*p0 .. +3 and 4*(p0 + 4) .. +3 of lane t & 63, p0 = t >> 6
};

template <bool kCoal = false>
__device__ __forceinline__ CombineBasis issue_combine_basis(const uint32_t *__restrict__ img) {
    constexpr size_t kComb = kCoal ? kImgCombine16Cols : kImgCombineCols;
    const uint32_t t = threadIdx.x, l = t & 63u, p0 = t >> 6;
    gbyte *g = (gbyte *)img;
    CombineBasis cb;
    cb.a = issue_b128(g + 4 * (kComb + l * 32 + 4 * p0));
    cb.b = issue_b128(g + 4 * (kComb + l * 32 + 4 * (p0 + 4)));
    return cb;
}

// slicing tables: thread t fills 16-byte slot t & 7 (copies 4*(t&1) .. +3 of S_j, j = (t&7) >> 1)
// of rows (t >> 3) + 32k, k = 0..7; consecutive lanes write consecutive slots (a thread-per-row
// fill put every lane of a ds_write_b128 on the same banks: 1.2 us per workgroup, measured).
// S_j[r0 + 32k] = S_j[r0] ^ S_j[32k] by linearity.
__device__ __forceinline__ void build_slices(char *b) {
    const uint32_t t = threadIdx.x;
    const uint32_t sj = (t & 7u) >> 1, r0 = t >> 3;
    uint32_t base = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t k = sel4(sj, kSliceBasis.lo[0][i], kSliceBasis.lo[1][i], kSliceBasis.lo[2][i],
                                kSliceBasis.lo[3][i]);
        base ^= ((r0 >> i) & 1u) ? k : 0u;
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
        const uint32_t v = base ^ sel4(sj, kSliceBasis.hi[0][kk], kSliceBasis.hi[1][kk], kSliceBasis.hi[2][kk],
                                       kSliceBasis.hi[3][kk]);
        *reinterpret_cast<u32x4 *>(b + (r0 + 32 * kk) * 256 + (t & 7u) * 16) = u32x4{v, v, v, v};
    }
}

// Horner nibble tables at kLdsHorner + p*64 + 4v: wave w builds p = w and w + 4 (lanes 0..15)
template <bool kCoal = false>
__device__ __forceinline__ void build_horner(char *b) {
    const uint32_t t = threadIdx.x, w = t >> 6, v = t & 63u;
    if (v >= 16) return;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        if ((uint32_t)(p & 3) != w) continue;
        uint32_t e = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t col = kCoal ? kHorner16Mat.c[4 * p + i] : kHornerMat.c[4 * p + i];
            e ^= ((v >> i) & 1u) ? col : 0u;
        }
        *reinterpret_cast<uint32_t *>(b + kLdsHorner + p * 64 + v * 4) = e;
    }
}

// combine entries (l, p, v) = XOR of columns 4p+bit for the set bits of v
__device__ __forceinline__ void build_combine(char *b, const CombineBasis &cb) {
    const uint32_t t = threadIdx.x, l = t & 63u, p0 = t >> 6;
    const uint32_t lane_base = (l >> 5) * 256 + 128 + (l & 31u) * 4;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const u32x4 c = h ? cb.b : cb.a;
        const uint32_t p = p0 + 4 * h;
#pragma unroll
        for (uint32_t v = 0; v < 16; ++v) {
            uint32_t e = 0;
            if (v & 1) e ^= c.x;
            if (v & 2) e ^= c.y;
            if (v & 4) e ^= c.z;
            if (v & 8) e ^= c.w;
            *reinterpret_cast<uint32_t *>(b + p * 8192 + v * 512 + lane_base) = e;
        }
    }
}

// LDS-only barrier: a __syncthreads() would also wait for the asm-issued row loads
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Issues the combine basis, lets `pre` issue kPre more asm loads (the first rows of the
// workgroup), builds the constant tables, waits for the basis only (vmcnt(kPre)), builds the
// combine tables and ends with an LDS-only barrier.
// kLatePre: `pre` runs after the slicing tables are built (the rows' addresses wait for loads issued before).
template <int kPre, class Pre, int kParts = 7, bool kCoal = false, bool kSync = true, bool kLatePre = false>
__device__ __forceinline__ void stage_tables(uint32_t *lds, const uint32_t *__restrict__ img, Pre pre) {
    CombineBasis cb = issue_combine_basis<kCoal>(img);
    if (!kLatePre) pre();
    char *b = reinterpret_cast<char *>(lds);
    if (kParts & 1) build_slices(b);
    if (kLatePre) pre();
    if (kParts & 4) build_horner<kCoal>(b);
    asm volatile("s_waitcnt vmcnt(%2) ; lampi-wait %0 %1" : "+v"(cb.a), "+v"(cb.b) : "n"(kPre) : "memory");
    if (kParts & 2) build_combine(b, cb);
    if (kSync) lds_barrier();
}

// ---- loads --------------------------------------------------------------------------
// Load the 64 bytes at signed offset o (relative to frag) into d[16] as LE words.
// Bytes at offsets < lo or >= hi read as zero; nothing outside [lo, hi) is dereferenced
// except within aligned 16-byte chunks that hold at least one byte inside (same page).
// `mask` selects whether any masking can be needed (wave-uniform).
__device__ __forceinline__ uint32_t byte_keep_mask(long long ow, long long lo, long long hi) {
    // keep byte j of the word at offset ow iff lo <= ow + j < hi
    long long a = lo - ow;  // bytes to drop at the bottom
    long long b = ow + 4 - hi;  // bytes to drop at the top
    uint32_t m = 0xFFFFFFFFu;
    if (a >= 4 || b >= 4) return 0;
    if (a > 0) m <<= 8 * a;
    if (b > 0) m &= 0xFFFFFFFFu >> (8 * b);
    return m;
}

__device__ __forceinline__ void load64(gbyte *frag, long long o, long long lo, long long hi,
                                       bool mask, uint32_t s16, uint32_t d[16]) {
    if (s16 != 0 && !mask) {
        // misaligned, every byte inside [lo, hi): four unaligned 16-byte loads (one
        // global_load_dwordx4 each; the memory pipeline splits them at line boundaries).  A plain
        // copy from 8-byte-aligned GM slot payloads runs at the aligned rate this way
        // (profiles/r02_copy_lds.txt, SLOT gather); the five aligned chunks + funnel shift below
        // cost one more load and 16 v_alignbyte per row.
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 v = *(gu32x4_a1 *)(frag + o + 16 * k);
            d[4 * k + 0] = v.x;
            d[4 * k + 1] = v.y;
            d[4 * k + 2] = v.z;
            d[4 * k + 3] = v.w;
        }
        return;
    }
    if (s16 == 0) {
        // 16-byte aligned chunks
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            long long c = o + 16 * k;
            u32x4 v = {0u, 0u, 0u, 0u};
            if (!mask || (c + 16 > lo && c < hi))
                v = *(gu32x4 *)(frag + c);
            d[4 * k + 0] = v.x;
            d[4 * k + 1] = v.y;
            d[4 * k + 2] = v.z;
            d[4 * k + 3] = v.w;
        }
    } else {
        // not 16-byte aligned ((frag + o) % 16 == s16, the same for every lane): the five aligned
        // 16-byte chunks covering [o, o + 64), funnel-shifted (word offset s16 / 4 is wave-uniform:
        // a switch; byte shift s16 % 4 by v_alignbyte).  A chunk holding a byte of [lo, hi) never
        // crosses a page.  (Seventeen dword loads per lane ran the misaligned fused copy at 32%.)
        const long long cb = o - (long long)s16;
        uint32_t a[20];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const long long c = cb + 16 * k;
            u32x4 v = {0u, 0u, 0u, 0u};
            if (c + 16 > lo && c < hi) v = *(gu32x4 *)(frag + c);
            a[4 * k + 0] = v.x;
            a[4 * k + 1] = v.y;
            a[4 * k + 2] = v.z;
            a[4 * k + 3] = v.w;
        }
        const uint32_t sb = s16 & 3u;
        switch (s16 >> 2) {  // wave-uniform
#define LAMPI_LOAD64_CASE(W)                                                                 \
    case W:                                                                                  \
        _Pragma("unroll") for (int w = 0; w < 16; ++w) d[w] =                                \
            __builtin_amdgcn_alignbyte(a[w + (W) + 1], a[w + (W)], sb);                      \
        break;
            LAMPI_LOAD64_CASE(0)
            LAMPI_LOAD64_CASE(1)
            LAMPI_LOAD64_CASE(2)
            LAMPI_LOAD64_CASE(3)
#undef LAMPI_LOAD64_CASE
        }
    }
    if (mask) {
#pragma unroll
        for (int w = 0; w < 16; ++w) d[w] &= byte_keep_mask(o + 4 * w, lo, hi);
    }
}

// ---- stores (fused copy) --------------------------------------------------------------
// Aligned word at dst + c: whole-word store when all four bytes lie in [lo, hi), byte stores
// for a word straddling an edge, nothing outside.
__device__ __forceinline__ void store_word(uint8_t *dst, long long c, uint32_t v, long long lo, long long hi) {
    if (c >= lo && c + 4 <= hi) {
        *(gwuint *)(dst + c) = v;
    } else if (c + 4 > lo && c < hi) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (c + j >= lo && c + j < hi) *(gwbyte *)(dst + c + j) = (uint8_t)(v >> (8 * j));
    }
}

// Write the 64 bytes d[16] (bytes [o, o+64) of the frame) to dst + o, keeping only bytes in
// [lo, hi).  m = (dst + o) & 3 and a16 = ((dst + o) & 15) == 0 are wave-uniform.  For m != 0 a
// lane writes the aligned words covering [o - m, o - m + 64): their first m bytes are the top
// of the previous lane's piece (`prev`), and the lane holding the frame's last piece (`tail`)
// also writes the word at o - m + 64.
__device__ __forceinline__ void store64(uint8_t *dst, long long o, const uint32_t d[16], long long lo, long long hi,
                                        uint32_t m, bool a16, uint32_t prev, bool tail) {
    if (o - (long long)m >= hi || o + 64 <= lo) return;
    if (m == 0) {
        if (a16 && o >= lo && o + 64 <= hi) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                st16((gwu32x4_a4 *)(dst + o + 16 * k), u32x4{d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]});
            return;
        }
#pragma unroll
        for (int w = 0; w < 16; ++w) store_word(dst, o + 4 * w, d[w], lo, hi);
        return;
    }
    const long long a = o - (long long)m;
    const uint32_t sh = 4u - m;
    store_word(dst, a, __builtin_amdgcn_alignbyte(d[0], prev, sh), lo, hi);
#pragma unroll
    for (int w = 1; w < 16; ++w) store_word(dst, a + 4 * w, __builtin_amdgcn_alignbyte(d[w], d[w - 1], sh), lo, hi);
    if (tail) store_word(dst, a + 64, __builtin_amdgcn_alignbyte(0u, d[15], sh), lo, hi);
}

// A whole 4 KiB row (lane l holds bytes [64l, 64l+64)) to a 4-byte-aligned dst with
// 1 KiB-coalesced stores: each quarter row goes through the wave's kStage-byte LDS area (its 16
// lanes write their 64 bytes, every lane reads back the 16-byte chunk at 16l and stores it).
// Lane-contiguous 64-byte stores run at 51% of the HBM roofline against 71% for coalesced ones
// (profiles/r01_copy_patterns.txt); dword-aligned dwordx4 stores (dst % 16 = 4, 8, 12) run at
// the aligned rate (dst + 8: 68%, against 61% for staging destination-aligned chunks with
// carried bytes and 21% for word stores).  LDS operations of one wave complete in order, so the
// area is reused without a barrier; the asm fences only keep the compiler from reordering them.
template <uint32_t kStage>
__device__ __forceinline__ void store_row_coalesced(uint32_t *stage, uint8_t *dst, const uint32_t d[16], int lane,
                                                    bool skip0 = false) {
    static_assert(kStage == 1024 || kStage == 2048, "half- or quarter-row staging");
    constexpr int kParts = kRowBytes / kStage;  // lanes 64/kParts per part
    constexpr int kLanes = 64 / kParts;
    constexpr int kRd = kStage / 1024;          // 1 KiB reads (and stores) per part
    u32x4 *st = (u32x4 *)stage;
#pragma unroll
    for (int h = 0; h < kParts; ++h) {
        if (lane / kLanes == h) {
            const int b = (lane % kLanes) * 4;
#pragma unroll
            for (int q = 0; q < 4; ++q) st[b + q] = u32x4{d[4 * q], d[4 * q + 1], d[4 * q + 2], d[4 * q + 3]};
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        u32x4 v[kRd];
#pragma unroll
        for (int i = 0; i < kRd; ++i) v[i] = st[64 * i + lane];
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < kRd; ++i) {
            gwbyte *c = (gwbyte *)(dst + h * kStage + 1024 * i + 16 * lane);
            if (h == 0 && i == 0 && lane == 0 && skip0) {  // the row's first word is the caller's
                *(gwuint *)(c + 4) = v[i].y;
                *(gwuint *)(c + 8) = v[i].z;
                *(gwuint *)(c + 12) = v[i].w;
            } else {
                st16((gwu32x4_a4 *)c, v[i]);  // dst is 4-byte aligned (dword-aligned dwordx4 store)
            }
        }
    }
}

// A row only partly inside the copy [lo, hi) (offsets relative to dst; the row's byte 0 at row0,
// dst + row0 dword-aligned): the same 1 KiB-coalesced staging as store_row_coalesced; a lane's
// 16-byte chunk goes out whole when it lies inside, word by word (store_word: whole words, bytes
// at an edge) when it straddles an edge, not at all outside.  Edge rows written lane by lane with
// dword stores (16 instructions touching 64 lines each) ran GM's 65,456-byte slot copies at
// about 51% of read + write.
__device__ __forceinline__ void store_row_coalesced_masked(uint32_t *stage, uint8_t *dst, long long row0,
                                                           const uint32_t d[16], int lane, long long lo, long long hi) {
    u32x4 *st = (u32x4 *)stage;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        if (lane / 16 == h) {
            const int b = (lane % 16) * 4;
#pragma unroll
            for (int q = 0; q < 4; ++q) st[b + q] = u32x4{d[4 * q], d[4 * q + 1], d[4 * q + 2], d[4 * q + 3]};
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        const u32x4 v = st[lane];
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const long long c = row0 + h * 1024 + 16 * lane;
        if (c >= lo && c + 16 <= hi) {
            st16((gwu32x4_a4 *)(dst + c), v);
        } else if (c + 16 > lo && c < hi) {
            store_word(dst, c, v.x, lo, hi);
            store_word(dst, c + 4, v.y, lo, hi);
            store_word(dst, c + 8, v.z, lo, hi);
            store_word(dst, c + 12, v.w, lo, hi);
        }
    }
}

// The reverse: a row loaded coalesced (lane l holds the 16-byte chunks at 16l + 1024q) into the
// lane-contiguous pieces the CRC runs on (lane l: bytes [64l, 64l + 64)), through the wave's 1 KiB
// staging area one quarter row at a time (every lane writes its chunk of quarter q, the 16 lanes
// whose pieces lie in it read them back).  One wave's LDS operations complete in order: no barrier.
__device__ __forceinline__ void rows_to_pieces(uint32_t *stage, uint32_t d[16], int lane) {
    u32x4 *st = (u32x4 *)stage;
    uint32_t e[16];
#pragma unroll
    for (int w = 0; w < 16; ++w) e[w] = 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        st[lane] = u32x4{d[4 * q], d[4 * q + 1], d[4 * q + 2], d[4 * q + 3]};
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        if ((lane >> 4) == q) {
            const int b = (lane & 15) * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 v = st[b + k];
                e[4 * k + 0] = v.x;
                e[4 * k + 1] = v.y;
                e[4 * k + 2] = v.z;
                e[4 * k + 3] = v.w;
            }
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int w = 0; w < 16; ++w) d[w] = e[w];
}

// d[15] of lane - 1 (lane 0 gets `carry`, the last lane's word of the previous row)
__device__ __forceinline__ uint32_t prev_lane_top(uint32_t d15, uint32_t carry, int lane) {
    const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((lane - 1) * 4, (int)d15);
    return lane == 0 ? carry : v;
}

// ---- CRC pieces -----------------------------------------------------------------------
struct CrcLane {
    uint32_t lanec;      // byte j: j*32 + 4c, the low LDS address byte of table j, copy c = lane & 7
    uint32_t sel[4];     // v_perm selectors: byte0 <- lanec.byte(j), byte1 <- X.byte(j), j = q ^ octet
    uint32_t comb_base;  // (l >> 5)*256 + 128 + 4*(l & 31): this lane's combine-table column
};

__device__ __forceinline__ CrcLane make_lane(int lane) {
    CrcLane k;
    const uint32_t c4 = (uint32_t)(lane & 7) * 4u;
    k.lanec = c4 | ((c4 + 32u) << 8) | ((c4 + 64u) << 16) | ((c4 + 96u) << 24);
    const uint32_t g = (uint32_t)(lane >> 3) & 3u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t j = (uint32_t)q ^ g;
        k.sel[q] = j | ((4u + j) << 8) | 0x0C0C0000u;
    }
    k.comb_base = ((uint32_t)lane >> 5) * 256u + 128u + ((uint32_t)lane & 31u) * 4u;
    return k;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32: a ^ b ^ c
}

// slicing-by-4 lookups of X (swapped domain): one v_perm + one ds_read_b32 each
struct Look4 {
    uint32_t t0, t1, t2, t3;
};
__device__ __forceinline__ Look4 look4(const uint32_t *lds, const CrcLane &k, uint32_t X) {
    Look4 r;
    r.t0 = lds_u32(lds, __builtin_amdgcn_perm(X, k.lanec, k.sel[0]));
    r.t1 = lds_u32(lds, __builtin_amdgcn_perm(X, k.lanec, k.sel[1]));
    r.t2 = lds_u32(lds, __builtin_amdgcn_perm(X, k.lanec, k.sel[2]));
    r.t3 = lds_u32(lds, __builtin_amdgcn_perm(X, k.lanec, k.sel[3]));
    return r;
}

// register C (swapped domain) through the 16 words of a lane's 64-byte piece:
// per word 4 v_perm + 4 ds_read_b32 + 2 v_bitop3 (the next word's data XOR is fused)
__device__ __forceinline__ uint32_t crc_piece(const uint32_t *lds, const CrcLane &k, uint32_t C,
                                              const uint32_t d[16]) {
    uint32_t X = C ^ d[0];
#pragma unroll
    for (int w = 0; w < 15; ++w) {
        const Look4 t = look4(lds, k, X);
        X = xor3(xor3(t.t0, t.t1, t.t2), t.t3, d[w + 1]);
    }
    const Look4 t = look4(lds, k, X);
    return xor3(t.t0, t.t1, t.t2) ^ t.t3;
}

// shift by 4032 zero bytes (all lanes read the same 16-entry tables: conflict free)
__device__ __forceinline__ uint32_t horner_shift(const uint32_t *lds, uint32_t C) {
    uint32_t r = lds_u32(lds, kLdsHorner | ((C << 2) & 0x3Cu));
#pragma unroll
    for (int p = 1; p < 8; ++p) r ^= lds_u32(lds, (kLdsHorner | ((C >> (4 * p - 2)) & 0x3Cu)) + p * 64);
    return r;
}

// lane l: shift by 64*(63-l) zero bytes (lane-private nibble tables, bank l % 32)
__device__ __forceinline__ uint32_t lane_combine(const uint32_t *lds, const CrcLane &k, uint32_t C) {
    const uint32_t b = k.comb_base;
    uint32_t r = lds_u32(lds, ((C << 9) & 0x1E00u) | b);
    r ^= lds_u32(lds, (((C << 5) & 0x1E00u) | b) + 8192);
    r ^= lds_u32(lds, (((C << 1) & 0x1E00u) | b) + 2 * 8192);
#pragma unroll
    for (int p = 3; p < 8; ++p) r ^= lds_u32(lds, (((C >> (4 * p - 9)) & 0x1E00u) | b) + p * 8192);
    return r;
}

// XOR of v over each row of 16 lanes (every lane of the row gets it): DPP butterflies.
__device__ __forceinline__ uint32_t row16_xor(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
    return v;
}

// XOR of v over the 64 lanes: the four row XORs combined by readlane.
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
    v = row16_xor(v);
    return __builtin_amdgcn_readlane(v, 0) ^ __builtin_amdgcn_readlane(v, 16) ^ __builtin_amdgcn_readlane(v, 32) ^
           __builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ uint32_t wave_add(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}

// XOR / sum of v over each group of kSub consecutive lanes (kSub = 1 .. 32, a power of two): the DPP
// butterflies of row16_xor cut after log2(kSub) levels -- every lane of a group of <= 16 gets the group's
// value -- and for 32, row_bcast:15 into rows 1 and 3 (their lanes, 31 and 63 among them, get it).
template <int kSub, bool kAdd>
__device__ __forceinline__ uint32_t group_reduce(uint32_t v) {
    static_assert(kSub >= 1 && kSub <= 32 && (kSub & (kSub - 1)) == 0, "groups of 1..32 lanes");
    auto op = [](uint32_t a, uint32_t b) { return kAdd ? a + b : a ^ b; };
    if constexpr (kSub >= 2) v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
    if constexpr (kSub >= 4) v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
    if constexpr (kSub >= 8) v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
    if constexpr (kSub >= 16) v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));
    if constexpr (kSub >= 32) v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
    return v;
}

// Fragments of a workgroup: wave w of workgroup b takes fragments b*4*fpw + w + 4i, i < fpw.
__device__ __forceinline__ uint32_t wg_first(uint32_t fpw) {
    return uniform(blockIdx.x * kWaves * fpw + (threadIdx.x >> 6));
}

struct RowGeom {
    uint32_t R;    // rows
    uint32_t P;    // frame padding in front of byte 0
    uint32_t s16;  // (addr - P) mod 16, the chunk misalignment (same for every lane)
};

__device__ __forceinline__ RowGeom crc_geom(const FragInfo &fi) {
    RowGeom g;
    g.R = (uint32_t)(((uint64_t)fi.len + (kRowBytes - 1)) / kRowBytes);
    g.P = g.R * kRowBytes - fi.len;
    g.s16 = (uint32_t)(((uintptr_t)fi.addr - g.P) & 15u);
    return g;
}

__device__ __forceinline__ void crc_load_row(const FragInfo &fi, const RowGeom &g, uint32_t r, int lane,
                                             uint32_t d[16]) {
    const long long o = (long long)r * kRowBytes + lane * kLaneBytes - (long long)g.P;
    // only row 0 of a padded or misaligned frame can touch bytes before the fragment
    const bool mask = (r == 0) && (g.P != 0 || (((uintptr_t)fi.addr & 15u) != 0));
    load64(fi.addr, o, 0, (long long)fi.len, mask, g.s16, d);
}

// XOR bytes_BE(partial) into frame bytes P..P+3 (row 0).
__device__ __forceinline__ void crc_inject(uint32_t d[16], const RowGeom &g, uint32_t partial, int lane) {
    const uint32_t v = __builtin_bswap32(partial);  // LE byte j = BE byte j of partial
    const uint32_t l0 = g.P >> 6;
    const uint32_t a = (g.P >> 2) & 15u;
    const uint32_t q = g.P & 3u;
    const uint32_t m0 = v << (8 * q);
    const uint32_t m1 = q ? (v >> (32 - 8 * q)) : 0u;
    const bool own = (uint32_t)lane == l0;
    const uint32_t mA = own ? m0 : 0u;
    const uint32_t mB = own ? m1 : 0u;
    const uint32_t mC = ((uint32_t)lane == l0 + 1 && a == 15u) ? m1 : 0u;
    d[0] ^= mC;
#pragma unroll
    for (uint32_t w = 0; w < 16; ++w) d[w] ^= (w == a) ? mA : ((w == a + 1) ? mB : 0u);
}

// ---- CRC, general fragments (descriptor batches, ragged messages) -----------------------
// kWv: waves per workgroup.  The fused copy (CopySource) runs 8-wave workgroups with a 1 KiB
// staging area per wave behind the tables (74 KiB: still two workgroups, now 16 waves per CU --
// each wave keeps one row in flight, so the wave count sets the bytes in flight).
template <class Src, int kWv = kWaves>
__global__ void __launch_bounds__(64 * kWv) crc_rows_kernel(Src src, size_t n, uint32_t fpw,
                                                            const uint32_t *__restrict__ img,
                                                            uint32_t *__restrict__ out) {
    static_assert(kWv >= kWaves, "the table builders need 256 threads");
    constexpr uint32_t kStage = Src::kCopy ? 1024u : 0u;     // a quarter row per part
    constexpr uint32_t kArea = kStage;
    __shared__ __attribute__((aligned(16))) uint32_t lds[(kLdsBytes + kWv * kArea) / 4];
    if constexpr (kWv == kWaves) {
        stage_tables<0>(lds, img, [] {});
    } else {
        if (threadIdx.x < 64 * kWaves) stage_tables<0, void (*)(), 7, false, false>(lds, img, [] {});
        lds_barrier();
    }

    const int lane = threadIdx.x & 63;
    const CrcLane k = make_lane(lane);
    const size_t f0 = uniform(blockIdx.x * kWv * fpw + (threadIdx.x >> 6));
    const size_t fend = f0 + (size_t)kWv * fpw;  // exclusive, stride kWv

    // next non-empty fragment at or after x (stride kWv); empty ones are answered directly
    auto next_nonempty = [&](size_t x, FragInfo &fi) -> size_t {
        for (; x < n && x < fend; x += kWv) {
            fi = src.get(x);
            fi.addr = (gbyte *)uniform64((uint64_t)(uintptr_t)fi.addr);
            fi.len = uniform(fi.len);
            fi.partial = uniform(fi.partial);
            if constexpr (Src::kCopy) {
                fi.dst = (uint8_t *)uniform64((uint64_t)(uintptr_t)fi.dst);
                fi.copylen = uniform(fi.copylen);
            }
            if (fi.len) return x;
            if (lane == 0) emit(src, out, x, fi.partial, fi);  // uicrc(p, 0, s) == s
        }
        return n;
    };

    // Copy sources load every row that starts inside its fragment (r > 0, or an unpadded frame)
    // coalesced -- lane l takes the 16 bytes at 16l + 1024q, one 1 KiB run per instruction, also
    // from sources that are not 16-byte aligned (unaligned dwordx4; a GM slot payload sits 72 bytes
    // in) -- stores it to a dword-aligned destination straight from those registers and hands the
    // CRC the lane-contiguous pieces through the wave's staging area (rows_to_pieces).  The other
    // rows (a padded frame's first) keep the lane-contiguous masked loads.
    auto coal_row = [&](const RowGeom &gg, uint32_t rr) -> bool { return Src::kCopy && (rr > 0 || gg.P == 0); };
    auto load_row = [&](const FragInfo &fi, const RowGeom &gg, uint32_t rr, uint32_t(&dd)[16]) {
        if (coal_row(gg, rr)) {
            gbyte *p = fi.addr + ((long long)rr * kRowBytes - (long long)gg.P) + 16 * lane;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32x4 v = ld16c((gu32x4_a1 *)(p + 1024 * q));
                dd[4 * q + 0] = v.x;
                dd[4 * q + 1] = v.y;
                dd[4 * q + 2] = v.z;
                dd[4 * q + 3] = v.w;
            }
        } else {
            crc_load_row(fi, gg, rr, lane, dd);
        }
    };

    FragInfo cur;
    size_t f = next_nonempty(f0, cur);
    if (f >= n) return;
    RowGeom g = crc_geom(cur);
    uint32_t r = 0;
    uint32_t d[16];
    load_row(cur, g, 0, d);
    uint32_t C = 0;
    uint32_t carry = 0;

    for (;;) {
        // prefetch the next row task
        FragInfo nfi = cur;
        RowGeom ng = g;
        size_t nf = f;
        uint32_t nr = r + 1;
        if (nr >= g.R) {
            nf = next_nonempty(f + kWv, nfi);
            nr = 0;
            if (nf < n) ng = crc_geom(nfi);
        }
        const bool more = nf < n;
        uint32_t nd[16];
        if (more) load_row(nfi, ng, nr, nd);

        if constexpr (Src::kCopy) {  // copy before the partial register is injected
            bool stored = false;
            if (coal_row(g, r)) {
                const long long row0 = (long long)r * kRowBytes - (long long)g.P;  // >= 0
                if (cur.copylen && row0 + kRowBytes <= (long long)cur.copylen &&
                    (((uintptr_t)cur.dst + (uint64_t)row0) & 3u) == 0) {
                    gwbyte *q = (gwbyte *)(cur.dst + row0) + 16 * lane;
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        st16((gwu32x4_a4 *)(q + 1024 * c), u32x4{d[4 * c], d[4 * c + 1], d[4 * c + 2], d[4 * c + 3]});
                    stored = true;
                }
                rows_to_pieces(lds + (kLdsBytes + (threadIdx.x >> 6) * kArea) / 4, d, lane);
            }
            if (cur.copylen && !stored) {
                const long long o = (long long)r * kRowBytes + lane * kLaneBytes - (long long)g.P;
                const uint32_t dm = (uint32_t)((uintptr_t)cur.dst - g.P) & 15u;
                const long long row0 = (long long)r * kRowBytes - (long long)g.P;
                const bool whole = row0 >= 0 && row0 + kRowBytes <= (long long)cur.copylen;
                uint32_t *area = lds + (kLdsBytes + (threadIdx.x >> 6) * kArea) / 4;
                if (whole && (dm & 3u) == 0) {
                    store_row_coalesced<kStage>(area, cur.dst + row0, d, lane);
                } else if (whole) {
                    // byte-misaligned: the aligned words covering [row0 - m, row0 - m + 4096) (as
                    // store64 forms them) go out coalesced at the dword-aligned dst + row0 - m; the
                    // row's first word (when it reaches before the copy) and, on the frame's last
                    // row, the word holding its last m bytes go through bounded word stores
                    if (r == 0) carry = 0;
                    const uint32_t m = dm & 3u, sh = 4u - m;
                    const uint32_t prev = prev_lane_top(d[15], carry, lane);
                    uint32_t v[16];
                    v[0] = __builtin_amdgcn_alignbyte(d[0], prev, sh);
#pragma unroll
                    for (int w = 1; w < 16; ++w) v[w] = __builtin_amdgcn_alignbyte(d[w], d[w - 1], sh);
                    const bool skip0 = row0 < 4;
                    store_row_coalesced<kStage>(area, cur.dst + row0 - m, v, lane, skip0);
                    if (skip0 && lane == 0) store_word(cur.dst, row0 - (long long)m, v[0], 0, (long long)cur.copylen);
                    if (lane == 63 && r + 1 == g.R)
                        store_word(cur.dst, row0 - (long long)m + kRowBytes, __builtin_amdgcn_alignbyte(0u, d[15], sh), 0,
                                   (long long)cur.copylen);
                } else if ((dm & 3u) == 0) {
                    store_row_coalesced_masked(area, cur.dst, row0, d, lane, 0, (long long)cur.copylen);
                } else {
                    if (r == 0) carry = 0;
                    const uint32_t prev = prev_lane_top(d[15], carry, lane);
                    store64(cur.dst, o, d, 0, (long long)cur.copylen, dm & 3u, false, prev,
                            lane == 63 && r + 1 == g.R);
                }
                carry = __builtin_amdgcn_readlane(d[15], 63);
            }
        }
        // process the current row
        if (r == 0) {
            if (g.P == 0) {
                C = (lane == 0) ? __builtin_bswap32(cur.partial) : 0u;
            } else {
                C = 0;
                crc_inject(d, g, cur.partial, lane);
            }
        } else {
            C = horner_shift(lds, C);
            if (r == 1 && g.P > (uint32_t)kRowBytes - 4 && lane == 0)  // register bytes spill into row 1
                d[0] ^= __builtin_bswap32(cur.partial) >> (8 * (kRowBytes - g.P));
        }
        C = crc_piece(lds, k, C, d);

        if (r + 1 == g.R) {
            C = wave_xor(lane_combine(lds, k, C));
            if (lane == 0) {
                uint32_t res = __builtin_bswap32(C);
                if (cur.len < 4) res ^= cur.partial << (8 * cur.len);
                emit(src, out, f, res, cur);
            }
        }
        if (!more) break;
#pragma unroll
        for (int w = 0; w < 16; ++w) d[w] = nd[w];
        cur = nfi;
        g = ng;
        f = nf;
        r = nr;
    }
}

constexpr uint32_t kFragsPerWg = 256;  // fragments per workgroup of crc_stream_kernel (at most)

// Two independent registers through their 16-word pieces, interleaved (two chains per wave)
__device__ __forceinline__ void crc_piece2(const uint32_t *lds, const CrcLane &k, uint32_t &C0, const uint32_t d0[16],
                                           uint32_t &C1, const uint32_t d1[16]) {
    uint32_t X0 = C0 ^ d0[0], X1 = C1 ^ d1[0];
#pragma unroll
    for (int w = 0; w < 15; ++w) {
        const Look4 t0 = look4(lds, k, X0);
        const Look4 t1 = look4(lds, k, X1);
        X0 = xor3(xor3(t0.t0, t0.t1, t0.t2), t0.t3, d0[w + 1]);
        X1 = xor3(xor3(t1.t0, t1.t1, t1.t2), t1.t3, d1[w + 1]);
    }
    const Look4 t0 = look4(lds, k, X0);
    const Look4 t1 = look4(lds, k, X1);
    C0 = xor3(t0.t0, t0.t1, t0.t2) ^ t0.t3;
    C1 = xor3(t1.t0, t1.t1, t1.t2) ^ t1.t3;
}

// ---- CRC, general fragments as piece streams (descriptor batches, ragged messages) ---------
// A workgroup owns up to kFragsPerWg consecutive fragments.  Fragment f is cut into
// np = ceil(L/64) 64-byte pieces, right-aligned: its first piece starts P = 64*np - L bytes
// before the fragment (zeros: free for a CRC from a zero register).  The non-empty fragments are
// split into 2*kWaves contiguous runs of about equal piece count ("chains", two per wave); a
// chain's pieces, fragment after fragment, form one stream cut into rows of 64 pieces, lane l
// taking piece l of every row.  Rows are full whatever the fragment sizes: the 4 KiB frame of
// crc_frags_kernel padded every fragment to whole rows (1.2x the lookups on config C) and needed
// lane-group packs for small fragments.
// Per row, lane l CRCs its piece from its start register -- 0; bswap(partial) for a fragment's
// first piece when P == 0 (otherwise partial is injected as data at byte P); for lane 0, the
// value carried from the previous row when its piece continues a fragment -- and shifts the
// result to the end of its segment (the lanes of its fragment in this row, [ss, e]) with the
// combine column of lane 63 - (e - l) (a shift by 64*(e - l) bytes).  A segmented XOR scan (DPP)
// leaves each segment's value at its last lane: the fragment's CRC where the fragment ends, the
// register carried into the next row's lane 0 at lane 63 otherwise.
// The boundary mask M of a row (bit p: a fragment of the chain starts at piece p) comes from the
// chain's piece starts in LDS: lane j marks word p_j of a per-chain scratch row, every lane
// reads its word back and a ballot collects them; a row inside one fragment skips that (M = 0).
struct StreamDesc {
    uint64_t addr;
    uint32_t len, partial;
};

// per-lane task word: bits 0..8 list position, 9..14 segment end e, 15..20 segment start ss,
// 21..24 (misaligned variant) the piece's byte misalignment, then the flags
constexpr uint32_t kTfFirst = 1u << 25, kTfLast = 1u << 26, kTfNull = 1u << 27, kTfSecond = 1u << 28;

template <int N>
struct RowN {
    u32x4 q[N];
};
template <int N>
struct AddrN {
    gbyte *p[N];
};

__device__ __forceinline__ void issue_rowN(const AddrN<4> &a, RowN<4> &r) {
    asm volatile(
        "global_load_dwordx4 %0, %4, off\n\t"
        "global_load_dwordx4 %1, %5, off\n\t"
        "global_load_dwordx4 %2, %6, off\n\t"
        "global_load_dwordx4 %3, %7, off"
        : "=&v"(r.q[0]), "=&v"(r.q[1]), "=&v"(r.q[2]), "=&v"(r.q[3])
        : "v"(a.p[0]), "v"(a.p[1]), "v"(a.p[2]), "v"(a.p[3])
        : "memory");
}
__device__ __forceinline__ void issue_rowN(const AddrN<5> &a, RowN<5> &r) {
    asm volatile(
        "global_load_dwordx4 %0, %5, off\n\t"
        "global_load_dwordx4 %1, %6, off\n\t"
        "global_load_dwordx4 %2, %7, off\n\t"
        "global_load_dwordx4 %3, %8, off\n\t"
        "global_load_dwordx4 %4, %9, off"
        : "=&v"(r.q[0]), "=&v"(r.q[1]), "=&v"(r.q[2]), "=&v"(r.q[3]), "=&v"(r.q[4])
        : "v"(a.p[0]), "v"(a.p[1]), "v"(a.p[2]), "v"(a.p[3]), "v"(a.p[4])
        : "memory");
}

__device__ __forceinline__ void issue_rowN(const AddrN<1> &a, RowN<1> &r) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(r.q[0]) : "v"(a.p[0]) : "memory");
}
__device__ __forceinline__ void issue_rowN(const AddrN<2> &a, RowN<2> &r) {
    asm volatile(
        "global_load_dwordx4 %0, %2, off\n\t"
        "global_load_dwordx4 %1, %3, off"
        : "=&v"(r.q[0]), "=&v"(r.q[1])
        : "v"(a.p[0]), "v"(a.p[1])
        : "memory");
}

// wait until at most N younger loads are outstanding; the two chains' registers of the slot are
// threaded through so no use is scheduled above the wait
template <int N>
__device__ __forceinline__ void wait_rows2(RowN<4> &a, RowN<4> &b) {
    asm volatile("s_waitcnt vmcnt(%8) ; lampi-wait %0 %1 %2 %3 %4 %5 %6 %7"
                 : "+v"(a.q[0]), "+v"(a.q[1]), "+v"(a.q[2]), "+v"(a.q[3]), "+v"(b.q[0]), "+v"(b.q[1]),
                   "+v"(b.q[2]), "+v"(b.q[3])
                 : "n"(N)
                 : "memory");
}
template <int N>
__device__ __forceinline__ void wait_rows2(RowN<5> &a, RowN<5> &b) {
    asm volatile("s_waitcnt vmcnt(%10) ; lampi-wait %0 %1 %2 %3 %4 %5 %6 %7 %8 %9"
                 : "+v"(a.q[0]), "+v"(a.q[1]), "+v"(a.q[2]), "+v"(a.q[3]), "+v"(a.q[4]), "+v"(b.q[0]),
                   "+v"(b.q[1]), "+v"(b.q[2]), "+v"(b.q[3]), "+v"(b.q[4])
                 : "n"(N)
                 : "memory");
}

// Waits whose count depends on a run-time (wave-uniform) condition must be ONE asm statement: two
// waits on two branches make the compiler merge the ring registers through a phi, and it then
// copies registers whose loads are still in flight before the wait (garbage; seen in the ISA).
// sel (SGPR): 0 -> vmcnt(A), 1 -> vmcnt(B), else vmcnt(C).
#define LAMPI_WAIT_SEL_ASM(OPS)            \
    "s_cmp_eq_u32 %[sel], 0\n\t"          \
    "s_cbranch_scc1 1f\n\t"               \
    "s_cmp_eq_u32 %[sel], 1\n\t"          \
    "s_cbranch_scc1 2f\n\t"               \
    "s_waitcnt vmcnt(%[c])\n\t"           \
    "s_branch 3f\n"                        \
    "1:\n\t"                              \
    "s_waitcnt vmcnt(%[a])\n\t"           \
    "s_branch 3f\n"                        \
    "2:\n\t"                              \
    "s_waitcnt vmcnt(%[b])\n"              \
    "3:\n\t"                              \
    "; lampi-wait " OPS

template <int A, int B, int C>
__device__ __forceinline__ void wait_sel(uint32_t sel, u32x4 &r) {
    asm volatile(LAMPI_WAIT_SEL_ASM("%0")
                 : "+v"(r)
                 : [sel] "s"(sel), [a] "n"(A), [b] "n"(B), [c] "n"(C)
                 : "scc", "memory");
}
template <int A, int B, int C>
__device__ __forceinline__ void wait_sel(uint32_t sel, u32x4 &r0, u32x4 &r1) {
    asm volatile(LAMPI_WAIT_SEL_ASM("%0 %1")
                 : "+v"(r0), "+v"(r1)
                 : [sel] "s"(sel), [a] "n"(A), [b] "n"(B), [c] "n"(C)
                 : "scc", "memory");
}

// shift by 64*(63 - l') zero bytes with lane l''s combine column (b = comb_col(l'))
__device__ __forceinline__ uint32_t combine_at(const uint32_t *lds, uint32_t b, uint32_t C) {
    uint32_t r = lds_u32(lds, ((C << 9) & 0x1E00u) | b);
    r ^= lds_u32(lds, (((C << 5) & 0x1E00u) | b) + 8192);
    r ^= lds_u32(lds, (((C << 1) & 0x1E00u) | b) + 2 * 8192);
#pragma unroll
    for (int p = 3; p < 8; ++p) r ^= lds_u32(lds, (((C >> (4 * p - 9)) & 0x1E00u) | b) + p * 8192);
    return r;
}

__device__ __forceinline__ uint32_t comb_col(uint32_t l) { return (l >> 5) * 256u + 128u + (l & 31u) * 4u; }

// inclusive scan inside segments (XOR for CRC values, + for sums): lane l gets the combination of
// lanes [ss, l] (pos = l - ss).  Row-local steps by row_shr (sources outside the row read 0),
// then row_bcast:15 / :31 carry across rows for lanes whose segment started in an earlier row.
template <bool kAdd>
__device__ __forceinline__ uint32_t seg_scan(uint32_t v, uint32_t pos, uint32_t lane) {
    auto op = [](uint32_t a, uint32_t b) { return kAdd ? a + b : a ^ b; };
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v = op(v, pos >= 1u ? t : 0u);
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v = op(v, pos >= 2u ? t : 0u);
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v = op(v, pos >= 4u ? t : 0u);
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v = op(v, pos >= 8u ? t : 0u);
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v = op(v, pos > (lane & 15u) ? t : 0u);
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    v = op(v, pos > (lane & 31u) ? t : 0u);
    return v;
}

// A chain: rows [c*R/8, (c+1)*R/8) of the workgroup's piece stream (R rows in all), so chains
// differ by at most one row.  A fragment crossing a chain start is checksummed in parts: the
// chain holding its first piece leaves the register at its end in sopen, later chains start it
// from 0 and leave either their open value (sopen) or, where the fragment ends, its value
// (shead); the parts are joined after the workgroup's rows (stream_join).
struct StreamChain {
    uint64_t rs, end;  // pieces [rs, end)
    uint32_t cur;      // list entry holding piece rs - 1 (head - 1 when the chain starts a fragment)
    uint32_t b;        // one past the last list entry with a piece in the chain
    uint32_t head;     // list entry holding piece rs
    uint32_t mid;      // 1: the chain starts inside fragment `head`
};

// a * b mod P (CRC-32/MPEG-2, normal MSB-first register domain), Horner over b's bits
__host__ __device__ constexpr uint32_t gf_mulmod(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 31; i >= 0; --i) {
        r = (r << 1) ^ ((r >> 31) ? 0x04C11DB7u : 0u);
        r ^= ((b >> i) & 1u) ? a : 0u;
    }
    return r;
}
// kRowShift[j] = x^(8 * 4096 * 2^j) mod P: the shift of a register past 2^j rows of zero bytes
struct RowShifts {
    uint32_t k[20];
};
constexpr RowShifts row_shifts() {
    RowShifts t{};
    uint32_t x = 2u;                                  // x^1
    for (int i = 0; i < 15; ++i) x = gf_mulmod(x, x);  // x^(2^15) = x^(8 * 4096)
    for (int j = 0; j < 20; ++j) {
        t.k[j] = x;
        x = gf_mulmod(x, x);
    }
    return t;
}
constexpr RowShifts kRowShift = row_shifts();
static_assert(gf_mulmod(0x80000000u, 2u) == 0x04C11DB7u, "x^31 * x = x^32 = P - x^32");

// The same multiplications as columns: kRowCols.c[j][i] = x^i * kRowShift.k[j] mod P, so
// v * kRowShift.k[j] = XOR of the columns of v's set bits -- 32 independent select-and-XORs on
// four accumulators instead of gf_mulmod's 32 dependent shift-reduce steps (a single thread's join
// tail: each multiply ~0.5 us as a dependent chain).
struct RowCols {
    uint32_t c[20][32];
};
constexpr RowCols row_cols() {
    RowCols t{};
    for (int j = 0; j < 20; ++j)
        for (int i = 0; i < 32; ++i) t.c[j][i] = gf_mulmod(1u << i, kRowShift.k[j]);
    return t;
}
constexpr RowCols kRowCols = row_cols();

template <int J>
__device__ __forceinline__ uint32_t mul_row_shift(uint32_t v) {
    uint32_t r[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t m = (uint32_t)((int32_t)(v << (31 - i)) >> 31);  // bit i of v as a mask
        r[i & 3] ^= m & kRowCols.c[J][i];
    }
    return (r[0] ^ r[1]) ^ (r[2] ^ r[3]);
}

// v (normal domain) * x^(8 * 4096 * h) mod P: the register after h rows of zero bytes, h < 2^20
template <int J = 0>
__device__ __forceinline__ uint32_t shift_rows(uint32_t v, uint32_t h) {
    if constexpr (J < 20) {
        if ((h >> J) & 1u) v = mul_row_shift<J>(v);
        return (h >> (J + 1)) ? shift_rows<J + 1>(v, h) : v;
    } else {
        return v;
    }
}

// C (swapped domain) after 64*m zero bytes, m < 2^26: the low six bits of m through lane
// (63 - (m & 63))'s combine column in LDS, the rows (h = m >> 6, 4096 bytes each) as products
// with compile-time constants x^(8 * 4096 * 2^j) mod P -- no memory traffic (the shift-by-2^e
// columns of the table image took one dependent round of 32 global loads per bit of h, and a
// fragment spanning all chains of a workgroup joined that way serially: 65,456-byte host calls
// spent ~20 us there)
__device__ uint32_t shift_pieces(const uint32_t *lds, const uint32_t *__restrict__ img, uint32_t C, uint64_t m) {
    (void)img;
    const uint32_t l = (uint32_t)(m & 63u);
    if (l) C = combine_at(lds, comb_col(63u - l), C);
    const uint32_t h = (uint32_t)(m >> 6);
    if (h) C = __builtin_bswap32(shift_rows(__builtin_bswap32(C), h));
    return C;
}

template <int K>
struct RowsN4 {
    RowN<4> r[K];
};

// kK chains per wave (1: 512-thread workgroups, 2: 256-thread); kChains = 8 either way.
// (Round 1 also ran the SUM fused copy on 16-byte-piece streams here; round 2 moved it to
// sum_rows_kernel, which measured faster on every layout: launch_sum_copy.)
// Timeline diagnostic (tools/microbench/stream_timeline.py, profiles/r05/configC_ab.txt; never a product
// path): per workgroup, 16 words of s_memrealtime stamps -- [0] entry, [7] descriptors and tables in, [8] prefix
// scan done, [1] chains set up, [9] first rows arrived, [2] first row checksummed, [3] rows done, [4] exit --
// and [5] HW_ID, [6] XCC_ID.
__device__ uint64_t *g_stream_diag = nullptr;
#define LAMPI_DIAG_STAMP(K)                                                                            \
    do {                                                                                               \
        if constexpr (kDiag) {                                                                         \
            if (threadIdx.x == 0) g_stream_diag[(size_t)blockIdx.x * 16 + (K)] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                              \
    } while (0)

template <bool kMis, int kD, int kK, bool kSum, bool kDiag = false>
__device__ __forceinline__ void stream_body(const uint32_t *lds, const StreamDesc *sdesc, const uint64_t *sstart,
                                            const uint16_t *sj, uint32_t *marks, const StreamChain *sch,
                                            uint32_t *sopen, uint32_t *shead, gbyte *zero, uint32_t *sres,
                                            uint32_t *__restrict__ out) {
    constexpr int kPB = 64;  // piece bytes
    constexpr int NL = kMis ? kPB / 16 + 1 : kPB / 16;  // loads per row
    constexpr int kW = kPB / 4;                          // words per piece
    const uint32_t lane = threadIdx.x & 63u;
    struct SChain {
        uint64_t rs, end;  // piece index of the next row's first piece, of the chain's end
        uint32_t cur, b;   // list position of the fragment holding piece rs - 1; chain end
        // list entry `cur` as the last one-segment row read it (hit: hot == 1): its descriptor,
        // first piece and the next entry's first piece, so a row inside it reads no LDS
        uint32_t hot, hlen, hpartial, hj;
        uint64_t haddr, hs, hnb;
    };
    struct STask {
        uint32_t info, sreg;  // per lane: task word, start register
        uint64_t M;           // boundary mask
        uint32_t fix;         // bit 0: a first piece needs byte masking, bit 1: partial injected as data,
                              // bit 2: null row
        uint32_t one;         // one-segment rows: list entry | output index << 16
    };
    SChain cs[kK];
    uint32_t head[kK], mid[kK];
    uint32_t nsteps = 0;
#pragma unroll
    for (int c = 0; c < kK; ++c) {
        cs[c].rs = uniform64(sch[c].rs);
        cs[c].end = uniform64(sch[c].end);
        cs[c].cur = uniform(sch[c].cur);  // wraps for head == 0: li = cur + (count >= 1)
        cs[c].b = uniform(sch[c].b);
        cs[c].hot = 0u;
        head[c] = uniform(sch[c].head);
        mid[c] = uniform(sch[c].mid);
        nsteps = max(nsteps, (uint32_t)((cs[c].end - cs[c].rs + 63) >> 6));
    }
    if (nsteps == 0) return;

    const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);  // lanes <= l
    auto issue_task = [&](SChain &c, uint32_t *mk, STask &t) -> AddrN<NL> {
        AddrN<NL> A;
        if (c.rs >= c.end) {  // chain done: null row
            t.info = kTfNull | (63u << 9);
            t.sreg = 0u;
            t.M = 0ull;
            t.fix = 4u;
            t.one = 0u;
#pragma unroll
            for (int q = 0; q < NL; ++q) A.p[q] = zero;
            return A;
        }
        uint64_t M = 0ull;
        const bool hit = c.hot && c.hnb >= c.rs + 64u;  // the row lies inside cached entry cur
        const uint64_t nb = hit ? c.hnb : uniform64(sstart[c.cur + 1u]);
        const uint64_t nb2 = hit ? ~0ull : (c.cur + 2u <= c.b ? uniform64(sstart[c.cur + 2u]) : ~0ull);
        if (nb2 >= c.rs + 64u) {  // at most one fragment starts in this row
            M = nb < c.rs + 64u ? (1ull << (uint32_t)(nb - c.rs)) : 0ull;
        } else {  // several: build the boundary mask
            const uint32_t i = c.cur + 1u + lane;
            const bool v = i <= c.b;
            const uint64_t p = sstart[v ? i : c.b] - c.rs;
            if (v && p < 64u) mk[(uint32_t)p] = 1u;
            const uint32_t m = mk[lane];
            mk[lane] = 0u;
            M = __builtin_amdgcn_ballot_w64(m != 0u);
        }
        if ((M & ~1ull) == 0ull) {  // one segment: every lane in list entry cur + M (scalar set-up)
            const uint32_t lr = c.cur + (uint32_t)M;
            if (!hit) {  // cache entry lr: it is `cur` after this row (M is 0 or 1)
                c.haddr = uniform64(sdesc[lr].addr);
                c.hlen = uniform(sdesc[lr].len);
                c.hpartial = uniform(sdesc[lr].partial);
                c.hs = uniform64(sstart[lr]);
                c.hj = uniform(sj[lr]);
                c.hnb = M ? nb2 : nb;  // first piece of entry lr + 1
                c.hot = 1u;
            }
            const uint64_t addr = c.haddr;
            const uint32_t len = c.hlen, partial = c.hpartial;
            const uint32_t k0 = (uint32_t)(c.rs - c.hs);  // lane 0's piece
            t.one = (lr & 0xFFFFu) | (c.hj << 16);
            const uint32_t np = (uint32_t)(((uint64_t)len + (kPB - 1)) / kPB);
            // CRC: pieces right-aligned (P leading zeros); SUM: left-aligned on the word grid
            const uint32_t P = kSum ? 0u : (np << 6) - len;
            const long long o0 = (long long)k0 * kPB - (long long)P;
            gbyte *pa = (gbyte *)(uintptr_t)addr + o0 + lane * (uint32_t)kPB;
            uint32_t sh = 0u;
            if constexpr (!kMis && kSum) {  // chunks past the fragment end read zeros
                const long long o = o0 + (long long)lane * kPB;
#pragma unroll
                for (int q = 0; q < kPB / 16; ++q) A.p[q] = (o + 16 * q < (long long)len) ? pa + 16 * q : zero;
            } else if constexpr (!kMis) {
#pragma unroll
                for (int q = 0; q < 4; ++q) A.p[q] = pa + 16 * q;
                if (o0 + 16 <= 0) {  // lane 0's first piece starts with whole chunks of padding
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (o0 + 16 * q + 16 <= 0 && lane == 0u) A.p[q] = zero;
                }
            } else {
                sh = (uint32_t)((addr + (uint64_t)o0) & 15u);
                gbyte *pb = pa - sh;
                const long long ob = o0 + (long long)lane * kPB - (long long)sh;
#pragma unroll
                for (int q = 0; q < NL; ++q) {
                    const long long r = ob + 16 * q;
                    A.p[q] = (r + 16 > 0 && r < (long long)len) ? pb + 16 * q : zero;
                }
            }
            const uint32_t k = k0 + lane;
            const bool first = k == 0u, last = k + 1u == np, second = k == 1u;
            t.info = (lr & 0x1FFu) | (63u << 9) | (sh << 21) | (first ? kTfFirst : 0u) | (last ? kTfLast : 0u) |
                     (second ? kTfSecond : 0u);
            t.sreg = (!kSum && first && P == 0u) ? __builtin_bswap32(partial) : 0u;
            t.M = M;
            if constexpr (kSum) {  // the last piece, if in this row and partial, is masked
                t.fix = (k0 + 64u >= np && (len % kPB) != 0u) ? 1u : 0u;
            } else {
                const bool needmask = k0 == 0u && (kMis ? P != 0u : (P & 15u) != 0u);
                const bool needinj = (k0 == 0u && P != 0u) || (k0 <= 1u && np > 1u && P > 60u);
                t.fix = (needmask ? 1u : 0u) | (needinj ? 2u : 0u);
            }
            c.cur += (uint32_t)M;
            c.rs += 64u;
            return A;
        }
        const uint32_t li = c.cur + (uint32_t)__popcll(M & le);
        const bool nul = li >= c.b;
        const uint32_t lr = nul ? c.b : li;
        const StreamDesc D = sdesc[lr];
        const uint32_t k = (uint32_t)(c.rs + lane - sstart[lr]);
        const uint32_t np = (uint32_t)(((uint64_t)D.len + (kPB - 1)) / kPB);
        const uint32_t P = kSum ? 0u : (np << 6) - D.len;  // mod 2^32: always < 64
        const long long o = (long long)k * kPB - (long long)P;
        gbyte *pa = (gbyte *)(uintptr_t)D.addr + o;
        uint32_t sh = 0u;
        if constexpr (!kMis && kSum) {
#pragma unroll
            for (int q = 0; q < kPB / 16; ++q) A.p[q] = (!nul && o + 16 * q < (long long)D.len) ? pa + 16 * q : zero;
        } else if constexpr (!kMis) {
#pragma unroll
            for (int q = 0; q < 4; ++q) A.p[q] = (!nul && o + 16 * q + 16 > 0) ? pa + 16 * q : zero;
        } else {
            sh = (uint32_t)((uintptr_t)pa & 15u);
            gbyte *pb = pa - sh;
            const long long ob = o - (long long)sh;
#pragma unroll
            for (int q = 0; q < NL; ++q) {
                const long long r = ob + 16 * q;
                A.p[q] = (!nul && r + 16 > 0 && r < (long long)D.len) ? pb + 16 * q : zero;
            }
        }
        const uint64_t above = lane == 63 ? 0ull : (M >> (lane + 1u));
        const uint32_t e = above ? lane + (uint32_t)__builtin_ctzll(above) : 63u;
        const uint64_t below = M & le;
        const uint32_t ss = below ? 63u - (uint32_t)__builtin_clzll(below) : 0u;
        const bool first = !nul && k == 0u, last = !nul && k + 1u == np, second = !nul && k == 1u;
        t.info = (lr & 0x1FFu) | (e << 9) | (ss << 15) | (sh << 21) | (first ? kTfFirst : 0u) |
                 (last ? kTfLast : 0u) | (nul ? kTfNull : 0u) | (second ? kTfSecond : 0u);
        t.sreg = (!kSum && first && P == 0u) ? __builtin_bswap32(D.partial) : 0u;
        t.M = M;
        if constexpr (kSum) {
            t.fix = __builtin_amdgcn_ballot_w64(last && (D.len % kPB) != 0u) ? 1u : 0u;
        } else {
            const bool needmask = first && (kMis ? P != 0u : (P & 15u) != 0u);
            const bool needinj = (first && P != 0u) || (second && P > 60u);
            t.fix = (__builtin_amdgcn_ballot_w64(needmask) ? 1u : 0u) | (__builtin_amdgcn_ballot_w64(needinj) ? 2u : 0u);
        }
        t.one = 0u;
        c.cur += (uint32_t)__popcll(M);
        c.rs += 64u;
        c.hot = 0u;
        return A;
    };

    // the lane's kW words, fixed up for first pieces
    auto prepare = [&](const RowN<NL> &raw, const STask &t, uint32_t d[kW]) {
        if constexpr (!kMis) {
#pragma unroll
            for (int q = 0; q < kPB / 16; ++q) {
                d[4 * q + 0] = raw.q[q].x;
                d[4 * q + 1] = raw.q[q].y;
                d[4 * q + 2] = raw.q[q].z;
                d[4 * q + 3] = raw.q[q].w;
            }
        } else {  // the aligned chunks covering the piece, funnel-shifted by the lane's misalignment
            uint32_t a[4 * NL];
#pragma unroll
            for (int q = 0; q < NL; ++q) {
                a[4 * q + 0] = raw.q[q].x;
                a[4 * q + 1] = raw.q[q].y;
                a[4 * q + 2] = raw.q[q].z;
                a[4 * q + 3] = raw.q[q].w;
            }
            const uint32_t sh = (t.info >> 21) & 15u, ws = sh >> 2, sb = sh & 3u;
            uint32_t b[kW + 1];
#pragma unroll
            for (int i = 0; i <= kW; ++i) b[i] = sel4(ws, a[i], a[i + 1], a[i + 2], a[i + 3]);
#pragma unroll
            for (int w = 0; w < kW; ++w) d[w] = __builtin_amdgcn_alignbyte(b[w + 1], b[w], sb);
        }
        if (kSum && (t.fix & 1u)) {  // zero the bytes of a partial last piece past the fragment end
            const uint32_t rem = sdesc[t.info & 0x1FFu].len % kPB;
            if ((t.info & kTfLast) && rem != 0u) {
#pragma unroll
                for (int w = 0; w < kW; ++w) d[w] &= byte_keep_mask(4 * w, 0, (long long)rem);
            }
        } else if (!kSum && (t.fix & 3u)) {
            const StreamDesc D = sdesc[t.info & 0x1FFu];
            const uint32_t P = (0u - D.len) & 63u;
            const bool first = (t.info & kTfFirst) != 0u;
            if ((t.fix & 1u) && first) {
#pragma unroll
                for (int w = 0; w < 16; ++w) d[w] &= byte_keep_mask(4 * w, (long long)P, 64);
            }
            if (t.fix & 2u) {
                const uint32_t v = __builtin_bswap32(D.partial);
                if (first && P != 0u) {  // bytes_BE(partial) at piece bytes P..P+3; what lies past
                    const uint32_t a = P >> 2, q = P & 3u;  // byte 63 goes to the second piece
                    const uint32_t m0 = v << (8 * q), m1 = q ? (v >> (32 - 8 * q)) : 0u;
#pragma unroll
                    for (uint32_t w = 0; w < 16; ++w) d[w] ^= (w == a) ? m0 : ((w == a + 1u) ? m1 : 0u);
                }
                if ((t.info & kTfSecond) && P > 60u) d[0] ^= v >> (8 * (64u - P));
            }
        }
    };

    // a fragment's value: its checksum, or (the head fragment of a chain that starts inside it) the
    // part for stream_join
    auto result = [&](int ch, uint32_t li, uint32_t x) {
        if (mid[ch] && li == head[ch]) {
            shead[ch] = x;
            return;
        }
        if constexpr (kSum) {
            sres[sj[li]] = x;
        } else {
            const StreamDesc D = sdesc[li];
            uint32_t res = __builtin_bswap32(x);
            if (D.len < 4u) res ^= D.partial << (8 * D.len);
            sres[sj[li]] = res;
        }
    };
    // segment values -> results and the carry of the open segment at lane 63.  v: the lane's
    // value shifted to its segment's end (combine column of lane 63 - (e - l); e = 63 in a
    // one-segment row).  No early exits: branches here keep the chains from interleaving.
    auto finish = [&](int ch, const STask &t, uint32_t v, uint32_t &carry) {
        uint32_t x;
        if ((t.M & ~1ull) == 0ull) {  // one segment (never a fragment shorter than 4 bytes)
            x = kSum ? wave_add(v) : wave_xor(v);
            if (lane == 63u && (t.info & kTfLast)) {
                if (mid[ch] && (t.one & 0xFFFFu) == head[ch])
                    shead[ch] = x;
                else
                    sres[t.one >> 16] = kSum ? x : __builtin_bswap32(x);
            }
        } else {
            x = seg_scan<kSum>(v, lane - ((t.info >> 15) & 63u), lane);
            if (((t.info >> 9) & 63u) == lane && (t.info & kTfLast)) result(ch, t.info & 0x1FFu, x);
            x = __builtin_amdgcn_readlane(x, 63);
        }
        carry = (t.fix & 4u) ? carry : x;  // a null row keeps the chain's final open value
    };

    const CrcLane kl = make_lane((int)lane);
    RowN<NL> ring[kD][kK];
    STask tk[kD][kK];
#pragma unroll
    for (int q = 0; q < kD; ++q) {
        AddrN<NL> A[kK];
#pragma unroll
        for (int c = 0; c < kK; ++c) A[c] = issue_task(cs[c], marks + 64 * c, tk[q][c]);
#pragma unroll
        for (int c = 0; c < kK; ++c) issue_rowN(A[c], ring[q][c]);
    }
    uint32_t carry[kK];
#pragma unroll
    for (int c = 0; c < kK; ++c) carry[c] = 0u;
    uint32_t step = 0u;
    auto process = [&](RowN<NL> (&raw)[kK], const STask (&t)[kK]) {
        uint32_t d[kK][kW], C[kK];
#pragma unroll
        for (int c = 0; c < kK; ++c) prepare(raw[c], t[c], d[c]);
#pragma unroll
        for (int c = 0; c < kK; ++c) {
            C[c] = t[c].sreg;
            if (lane == 0u && !(t[c].info & (kTfFirst | kTfNull))) C[c] = carry[c];
        }
        if constexpr (kSum) {
#pragma unroll
            for (int c = 0; c < kK; ++c)
#pragma unroll
                for (int w = 0; w < kW; w += 2) C[c] = C[c] + d[c][w] + d[c][w + 1];
        } else if constexpr (kK == 2) {
            crc_piece2(lds, kl, C[0], d[0], C[1], d[1]);
        } else {
            C[0] = crc_piece(lds, kl, C[0], d[0]);
        }
        uint32_t v[kK];
#pragma unroll
        for (int c = 0; c < kK; ++c)
            v[c] = kSum ? C[c] : combine_at(lds, comb_col(lane + 63u - ((t[c].info >> 9) & 63u)), C[c]);
#pragma unroll
        for (int c = 0; c < kK; ++c) finish(c, t[c], v[c], carry[c]);
    };
    auto wait_slot = [&](RowN<NL> (&r)[kK], auto S) {
        (void)S;
        if constexpr (kK == 2) {
            wait_rows2<(kD - 1) * 2 * NL>(r[0], r[1]);
        } else if constexpr (NL == 4) {
            asm volatile("s_waitcnt vmcnt(%4) ; lampi-wait %0 %1 %2 %3"
                         : "+v"(r[0].q[0]), "+v"(r[0].q[1]), "+v"(r[0].q[2]), "+v"(r[0].q[3])
                         : "n"((kD - 1) * NL)
                         : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(%5) ; lampi-wait %0 %1 %2 %3 %4"
                         : "+v"(r[0].q[0]), "+v"(r[0].q[1]), "+v"(r[0].q[2]), "+v"(r[0].q[3]), "+v"(r[0].q[4])
                         : "n"((kD - 1) * NL)
                         : "memory");
        }
    };
#define LAMPI_STREAM_STEP(S)                                                                  \
    if constexpr ((S) < kD) {                                                                 \
        wait_slot(ring[S], std::integral_constant<int, (S)>{});                               \
        if (step == 0u) LAMPI_DIAG_STAMP(9);                                                  \
        if (step == nsteps) break;                                                            \
        process(ring[S], tk[S]);                                                              \
        if (step == 0u) LAMPI_DIAG_STAMP(2);                                                  \
        ++step;                                                                               \
        {                                                                                     \
            AddrN<NL> A[kK];                                                                  \
            _Pragma("unroll") for (int c = 0; c < kK; ++c) A[c] =                             \
                issue_task(cs[c], marks + 64 * c, tk[S][c]);                                  \
            _Pragma("unroll") for (int c = 0; c < kK; ++c) issue_rowN(A[c], ring[S][c]);      \
        }                                                                                     \
    }
    for (;;) {
        LAMPI_STREAM_STEP(0)
        LAMPI_STREAM_STEP(1)
        LAMPI_STREAM_STEP(2)
        LAMPI_STREAM_STEP(3)
        LAMPI_STREAM_STEP(4)
        LAMPI_STREAM_STEP(5)
        LAMPI_STREAM_STEP(6)
        LAMPI_STREAM_STEP(7)
    }
#undef LAMPI_STREAM_STEP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the rows in flight before exit
    if (lane == 0u) {  // the chains' open values (used only where a fragment continues)
#pragma unroll
        for (int c = 0; c < kK; ++c) sopen[c] = carry[c];
    }
}

// kK: chains per wave, kWv: waves per workgroup (kWv * kK chains); kWaveCap > 0 asks the
// compiler for that many waves per SIMD.  (Round 1's ablated variants -- loads and task walk
// only, no piece lookups -- ran as a template switch here until commit d95cfff:
// profiles/r01_stream_ablation.txt.)
template <class Src, int kD = 3, int kK = 2, bool kSum = false, int kWv = 8 / kK, int kWaveCap = 0,
          bool kDiag = false>
__global__ void __launch_bounds__(64 * kWv) __attribute__((amdgpu_waves_per_eu(kWaveCap > 0 ? kWaveCap : 1)))
crc_stream_kernel(Src src, size_t n, uint32_t fpg, const uint32_t *__restrict__ img, uint32_t *__restrict__ out,
                  const uint32_t *__restrict__ plan) {
    static_assert(!Src::kCopy, "fused copies run crc_rows_kernel / sum_rows_kernel");
    constexpr int kPB = 64;  // piece bytes
    constexpr uint32_t kThreads = 64 * kWv;
    constexpr uint32_t kChains = kWv * kK;
    static_assert(kThreads >= kFragsPerWg, "one fragment per thread in the set-up");
    __shared__ __attribute__((aligned(16))) uint32_t lds[kSum ? 4 : 65536 / 4];  // slicing + combine tables
    __shared__ StreamDesc sdesc[kFragsPerWg + 1];
    __shared__ uint64_t sstart[kFragsPerWg + 1];  // first piece of list entry i (workgroup-relative)
    __shared__ uint16_t sj[kFragsPerWg];          // fragment (workgroup-relative) of list entry i
    __shared__ uint32_t marks[kChains * 64];      // boundary scratch, 64 words per chain
    __shared__ StreamChain schain[kChains];
    __shared__ uint32_t chead[kChains], sopen[kChains], shead[kChains];
    __shared__ uint32_t sjoin[kChains];           // stream_join: the parts of the fragment chain c starts
    __shared__ uint32_t sres[kFragsPerWg];        // the workgroup's checksums, stored at the end
    __shared__ uint64_t wpieces[kWv];
    __shared__ uint32_t wcount[kWv];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, t = threadIdx.x;
    LAMPI_DIAG_STAMP(0);
    if constexpr (kDiag) {
        if (t == 0) {
            g_stream_diag[(size_t)blockIdx.x * 16 + 5] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (31 << 11));
            g_stream_diag[(size_t)blockIdx.x * 16 + 6] = (uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (31 << 11));
        }
    }
    size_t base = (size_t)blockIdx.x * fpg;
    uint32_t nwg = (uint32_t)min((size_t)fpg, n - base);
    if constexpr (IsSeg<Src>::value) {  // the plan's workgroups: plan[0] of them, segments [plan[1+i], plan[2+i])
        const uint32_t g = plan[0];
        if (blockIdx.x >= g) return;  // the launch is sized for the largest plan
        base = plan[1 + blockIdx.x];
        nwg = plan[2 + blockIdx.x] - (uint32_t)base;
    }

    FragInfo mine{nullptr, 0u, 0u, nullptr, 0u};
    if (t < nwg) mine = src.get(base + t);
    if (t < kChains) {
        chead[t] = 0u;
        sjoin[t] = 0u;  // read after the rows
    }
    auto nopre = [] {};
    if constexpr (kSum) {
        __syncthreads();
    } else if constexpr (kThreads == 256) {
        stage_tables<0, decltype(nopre), 3>(lds, img, nopre);  // no Horner tables; waits for the descriptors too
    } else {
        if (t < 256) {  // the table builders are written for 256 threads
            CombineBasis cb = issue_combine_basis<false>(img);
            char *b = reinterpret_cast<char *>(lds);
            build_slices(b);
            asm volatile("s_waitcnt vmcnt(0) ; lampi-wait %0 %1" : "+v"(cb.a), "+v"(cb.b) : : "memory");
            build_combine(b, cb);
        }
        __syncthreads();
    }
    LAMPI_DIAG_STAMP(7);
    const bool ne = t < nwg && mine.len != 0u;              // list entries: the non-empty fragments
    if (t < nwg && mine.len == 0u) sres[t] = kSum ? 0u : mine.partial;  // uicrc(p, 0, s) == s, uicsum(p, 0) == 0
    const uint64_t np = ne ? (((uint64_t)mine.len + (kPB - 1)) / kPB) : 0ull;
    // CRC pieces end at the fragment end, SUM pieces start at the fragment start
    const bool mis = ne && ((((uintptr_t)mine.addr) + (kSum ? 0u : mine.len)) & 15u) != 0u;
    uint64_t ip = np;
    uint32_t ic = ne ? 1u : 0u;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)ip, s, 64);
        const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(ip >> 32), s, 64);
        const uint32_t vc = (uint32_t)__shfl_up((int)ic, s, 64);
        if (lane >= (uint32_t)s) {
            ip += ((uint64_t)hi << 32) | lo;
            ic += vc;
        }
    }
    if (lane == 63u) {
        wpieces[wave] = ip;
        wcount[wave] = ic;
    }
    __syncthreads();
    uint64_t op = 0ull, total = 0ull;
    uint32_t oc = 0u, nne = 0u;
#pragma unroll
    for (uint32_t w = 0; w < kWv; ++w) {
        const uint64_t a = wpieces[w];
        const uint32_t b = wcount[w];
        if (w < wave) {
            op += a;
            oc += b;
        }
        total += a;
        nne += b;
    }
    const uint64_t ex = op + ip - np;
    const uint32_t li = oc + ic - (ne ? 1u : 0u);
    const uint64_t R = (total + 63u) >> 6;  // rows; chain c starts at piece 64 * floor(c * R / kChains)
    if (ne) {
        sdesc[li] = StreamDesc{(uint64_t)(uintptr_t)mine.addr, mine.len, mine.partial};
        sstart[li] = ex;
        sj[li] = (uint16_t)t;
#pragma unroll
        for (uint32_t c = 0; c < kChains; ++c) {
            const uint64_t pc = 64u * ((c * R) / kChains);
            if (ex <= pc && pc < ex + np) chead[c] = li;
        }
    }
    if (t == 0) sstart[nne] = total;
    __syncthreads();
    LAMPI_DIAG_STAMP(8);
    if (t < kChains) {
        StreamChain ch;
        ch.rs = 64u * ((t * R) / kChains);
        ch.end = t + 1 == kChains ? total : 64u * (((t + 1) * R) / kChains);
        ch.head = chead[t];
        ch.mid = sstart[ch.head] < ch.rs ? 1u : 0u;
        ch.cur = ch.mid ? ch.head : ch.head - 1u;
        if (t + 1 == kChains) {
            ch.b = nne;
        } else {
            const uint32_t hn = chead[t + 1];
            ch.b = sstart[hn] < ch.end ? hn + 1u : hn;
        }
        if (nne == 0) ch = StreamChain{0ull, 0ull, 0u, 0u, 0u, 0u};
        schain[t] = ch;
    }
    for (uint32_t i = t; i < kChains * 64; i += kThreads) marks[i] = 0u;
    const bool anymis = __syncthreads_or(mis) != 0;
    gbyte *zero = (gbyte *)(img + kImgZero);
    LAMPI_DIAG_STAMP(1);
    if (anymis)  // five loads per row: a one-slot ring keeps its registers within the aligned variant's
        stream_body<true, 1, kK, kSum, kDiag>(lds, sdesc, sstart, sj, marks + 64 * kK * wave, schain + kK * wave,
                                             sopen + kK * wave, shead + kK * wave, zero, sres, out);
    else
        stream_body<false, kD, kK, kSum, kDiag>(lds, sdesc, sstart, sj, marks + 64 * kK * wave, schain + kK * wave,
                                               sopen + kK * wave, shead + kK * wave, zero, sres, out);
    __syncthreads();
    LAMPI_DIAG_STAMP(3);
    // stream_join: fragments crossing chain starts, every chain's part at once.  A fragment f
    // crossing chains a (where it starts) .. b (where it ends) is the XOR (SUM: sum) of each
    // chain's part shifted past the rest of f: chains a..b-1 leave their open value (sopen),
    // chain b its final part (shead).  Thread c adds chain c's part of the fragment it starts
    // inside (head, mid) and of the fragment it starts that crosses its end into sjoin[start
    // chain]; the start chain's thread then stores the result.  (Round 1 joined the parts one
    // after another in one thread: a fragment spanning all twelve chains took eleven dependent
    // shifts, 256 KiB fragments one per workgroup ran at 47%.)
    uint32_t gown = ~0u;  // the crossing fragment this thread's chain starts (its result is stored here)
    if (t < kChains && schain[t].rs < schain[t].end) {
        const uint64_t rs = schain[t].rs, end = schain[t].end;
        if (schain[t].mid) {  // part of the fragment this chain starts inside
            const uint32_t h = schain[t].head;
            const uint64_t sf = sstart[h], ef = sstart[h + 1];
            uint32_t a = t;
            while (a > 0 && schain[a - 1].rs > sf) --a;  // a - 1: the chain holding h's first piece
            const uint32_t v = ef <= end ? shead[t] : (kSum ? sopen[t] : shift_pieces(lds, img, sopen[t], ef - end));
            if (kSum)
                atomicAdd(&sjoin[a - 1], v);
            else
                atomicXor(&sjoin[a - 1], v);
        }
        if (t + 1 < kChains) {  // the fragment open at this chain's end, when it starts here
            const uint32_t g = schain[t + 1].head;
            const uint64_t sg = sstart[g], eg = sstart[g + 1];
            if (sg >= rs && sg < end && eg > end) {
                const uint32_t v = kSum ? sopen[t] : shift_pieces(lds, img, sopen[t], eg - end);
                if (kSum)
                    atomicAdd(&sjoin[t], v);
                else
                    atomicXor(&sjoin[t], v);
                gown = g;
            }
        }
    }
    __syncthreads();
    if (gown != ~0u) sres[sj[gown]] = kSum ? sjoin[t] : __builtin_bswap32(sjoin[t]);
    __syncthreads();
    if (t >= nwg) return;
    if constexpr (HasSegments<Src>::value) {  // a segment: its fragment's value, or its part of a split one
        const SegDesc x = src.segment(base + t);
        if (x.rows == kSegSkip) return;
        uint32_t v = sres[t];
        if (!(x.rows & kSegSplit)) {
            out[x.frag] = v;
        } else if constexpr (kSum) {
            atomicAdd(out + x.frag, v);
        } else {
            atomicXor(out + x.frag, shift_rows(v, x.rows & ~kSegSplit));  // past the fragment's later rows
        }
    } else {
        emit(src, out, base + t, sres[t], mine);
    }
    LAMPI_DIAG_STAMP(4);
}

// The byte-balanced plan of a descriptor batch (n <= kPlanMax fragments, one 1024-thread workgroup):
//   T = total bytes; the window B = max(ceil(T / gb), min(384 KiB, max(64 KiB, ceil(T / 256)))), rounded
//   up to a power of two (shifts, not 64-bit divisions: those made a single-threaded plan of 16K
//   fragments take 60-75 us) -- at most gb windows (gb <= 2048 from the host), ~384-512 KiB per
//   workgroup (the table staging amortised, as the count split's 96 x 4 KiB) and about 256
//   workgroups for small batches (the prologue-bound sizes: DESIGN.md 6);
//   fragments longer than B -> ceil(len / B) segments (SegDesc, in fragment order);
//   workgroup i = segments [plan[1+i], plan[2+i]): a new one starts at segment 0, every kPlanF-th
//   segment, and where a segment starts in a new B-byte window of the batch -- at most kPlanF
//   segments and ~2B bytes each; plan[0] = the number of workgroups.
// out[f] of a split fragment is zeroed (its parts are XORed / added in).
constexpr uint32_t kPlanMax = 32768;
constexpr uint32_t kPlanF = 96;

// exclusive prefix sum over the kT threads of the workgroup (kT = 64: one wave, no barrier)
template <uint32_t kT>
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t *sh, uint64_t *total) {
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint64_t x = v;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        const uint64_t y = __shfl_up(x, s, 64);
        if (lane >= (uint32_t)s) x += y;
    }
    if constexpr (kT == 64) {
        *total = __shfl(x, 63, 64);
        return x - v;
    } else {
        if (lane == 63u) sh[w] = x;
        __syncthreads();
        uint64_t before = 0, all = 0;
#pragma unroll
        for (uint32_t i = 0; i < kT / 64; ++i) {
            if (i < w) before += sh[i];
            all += sh[i];
        }
        __syncthreads();
        *total = all;
        return before + x - v;
    }
}

// one wave for n <= 64 (a few microseconds less than the 1024-thread plan on every small call),
// 256 threads up to 2048 fragments, 1024 up to kPlanMax
template <uint32_t kT, uint32_t kMax>
__global__ void __launch_bounds__(kT) plan_kernel(const lampi_frag_desc *__restrict__ d, uint32_t n, int sum,
                                                  uint32_t gb, SegDesc *__restrict__ segs, uint32_t *__restrict__ plan,
                                                  uint32_t *__restrict__ out) {
    constexpr uint32_t kPlanThreads = kT;
    __shared__ uint32_t lens[kMax];
    __shared__ uint64_t sh[kT / 64 + 1];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < n; i += kPlanThreads) lens[i] = d[i].length;
    __syncthreads();
    const uint32_t per = (n + kPlanThreads - 1) / kPlanThreads;
    const uint32_t f0 = min(n, t * per), f1 = min(n, f0 + per);
    uint64_t mine = 0;
    for (uint32_t f = f0; f < f1; ++f) mine += lens[f];
    uint64_t T = 0;
    const uint64_t byte0 = block_excl_scan64<kT>(mine, sh, &T);
    const uint64_t want = max((T + gb - 1) / gb, min((uint64_t)384 << 10, max((uint64_t)64 << 10, (T + 255) / 256)));
    const uint32_t lb = 64u - (uint32_t)__clzll(want - 1);  // B = 2^lb >= want (>= 64 KiB)
    const uint64_t B = 1ull << lb;
    auto nseg = [&](uint32_t len) -> uint32_t { return len > B ? (uint32_t)(((uint64_t)len + B - 1) >> lb) : 1u; };
    // segment k of a fragment of len bytes cut into K: [a, e)
    auto seg = [&](uint32_t len, uint32_t K, uint32_t k, uint32_t *a, uint32_t *e) {
        if (sum) {
            *a = (uint32_t)((uint64_t)k << lb);
            *e = (uint32_t)min((uint64_t)len, (uint64_t)(k + 1) << lb);
        } else {
            *e = (uint32_t)(len - ((uint64_t)(K - 1 - k) << lb));
            *a = k == 0 ? 0u : (uint32_t)(*e - B);
        }
    };
    uint64_t kmine = 0;
    for (uint32_t f = f0; f < f1; ++f) kmine += nseg(lens[f]);
    uint64_t M = 0;
    const uint64_t seg0 = block_excl_scan64<kT>(kmine, sh, &M);
    // the segment before this thread's first one: the last segment of fragment f0 - 1
    uint64_t prev_len = 0;
    if (f0 > 0 && f0 < f1) {
        const uint32_t L = lens[f0 - 1], K = nseg(L);
        uint32_t a, e;
        seg(L, K, K - 1, &a, &e);
        prev_len = e - a;
    }
    // pass 1: write the segments, count workgroup starts
    uint32_t j = (uint32_t)seg0;  // segments < n + gb < 2^32
    uint64_t P = byte0, starts = 0;
    uint64_t Pprev = P - prev_len;
    for (uint32_t f = f0; f < f1; ++f) {
        const uint32_t L = lens[f], K = nseg(L);
        if (K > 1) out[f] = 0u;
        for (uint32_t k = 0; k < K; ++k, ++j) {
            uint32_t a, e;
            seg(L, K, k, &a, &e);
            const uint32_t rows = sum ? 0u : (K - 1 - k) << (lb - 12);
            segs[j] = SegDesc{f, a, e - a, rows | (K > 1 ? kSegSplit : 0u)};
            if (j == 0 || j % kPlanF == 0 || (P >> lb) != (Pprev >> lb)) ++starts;
            Pprev = P;
            P += e - a;
        }
    }
    uint64_t G = 0;
    const uint64_t g0 = block_excl_scan64<kT>(starts, sh, &G);
    // pass 2: the workgroup starts
    j = (uint32_t)seg0;
    P = byte0;
    Pprev = P - prev_len;
    uint32_t g = (uint32_t)g0;
    for (uint32_t f = f0; f < f1; ++f) {
        const uint32_t L = lens[f], K = nseg(L);
        for (uint32_t k = 0; k < K; ++k, ++j) {
            uint32_t a, e;
            seg(L, K, k, &a, &e);
            if (j == 0 || j % kPlanF == 0 || (P >> lb) != (Pprev >> lb)) plan[1 + g++] = j;
            Pprev = P;
            P += e - a;
        }
    }
    if (t == 0) {
        plan[0] = (uint32_t)G;
        plan[1 + G] = (uint32_t)M;
    }
}

// ---- CRC fused copy of messages, table-light (lampi_msg_bcopy) ------------------------------------
// The copy shape that reaches ~75% of read + write into GM ring slots on MI355X is one 4 KiB row per
// wave in short-lived 4-wave workgroups holding at most ~36 KiB of LDS, four per CU (the same with
// 52 / 80 KiB: 72% / 50%; tools/microbench/copy_occ.hip, profiles/r03/copy_occ.txt).  The 64 KiB
// table set of the other CRC kernels does not fit that, so this kernel keeps only
//   [0, 32 KiB)        the slicing tables in 128-byte rows: entry e of S_j, copy c at e*128 + j*32 + 4c.
//                      Lane octet g reads table q ^ g in instruction q: 32 distinct banks per 32-lane
//                      group.  One v_perm puts X's byte into bits 8..15 and twice the table offset into
//                      bits 0..7; a shift right by one makes the address.  Built from compile-time
//                      constants.
//   [32 KiB, +3.5 KiB) nibble tables of seven uniform shifts (every lane reads the same 16 entries per
//                      lookup: conflict free), copied from the table image: 1024 bytes, and 16 * 2^j
//                      bytes for j = 0..5
// and no per-lane combine tables.  Lane l holds the 16-byte chunks at 16l + 1024q of its row (q = 0..3,
// the coalesced layout: each load and store instruction covers 1 KiB).  It CRCs each chunk from a
// zero register (four independent chains of four words), joins them by Horner over the 1024-byte
// step, and a six-level DPP tree XORs shift_{16(63-l)}(R_l) over the lanes into lane 63.  A
// fragment's rows are right-aligned in a frame of R = ceil(L / 4096) rows (the leading padding reads
// as zeros, free for a zero register) and its register is injected into its first four bytes.
// R == 1: the row value is the fragment's checksum.  R > 1: row values go to scratch and
// crc_light_join_kernel shifts each past its fragment's later rows and XORs them.
// Preconditions (launch_msg_bcopy): base and frag_len and msg_len multiples of 16, dst and dst_stride
// of 4 (a dword-aligned dwordx4 store runs at the aligned rate).
constexpr int kBufNt = 2;  // buffer instruction cache policy: nt (gfx940+ CPol::NT, the SLC bit)
constexpr uint32_t kLtNib = 32768;
constexpr uint32_t kLtTab = 4 * kLightTableWords;  // bytes between the nibble tables
constexpr uint32_t kLtBytes = kLtNib + kLightTables * kLtTab;

// slicing tables in 128-byte rows (build_slices' fill with half the row stride), from the basis of the
// thread's table j in the image (bs: its 16 words, kImgSliceBasis) -- the per-lane selection of
// compile-time constants cost ~150 VALU per wave (gfx9 VALU takes no literal operands: every constant
// needed a v_mov), about a fifth of the kernel's VALU, which bounds it (SQ counters,
// profiles/r03/pmc_light_*)
// (kT = 256 * m: thread t takes rows part * 8 / m .. of thread t % 256's eight, part = t / 256)
template <int kT = 256>
__device__ __forceinline__ void build_slices_light(char *b, const u32x4 bs[4]) {
    static_assert(kT == 256 || kT == 512 || kT == 1024, "256, 512 or 1024 threads");
    constexpr int kRows = 8 * 256 / kT;
    const uint32_t t = threadIdx.x, r0 = (t >> 3) & 31u, part = t >> 8;  // (part: wave-uniform)
    uint32_t base = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) base ^= ((r0 >> i) & 1u) ? bs[i >> 2][i & 3] : 0u;
#pragma unroll
    for (int kk = 0; kk < kRows; ++kk) {
        uint32_t v = bs[(5 + kk) >> 2][(5 + kk) & 3];
#pragma unroll
        for (int p = 1; p < 256 * 8 / (kRows * 256); ++p) {
            const int i = 5 + p * kRows + kk;
            v = part == (uint32_t)p ? bs[i >> 2][i & 3] : v;
        }
        v ^= base;
        *reinterpret_cast<u32x4 *>(b + (r0 + 32 * (kk + kRows * part)) * 128 + (t & 7u) * 16) = u32x4{v, v, v, v};
    }
}

// register after the shift of nibble table `base` (a byte address in LDS; swapped domain)
// (the byte offsets of all eight lookups from two masks: a holds 4 * nibbles 0, 2, 4, 6 in its bytes, b
// 4 * nibbles 1, 3, 5, 7 -- one bit-field extract per lookup instead of a shift and a mask -- and the
// eight entries XORed as a three-input tree)
__device__ __forceinline__ uint32_t light_shift_at(const uint32_t *lds, uint32_t base, uint32_t C) {
    uint32_t a = (C << 2) & 0x3C3C3C3Cu, b = (C >> 2) & 0x3C3C3C3Cu;
    asm("" : "+v"(a), "+v"(b));  // (opaque: otherwise folded back into a shift and a mask per lookup)
    uint32_t e[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        e[2 * k] = lds_u32(lds, base + 128u * k + ((a >> (8 * k)) & 0xFFu));
        e[2 * k + 1] = lds_u32(lds, base + 128u * k + 64u + ((b >> (8 * k)) & 0xFFu));
    }
    return xor3(xor3(e[0], e[1], e[2]), xor3(e[3], e[4], e[5]), e[6]) ^ e[7];
}
template <int kTab>
__device__ __forceinline__ uint32_t light_shift(const uint32_t *lds, uint32_t C) {
    return light_shift_at(lds, kLtNib + kLtTab * kTab, C);
}

// four words from a zero register through the compact slicing tables
__device__ __forceinline__ uint32_t light_chunk(const uint32_t *lds, uint32_t lanec2, const uint32_t sel[4],
                                                const u32x4 &d) {
    auto look = [&](uint32_t X) {
        const uint32_t t0 = lds_u32(lds, __builtin_amdgcn_perm(X, lanec2, sel[0]) >> 1);
        const uint32_t t1 = lds_u32(lds, __builtin_amdgcn_perm(X, lanec2, sel[1]) >> 1);
        const uint32_t t2 = lds_u32(lds, __builtin_amdgcn_perm(X, lanec2, sel[2]) >> 1);
        const uint32_t t3 = lds_u32(lds, __builtin_amdgcn_perm(X, lanec2, sel[3]) >> 1);
        return Look4{t0, t1, t2, t3};
    };
    Look4 t = look(d.x);
    t = look(xor3(xor3(t.t0, t.t1, t.t2), t.t3, d.y));
    t = look(xor3(xor3(t.t0, t.t1, t.t2), t.t3, d.z));
    t = look(xor3(xor3(t.t0, t.t1, t.t2), t.t3, d.w));
    return xor3(t.t0, t.t1, t.t2) ^ t.t3;
}

// raw buffer descriptor over [p, p + bytes): loads past either end read zeros, stores there are dropped
// (gfx9 raw buffers, stride 0: the range check is offset >= num_records, in bytes)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t light_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}

template <int kWv = 4>
__global__ void __launch_bounds__(64 * kWv) crc_light_copy_kernel(const uint8_t *__restrict__ base, size_t msg_len,
                                                                  uint32_t frag_len, uint32_t R, size_t nitems,
                                                                  uint32_t partial, uint8_t *__restrict__ dst,
                                                                  size_t dst_stride, const uint32_t *__restrict__ img,
                                                                  uint32_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLtBytes / 4];
    const uint32_t t = threadIdx.x, lane = t & 63u;
    // (fragment, row) of this wave, wave-uniform: the fragment's source and slot become buffer
    // descriptors in SGPRs
    const size_t item = (size_t)blockIdx.x * kWv + __builtin_amdgcn_readfirstlane(t >> 6);
    const bool live = item < nitems;
    const size_t f = live ? item / R : 0;
    const uint32_t r = live ? (uint32_t)(item - f * R) : 0u;
    const size_t foff = f * frag_len;
    const uint32_t L = live ? (uint32_t)min((size_t)frag_len, msg_len - foff) : 0u;
    const uint32_t P = R * (uint32_t)kRowBytes - L;  // frame padding (a multiple of 16)
    // the uniform shift tables from the image (L2) first: vmcnt counts in order, so waiting for this
    // load leaves the row loads issued after it in flight
    // (396 16-byte pieces: two per thread for the first 140; the clamped rest load and store the last
    // piece again -- a load or store under a branch waits for itself before the row loads issue)
    constexpr uint32_t kNibPieces = kLightTables * kLightTableWords / 4;
    static_assert(kNibPieces > 256 && kNibPieces <= 512, "two nibble-table pieces per thread at most");
    const u32x4 nib = reinterpret_cast<const u32x4 *>(img + kImgLightNib)[min(t, kNibPieces - 1)];
    const uint32_t t2 = min(256u + t, kNibPieces - 1);
    u32x4 nib2 = nib;
    if constexpr (kWv == 4) nib2 = reinterpret_cast<const u32x4 *>(img + kImgLightNib)[t2];
    u32x4 bs[4];  // the slicing basis of table (t & 7) >> 1
#pragma unroll
    for (int i = 0; i < 4; ++i) bs[i] = reinterpret_cast<const u32x4 *>(img + kImgSliceBasis)[((t & 7u) >> 1) * 4 + i];
    // the row's chunks: frame offset 4096r + 1024q + 16l, fragment byte o[q] = that - P, through a
    // buffer descriptor of the fragment's L bytes: the frame padding (o < 0, a huge unsigned offset)
    // reads as zeros and its stores are dropped by the range check, with no select per chunk.  The
    // 1024q goes into the VGPR offset (not the instruction's): the check then never sees a wrapped sum.
    const __amdgpu_buffer_rsrc_t src_rs = light_rsrc(base + foff, L);
    const __amdgpu_buffer_rsrc_t dst_rs = light_rsrc(dst + f * dst_stride, L);
    uint32_t o[4];
    u32x4 d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        o[q] = r * (uint32_t)kRowBytes + 1024u * q + 16u * lane - P;
        asm volatile("" : "+v"(o[q]));  // (kept whole: the compiler would fold 1024q into the immediate)
        d[q] = __builtin_amdgcn_raw_buffer_load_b128(src_rs, o[q], 0, kBufNt);
    }
    // tables: slicing from the basis, then the uniform shifts, while the row loads fly
    build_slices_light<64 * kWv>(reinterpret_cast<char *>(lds), bs);
    reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds) + kLtNib)[min(t, kNibPieces - 1)] = nib;
    if constexpr (kWv == 4)
        reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds) + kLtNib)[t2] = nib2;  // (t >= 140: the last piece again)
    __syncthreads();
    if (!live) return;
    // the copy: every chunk of the fragment, 16-byte stores (dword-aligned slots run at the aligned rate)
#pragma unroll
    for (int q = 0; q < 4; ++q) __builtin_amdgcn_raw_buffer_store_b128(d[q], dst_rs, o[q], 0, kBufNt);
    // the fragment's register enters as data in its first four bytes (frame offset P)
    if ((P >> 12) == r && ((P >> 4) & 63u) == lane) {
        const uint32_t qi = (P >> 10) & 3u, inj = __builtin_bswap32(partial);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if ((uint32_t)q == qi) d[q].x ^= inj;
    }
    // lane constants: twice the table offsets j*32 + 4c (c = lane & 7), selectors for table q ^ octet
    const uint32_t c8 = (lane & 7u) * 8u;
    const uint32_t lanec2 = c8 | ((c8 + 64u) << 8) | ((c8 + 128u) << 16) | ((c8 + 192u) << 24);
    const uint32_t g = (lane >> 3) & 3u;
    uint32_t sel[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t j = (uint32_t)q ^ g;
        sel[q] = j | ((4u + j) << 8) | 0x0C0C0000u;
    }
    const uint32_t c0 = light_chunk(lds, lanec2, sel, d[0]);
    const uint32_t c1 = light_chunk(lds, lanec2, sel, d[1]);
    const uint32_t c2 = light_chunk(lds, lanec2, sel, d[2]);
    const uint32_t c3 = light_chunk(lds, lanec2, sel, d[3]);
    uint32_t v = light_shift<0>(lds, light_shift<0>(lds, light_shift<0>(lds, c0) ^ c1) ^ c2) ^ c3;
    // lane tree, three levels: after level j the last lane of every 2^(j+1)-lane block holds that block's
    // value relative to the block's end
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)light_shift<1>(lds, v), 0x111, 0xF, 0xF, false);  // row_shr:1
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)light_shift<2>(lds, v), 0x112, 0xF, 0xF, false);  // row_shr:2
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)light_shift<3>(lds, v), 0x114, 0xF, 0xF, false);  // row_shr:4
    // then each eight-lane group g (its last lane 8g + 7) shifts by 128 * (7 - g) to the row end through
    // its own table (tables 4..10, 576 bytes apart: groups 0..3 and 4..7 each read 64 distinct banks;
    // group 7 needs none) -- one lookup round instead of three more tree levels -- and the eight values
    // are XORed into lane 63: row_shr:8, row_bcast:15, row_bcast:31
    const uint32_t grp = lane >> 3;
    if (grp < 7u) v = light_shift_at(lds, kLtNib + kLtTab * (4u + grp), v);
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    if (lane == 63u) out[R == 1 ? f : item] = __builtin_bswap32(v);
}

// out[f] = XOR over the rows r of fragment f of row value r shifted past the R - 1 - r rows after it
// (normal domain).  R <= kJoinThreadRows: one thread per fragment, Horner over its rows with the
// constant multiply by x^(8 * 4096) (GM's 16 rows: 15 multiplies, a few VALU per fragment and row
// across the wave -- one wave per fragment spent ~420 VALU on each); longer fragments: one wave each,
// lanes take rows l, l + 64, ... and shift them directly.
constexpr uint32_t kJoinThreadRows = 32;
__global__ void __launch_bounds__(256) crc_light_join_kernel(const uint32_t *__restrict__ rows, size_t n, uint32_t R,
                                                             uint32_t *__restrict__ out) {
    if (R <= kJoinThreadRows) {
        const size_t f = (size_t)blockIdx.x * 256 + threadIdx.x;
        if (f >= n) return;
        const uint32_t *p = rows + f * R;
        uint32_t acc = p[0];
        for (uint32_t r = 1; r < R; ++r) acc = mul_row_shift<0>(acc) ^ p[r];
        out[f] = acc;
        return;
    }
    const size_t f = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (f >= n) return;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t acc = 0;
    for (uint32_t r = lane; r < R; r += 64) acc ^= shift_rows(rows[f * R + r], R - 1 - r);
    acc = wave_xor(acc);
    if (lane == 0) out[f] = acc;
}

// ---- CRC fused copy of descriptor batches, table-light (lampi_frag_bcopy_batch, CopyToApp) --------
// crc_light_copy_kernel's tables and row step for descriptors: one wave per fragment (fragment f of
// the batch = wave blockIdx.x * 4 + w), its rows walked in order with the next row's loads in flight,
// the Horner over the 1024-byte step carried from row to row (a lane's last chunk of a row and its
// first of the next are 1024 bytes apart too), one lane tree per fragment.  Any source and
// destination alignment, copylen <> csumlen: L = max(copylen, csumlen) bytes are checksummed in a
// right-aligned frame of R = ceil(L / 4096) rows (front padding P = 4096R - L, any byte count) read
// through a buffer descriptor of the L source bytes (padding reads zero); the chunk that straddles the
// fragment's start (P % 16 != 0) is rebuilt from the fragment's first 16 bytes.  The first copylen
// bytes go out through a buffer descriptor of the destination: whole chunks as 16-byte stores, the
// (at most two) chunks cut by the copy's start or end byte by byte -- their vector store is aimed out
// of range.  The register enters as data at frame offset P (any byte offset: two words).  Fragments
// under 16 bytes: one lane, byte steps on S_3.  Fragments up to 2^32 - 17 bytes.
__device__ __forceinline__ uint32_t pick4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, int i) {
    return i == 0 ? a : i == 1 ? b : i == 2 ? c : i == 3 ? d : 0u;
}
// 16 bytes (little endian) moved s bytes toward higher addresses, 0 < s < 16, zeros shifted in
__device__ __forceinline__ u32x4 shl_bytes16(const u32x4 &v, uint32_t s) {
    const int k = (int)(s >> 2);
    const uint32_t m = (s & 3u) * 8u;
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t lo = pick4(v.x, v.y, v.z, v.w, i - k);
        const uint32_t hi = pick4(v.x, v.y, v.z, v.w, i - k - 1);
        o[i] = m ? (lo << m) | (hi >> (32u - m)) : lo;
    }
    return u32x4{o[0], o[1], o[2], o[3]};
}

// Row groups (W > 1, LAMPI_CSUM_ROWS_HINT): fragment f runs as W waves, wave g taking rows
// [g*k, min((g+1)*k, R)) with k = ceil(R / W) -- GM's 16-row payloads one row per wave, the shape of the
// message copy -- and leaves the groups' values (each from a zero register, the first with the fragment's
// register in it, the lane tree at the group's last row) in groups[f*W + g]; crc_light_group_join_kernel
// shifts each past the fragment's later rows, XORs them and emits.  A fragment of one group emits here.
template <bool B>
struct BoolC {
    static constexpr bool value = B;
};
enum { kStepWalk, kStepHalf, kStepLast };
template <int M>
struct StepC {
    static constexpr int value = M;
};

// Bytes 0..nb-1 of v (nb <= 16, wave-uniform) to offsets ob.. of a buffer descriptor, on the lanes with
// `on` (the others aimed out of range): whole words as dword stores, then a short and a byte -- byte stores
// cost (sixteen of them per cut chunk: 445 against 489 us per GiB of IB copies for eight).  Unaligned dword
// stores are fine; bytes past the descriptor's range (copylen) are dropped, and the caller keeps ob + nb
// within it unless those bytes are to be dropped.
__device__ __forceinline__ void store_bytes(const u32x4 &v, __amdgpu_buffer_rsrc_t rs, bool on, uint32_t ob,
                                            uint32_t nb) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const uint32_t o = on ? ob : 0xFFFFFFF0u;  // (o + 15 < 2^32)
    const uint32_t nw = nb >> 2, rem = nb & 3u;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if ((uint32_t)i < nw) __builtin_amdgcn_raw_buffer_store_b32(w[i], rs, o + 4 * i, 0, kBufNt);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if ((uint32_t)i == nw && rem != 0) {
            if (rem & 2u) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)w[i], rs, o + 4 * i, 0, kBufNt);
            if (rem & 1u)
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w[i] >> (8 * (rem & 2u))), rs, o + 4 * i + (rem & 2u), 0,
                                                     kBufNt);
        }
}

// One fragment (or one row group of it) on one wave: geometry, source / destination descriptors and
// the row loads (ok false: offsets aimed out of range, no memory traffic -- a prefetch past the last
// row; hf: a half frame's row, chunks q = 0, 1 only).
struct LightFrag {
    FragInfo fi;
    uint32_t L, R, P, r0, r1;
    bool half, whole, live;
    __amdgpu_buffer_rsrc_t srs, drs;
    __device__ void init(const FragInfo &x, bool alive, uint32_t W, uint32_t g) {
        fi = x;
        live = alive;
        L = fi.len;
        R = (uint32_t)(((uint64_t)L + kRowBytes - 1) / kRowBytes);
        // fragments of at most 2 KiB take a half frame: chunks q = 0, 1 of the row (its first 2 KiB), half
        // the lookups of a 4 KiB frame (IB's 1,976-byte payloads were 52% padding)
        half = R == 1u && L <= (uint32_t)kRowBytes / 2u;
        P = (half ? (uint32_t)kRowBytes / 2u : R * (uint32_t)kRowBytes) - L;  // (L < 2^32 - 16)
        // this wave's rows [r0, r1) (all of them for W == 1); a group past the last row has nothing to do
        const uint32_t k = W > 1 ? (R + W - 1) / W : R;
        r0 = W > 1 ? min(g * k, R) : 0u;
        r1 = W > 1 ? min(r0 + k, R) : R;
        whole = W <= 1u;  // one wave per fragment: it emits the checksum (row groups: the join kernel, for all)
        if (W > 1 && g > 0u && r0 >= r1) live = false;
        srs = light_rsrc((const void *)fi.addr, L);
        drs = light_rsrc(fi.dst, fi.copylen);
    }
    __device__ void load_row(uint32_t lane, uint32_t r, bool ok, u32x4 (&d)[4], uint32_t (&o)[4],
                             bool hf = false) const {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            o[q] = (ok && (!hf || q < 2)) ? r * (uint32_t)kRowBytes + 1024u * q + 16u * lane - P : 0xFFFFFFF0u;
            asm volatile("" : "+v"(o[q]));  // whole offsets: padding offsets wrap to huge values, out of range
            d[q] = __builtin_amdgcn_raw_buffer_load_b128(srs, o[q], 0, kBufNt);
        }
    }
    // the fragment's first 16 bytes, for the chunk its start cuts (a load here rather than under that
    // branch: the compiler's merged waits after a branch with a load drained every row's prefetch)
    __device__ u32x4 load_head() const { return __builtin_amdgcn_raw_buffer_load_b128(srs, 0u, 0, 0); }
};

// lane constants of light_chunk: twice the table offsets j*32 + 4c (c = lane & 7), selectors for table
// q ^ octet
__device__ __forceinline__ void light_lane_consts(uint32_t lane, uint32_t &lanec2, uint32_t (&sel)[4]) {
    const uint32_t c8 = (lane & 7u) * 8u;
    lanec2 = c8 | ((c8 + 64u) << 8) | ((c8 + 128u) << 16) | ((c8 + 192u) << 24);
    const uint32_t oct = (lane >> 3) & 3u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t j = (uint32_t)q ^ oct;
        sel[q] = j | ((4u + j) << 8) | 0x0C0C0000u;
    }
}

// The register enters as data at frame offset P: bytes P..P+3 (two words when P % 4 != 0, chunk kP and,
// for P % 16 > 12, the next).  k(q): the frame chunk index of the lane's chunk q.
template <class KOf>
__device__ __forceinline__ void inject_register(u32x4 (&dc)[4], uint32_t P, uint32_t partial, KOf k_of) {
    const uint32_t kP = P >> 4, sP = P & 15u;
    const uint32_t inj = __builtin_bswap32(partial);
    const uint32_t w = sP >> 2, m = (sP & 3u) * 8u;
    const uint32_t lo = inj << m, hi = m ? inj >> (32u - m) : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t k = k_of(q);
        const uint32_t a = k == kP ? lo : 0u, b = k == kP ? hi : 0u;
        const uint32_t c = (k == kP + 1u && w == 3u) ? hi : 0u;
        dc[q].x ^= (w == 0 ? a : 0u) ^ c;
        dc[q].y ^= (w == 1 ? a : 0u) ^ (w == 0 ? b : 0u);
        dc[q].z ^= (w == 2 ? a : 0u) ^ (w == 1 ? b : 0u);
        dc[q].w ^= (w == 3 ? a : 0u) ^ (w == 2 ? b : 0u);
    }
}

// The rest of one fragment (group) on its wave, after the tables are in LDS: its first row (d, o) and
// head are already loaded.  Short fragments (under 16 bytes) run on lane 0.
// In row groups (F.whole false) every group hands its value (normal domain) to sink, the fragment's only
// group (and a short fragment's) too: the join kernel emits every fragment.
template <class Src, class Sink>
__device__ __forceinline__ void light_frag_run(const Src &src, size_t f, const LightFrag &F, const uint32_t *lds,
                                               uint32_t lane, uint32_t *out, Sink sink, u32x4 (&d)[4],
                                               uint32_t (&o)[4], const u32x4 &head) {
    const FragInfo &fi = F.fi;
    const uint32_t L = F.L, P = F.P, r0 = F.r0, r1 = F.r1;
    if (L < 16) {  // short fragments (and empty ones: the register itself)
        if (lane == 0) {
            uint32_t C = __builtin_bswap32(fi.partial);
            for (uint32_t i = 0; i < L; ++i) C = (C >> 8) ^ lds[((C ^ fi.addr[i]) & 255u) * 32u + 24u];
            if (F.whole)
                emit(src, out, f, __builtin_bswap32(C), fi);
            else
                sink(__builtin_bswap32(C));
        }
        if constexpr (Src::kCopy)
            if (lane < fi.copylen) ((gbyte_w *)fi.dst)[lane] = fi.addr[lane];
        return;
    }
    uint32_t lanec2, sel[4];
    light_lane_consts(lane, lanec2, sel);
    const uint32_t grp = lane >> 3;
    const uint32_t gbase = kLtNib + kLtTab * (4u + min(grp, 6u));
    const uint32_t kP = P >> 4, sP = P & 15u;        // the chunk holding the fragment's first byte, and where
    const uint64_t cend = (uint64_t)fi.copylen + P;  // the copy's end in the frame
    uint32_t acc = 0;
    // the copy of the chunk cut by the fragment's start: the head's first min(16 - sP, copylen) bytes at
    // offsets 0.. from the lane holding it (the chunk's own offsets start below zero, which is not out of
    // range once the compiler folds the byte index into the instruction offset; here, outside the row loop,
    // it costs no registers there)
    if constexpr (Src::kCopy)
        if (r0 == 0 && sP != 0) store_bytes(head, F.drs, lane == (kP & 63u), 0u, min(16u - sP, fi.copylen));
    // (hf: BoolC<true> for a half frame -- its own copy of the body, kept out of the row loop)
    // (mode: kStepWalk a row with the next row's loads in flight, kStepHalf a half frame, kStepLast a group's only
    // row -- no prefetch: its four loads aimed out of range still took address-pipeline slots)
    auto step = [&](auto mode, uint32_t r, u32x4 (&dc)[4], const uint32_t (&oc)[4], u32x4 (&dn)[4],
                    uint32_t (&on)[4]) {
        if constexpr (decltype(mode)::value == kStepWalk) F.load_row(lane, r + 1, r + 1 < r1, dn, on);
        if (r == 0 && sP != 0) {  // the chunk cut by the fragment's start: [zeros | first 16 - sP bytes]
            const u32x4 v = shl_bytes16(head, sP);
            const bool mine = lane == (kP & 63u);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if ((uint32_t)q == (kP >> 6) && mine) dc[q] = v;
        }
        // the copy: whole chunks of [P, cend) as 16-byte stores (the others aimed out of range)
        const uint32_t rbase = r * (uint32_t)kRowBytes + 16u * lane;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t x = rbase + 1024u * q;
            const bool full = x >= P && x + 16u <= cend;
            if constexpr (Src::kCopy)
                __builtin_amdgcn_raw_buffer_store_b128(dc[q], F.drs, full ? oc[q] : 0xFFFFFFF0u, 0, kBufNt);
        }
        // chunks cut by the copy's start or end (at most two per fragment, wave-uniform frame chunks kP and
        // kE): sixteen byte stores from one lane each, through the destination's buffer descriptor, whose
        // range check drops the bytes past copylen -- the start's bytes from the fragment's first 16 (the
        // head) at offsets 0..15, so no offset is below zero (a wrapped one is not out of range once the
        // compiler folds the byte index into the instruction offset)
        if constexpr (Src::kCopy) {
            const bool any = fi.copylen != 0;
            // the end (the start went out with the head, above): the chunk holding the copy's last byte
            // (16 kE >= P: no offset below zero)
            const uint64_t kE = (cend - 1) >> 4;
            if (any && (cend & 15u) != 0 && (kE >> 8) == r && !(sP != 0 && kE == kP) && lane == (kE & 63u)) {
                const uint32_t qk = (uint32_t)(kE >> 6) & 3u;
                const u32x4 v = qk == 0 ? dc[0] : qk == 1 ? dc[1] : qk == 2 ? dc[2] : dc[3];
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                const uint32_t ob = (uint32_t)(16u * kE - P);
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w[j >> 2] >> (8 * (j & 3))), F.drs, ob + j, 0, kBufNt);
            }
        }
        // the register: in row 0, or row 1 when kP is row 0's last chunk
        if (r == 0 || (r == 1 && kP == 255u))
            inject_register(dc, P, fi.partial, [&](int q) { return 256u * r + lane + 64u * q; });
        const uint32_t c0 = light_chunk(lds, lanec2, sel, dc[0]);
        const uint32_t c1 = light_chunk(lds, lanec2, sel, dc[1]);
        if constexpr (decltype(mode)::value == kStepHalf) {  // (one row: r == r0 == 0; chunks 2, 3 lie past the frame)
            acc = light_shift<0>(lds, c0) ^ c1;
        } else {
            const uint32_t c2 = light_chunk(lds, lanec2, sel, dc[2]);
            const uint32_t c3 = light_chunk(lds, lanec2, sel, dc[3]);
            const uint32_t v0 = r == r0 ? c0 : light_shift<0>(lds, acc) ^ c0;
            acc = light_shift<0>(lds, light_shift<0>(lds, light_shift<0>(lds, v0) ^ c1) ^ c2) ^ c3;
        }
        if (r + 1 == r1) {
            uint32_t v = acc;
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)light_shift<1>(lds, v), 0x111, 0xF, 0xF, false);
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)light_shift<2>(lds, v), 0x112, 0xF, 0xF, false);
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)light_shift<3>(lds, v), 0x114, 0xF, 0xF, false);
            const uint32_t wv = light_shift_at(lds, gbase, v);
            v = grp < 7u ? wv : v;
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
            if (lane == 63u) {
                if (F.whole)
                    emit(src, out, f, __builtin_bswap32(v), fi);
                else
                    sink(__builtin_bswap32(v));
            }
        }
    };
    u32x4 d2[4];
    uint32_t o2[4];
    if (F.half) {
        step(StepC<kStepHalf>{}, 0u, d, o, d2, o2);
        return;
    }
    if (r1 - r0 == 1u) {  // a 4 KiB fragment, or a row group of one row (GM's row groups)
        step(StepC<kStepLast>{}, r0, d, o, d2, o2);
        return;
    }
    for (uint32_t r = r0; r < r1; r += 2) {
        step(StepC<kStepWalk>{}, r, d, o, d2, o2);
        if (r + 1 >= r1) break;
        step(StepC<kStepWalk>{}, r + 1, d2, o2, d, o);
    }
}

// One fragment (or row group) per wave: item = 4 * blockIdx.x + wave, four waves per workgroup.
template <class Src, int kWv = 4>
__global__ void __launch_bounds__(64 * kWv) crc_light_frag_copy_kernel(const Src src, size_t n,
                                                                       const uint32_t *__restrict__ img,
                                                                       uint32_t *__restrict__ out, uint32_t W,
                                                                       uint32_t *__restrict__ groups) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLtBytes / 4];
    const uint32_t t = threadIdx.x, lane = t & 63u;
    const size_t item = (size_t)blockIdx.x * kWv + __builtin_amdgcn_readfirstlane(t >> 6);
    constexpr uint32_t kNibPieces = kLightTables * kLightTableWords / 4;
    const u32x4 nib = reinterpret_cast<const u32x4 *>(img + kImgLightNib)[min(t, kNibPieces - 1)];
    const uint32_t t2 = min(256u + t, kNibPieces - 1);
    u32x4 nib2 = nib;
    if constexpr (kWv == 4) nib2 = reinterpret_cast<const u32x4 *>(img + kImgLightNib)[t2];
    u32x4 bs[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bs[i] = reinterpret_cast<const u32x4 *>(img + kImgSliceBasis)[((t & 7u) >> 1) * 4 + i];
    const size_t f = item / W;
    const uint32_t g = (uint32_t)(item - f * W);
    FragInfo fi{nullptr, 0u, 0u, nullptr, 0u};
    if (f < n) fi = src.get(f);
    LightFrag F;
    F.init(fi, f < n && !(IsSplit<Src>::value && fi.aux), W, g);
    if constexpr (IsRecv<Src>::value)  // row groups: the join kernel gives every verdict, this launch zeroes them
        if (W > 1u && lane == 0u && f < n && g == 0u) zero_verdict_words(src, f);
    u32x4 d[4];
    uint32_t o[4];
    // the first row's loads before the table staging (after it: 4 KiB copies 73 -> 66%, profiles/r04/late_loads_ab.txt)
    F.load_row(lane, F.r0, F.live, d, o, F.half);  // (an empty or dead wave's descriptor reads nothing but zeros)
    const u32x4 head = F.load_head();
    if constexpr (IsSplit<Src>::value || IsSparse<Src>::value)  // the size split's light launch: most workgroups
        if (!__syncthreads_or(F.live)) return;  // hold no fragment of its class and leave before staging the tables
    build_slices_light<64 * kWv>(reinterpret_cast<char *>(lds), bs);
    reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds) + kLtNib)[min(t, kNibPieces - 1)] = nib;
    if constexpr (kWv == 4) reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds) + kLtNib)[t2] = nib2;
    __syncthreads();
    if (!F.live) return;
    light_frag_run(src, f, F, lds, lane, out, [&](uint32_t v) { groups[f * W + g] = v; }, d, o, head);
}

// IB-sized fragments two to a wave (crc_light_pair_copy_kernel; the launcher picks it when the stream's
// learned batch shape says every sampled fragment was at most 2 KiB): a 4-wave workgroup takes eight
// fragments, wave w fragments 2w and 2w + 1, half-wave h (lanes 32h .. 32h + 31) one of them in a 2 KiB
// half frame (front padding P = 2048 - L).  Lane l' = l & 31 holds the frame's chunks k = 32q + l' (frame
// bytes 512q + 16l', q = 0..3): four chunks, as a lane of a 4 KiB row has, so a wave does one row's
// lookups for two fragments and the workgroup's table staging serves eight (one wave per 1,976-byte IB
// payload spent a whole wave's prologue and tree on 4 KB of traffic).  Each half's geometry is
// wave-uniform (its descriptor is a scalar load).  Loads are global with per-lane addresses (two
// fragments: no single buffer descriptor), chunks wholly in the padding reading the table image's zero
// chunk; the chunk cut by the fragment's start is rebuilt from its first 16 bytes.  Stores go through a
// buffer descriptor per half, every store instruction issued by every lane with the offsets of lanes
// that must not store aimed out of range -- whole chunks as 16-byte stores, the chunks cut by the
// copy's ends as sixteen byte stores -- so no memory operation sits under a branch (the compiler's
// merged waits after a branch with a store waited for every store to complete: 760 us against 520 per
// GiB, profiles/r04/pairs_ab.txt).  Horner over the 512-byte step (light group table 3), a three-level
// lane tree within 16-lane rows, the 8-lane groups shifted by 128 (3 - g') (light group tables 8..10) and
// row_shr:8 + row_bcast:15 leave the fragments' values in lanes 31 and 63.  A wave holding a fragment
// under 16 bytes or over 2 KiB stages its part of the tables, leaves its index in a per-stream list and
// exits; crc_light_pair_leftover_kernel, launched after it, runs those waves' two fragments through
// light_frag_run (rare; inside this kernel the walk's registers took it from 52 to 137 VGPRs).
// Fragments f0 and f0 + 1 (if < n) of a leftover pair, each on the whole wave through light_frag_run.
template <class Src>
__device__ __forceinline__ void light_pair_fallback(const Src src, size_t f0, size_t n, const uint32_t *lds,
                                                    uint32_t lane, uint32_t *out) {
#pragma nounroll
    for (uint32_t k = 0; k < 2; ++k) {
        const size_t f = f0 + k;
        if (f >= n) break;
        LightFrag F;
        F.init(src.get(f), true, 1u, 0u);
        u32x4 dd[4];
        uint32_t oo[4];
        F.load_row(lane, F.r0, F.live, dd, oo, F.half);
        const u32x4 hh = F.load_head();
        light_frag_run(src, f, F, lds, lane, out, [](uint32_t) {}, dd, oo, hh);
    }
}

template <class Src, int kWv = 4>
__global__ void __launch_bounds__(64 * kWv) crc_light_pair_copy_kernel(const Src src, size_t n,
                                                                       const uint32_t *__restrict__ img,
                                                                       uint32_t *__restrict__ out, uint32_t *left,
                                                                       uint32_t *__restrict__ list) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLtBytes / 4];
    const uint32_t t = threadIdx.x, lane = t & 63u;
    const size_t wave = (size_t)blockIdx.x * kWv + __builtin_amdgcn_readfirstlane(t >> 6), f0 = wave * 2;
    constexpr uint32_t kNibPieces = kLightTables * kLightTableWords / 4;
    const u32x4 nib = reinterpret_cast<const u32x4 *>(img + kImgLightNib)[min(t, kNibPieces - 1)];
    const uint32_t t2 = min(256u + t, kNibPieces - 1);
    u32x4 nib2 = nib;
    if constexpr (kWv == 4) nib2 = reinterpret_cast<const u32x4 *>(img + kImgLightNib)[t2];
    u32x4 bs[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bs[i] = reinterpret_cast<const u32x4 *>(img + kImgSliceBasis)[((t & 7u) >> 1) * 4 + i];
    FragInfo fa{nullptr, 0u, 0u, nullptr, 0u}, fb{nullptr, 0u, 0u, nullptr, 0u};
    const bool la = f0 < n, lb = f0 + 1 < n;
    if (la) fa = src.get(f0);
    if (lb) fb = src.get(f0 + 1);
    auto pairable = [](const FragInfo &x) { return x.len >= 16u && x.len <= (uint32_t)kRowBytes / 2u; };
    const bool pair = la && pairable(fa) && (!lb || pairable(fb));  // (wave-uniform)
    // this lane's half: its fragment's chunks and first 16 bytes, loaded before the table staging
    const uint32_t h = lane >> 5, lp = lane & 31u;
    const bool live = pair && (h ? lb : la);
    gbyte *const addr = h ? fb.addr : fa.addr;
    const uint32_t L = h ? fb.len : fa.len;
    const uint32_t P = (uint32_t)kRowBytes / 2u - L;  // (a live half: 16 <= L <= 2048)
    gbyte *zero = (gbyte *)(img + kImgZero);
    u32x4 d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t x = 512u * q + 16u * lp;  // frame offset of the chunk
        d[q] = ld16c((gu32x4_a1 *)(live && x >= P ? addr + (x - P) : zero));
    }
    u32x4 head = ld16c((gu32x4_a1 *)(live ? addr : zero));
    build_slices_light<64 * kWv>(reinterpret_cast<char *>(lds), bs);
    // (eight waves: one nibble-table piece per thread, the clamped rest storing the last piece again)
    reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds) + kLtNib)[min(t, kNibPieces - 1)] = nib;
    if constexpr (kWv == 4) reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds) + kLtNib)[t2] = nib2;
    __syncthreads();
    if (!la) return;
    if (!pair) {  // left to crc_light_pair_leftover_kernel
        if (lane == 0) list[atomicAdd(left, 1u)] = (uint32_t)wave;
        return;
    }
    // the chunk loads complete, and seen by the compiler as defined here: its waitcnt pass otherwise lost
    // track of them across the branches below and put a vmcnt(0) -- every store issued so far -- before
    // each byte store
    asm volatile("s_waitcnt vmcnt(0) ; lampi-wait %0 %1 %2 %3 %4"
                 : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(head)::"memory");
    const uint32_t kP = P >> 4, sP = P & 15u;
    if (live && sP != 0 && (kP & 31u) == lp) {  // the chunk cut by the fragment's start
        const u32x4 v = shl_bytes16(head, sP);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if ((uint32_t)q == (kP >> 5)) d[q] = v;
    }
    if constexpr (Src::kCopy) {
        const __amdgpu_buffer_rsrc_t rs0 = light_rsrc(fa.dst, fa.copylen), rs1 = light_rsrc(fb.dst, lb ? fb.copylen : 0u);
        const uint32_t cend = P + (h ? fb.copylen : fa.copylen);  // the copy's end in the frame (<= 2048)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t x = 512u * q + 16u * lp;
            const bool full = live && x >= P && x + 16u <= cend;
            __builtin_amdgcn_raw_buffer_store_b128(d[q], rs0, full && h == 0 ? x - P : 0xFFFFFFF0u, 0, kBufNt);
            __builtin_amdgcn_raw_buffer_store_b128(d[q], rs1, full && h == 1 ? x - P : 0xFFFFFFF0u, 0, kBufNt);
        }
        // the chunks cut by the copy's start or end (frame chunks kc, wave-uniform per half): sixteen byte
        // stores, only the lane holding the chunk aimed in range; the descriptor's range check drops the
        // bytes outside [0, copylen)
        auto cut = [&](const FragInfo &x, uint32_t hh, const __amdgpu_buffer_rsrc_t &rs) {
            if (x.copylen == 0) return;
            const uint32_t Px = (uint32_t)kRowBytes / 2u - x.len, kPx = Px >> 4, sPx = Px & 15u;
            const uint32_t ce = Px + x.copylen, kE = (ce - 1) >> 4;
            // the start: the head's first 16 - sP bytes at offsets 0.. (the half's first lane holds the same
            // head; the rest of the chunk belongs to the next, whole one)
            if (sPx != 0) store_bytes(head, rs, lane == 32u * hh, 0u, min(16u - sPx, x.copylen));
            if ((ce & 15u) != 0 && !(sPx != 0 && kE == kPx)) {
                const int qk = (int)(kE >> 5);  // (component selects: a select of whole vectors went to scratch)
                const u32x4 v = {pick4(d[0].x, d[1].x, d[2].x, d[3].x, qk), pick4(d[0].y, d[1].y, d[2].y, d[3].y, qk),
                                 pick4(d[0].z, d[1].z, d[2].z, d[3].z, qk), pick4(d[0].w, d[1].w, d[2].w, d[3].w, qk)};
                store_bytes(v, rs, lane == 32u * hh + (kE & 31u), 16u * kE - Px, ce & 15u);
            }
        };
        cut(fa, 0u, rs0);
        if (lb) cut(fb, 1u, rs1);
    }
    // the register enters as data at frame offset P: words w, w + 1 of chunk kP (shifted by sP % 4 bytes),
    // spilling into chunk kP + 1 for w = 3 -- wave-uniform per half, only the lanes holding those chunks
    // change
    auto inject = [&](const FragInfo &x, uint32_t hh) {
        const uint32_t Px = (uint32_t)kRowBytes / 2u - x.len, kPx = Px >> 4, sPx = Px & 15u;
        const uint32_t inj = __builtin_bswap32(x.partial), w = sPx >> 2, m = (sPx & 3u) * 8u;
        const uint32_t lo = inj << m, hi = m ? inj >> (32u - m) : 0u;
        auto xor_word = [&](uint32_t k, uint32_t c, uint32_t val) {  // (k, c uniform)
            if (lane != 32u * hh + (k & 31u)) return;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if ((uint32_t)q == (k >> 5)) {
                    if (c == 0) d[q].x ^= val;
                    else if (c == 1) d[q].y ^= val;
                    else if (c == 2) d[q].z ^= val;
                    else d[q].w ^= val;
                }
        };
        xor_word(kPx, w, lo);
        if (hi != 0u) xor_word(w == 3u ? kPx + 1u : kPx, w == 3u ? 0u : w + 1u, hi);
    };
    inject(fa, 0u);
    if (lb) inject(fb, 1u);
    uint32_t lanec2, sel[4];
    light_lane_consts(lane, lanec2, sel);
    constexpr uint32_t kShift512 = kLtNib + kLtTab * (4u + 3u);  // group table 3: 128 * (7 - 3) bytes
    const uint32_t c0 = light_chunk(lds, lanec2, sel, d[0]);
    const uint32_t c1 = light_chunk(lds, lanec2, sel, d[1]);
    const uint32_t c2 = light_chunk(lds, lanec2, sel, d[2]);
    const uint32_t c3 = light_chunk(lds, lanec2, sel, d[3]);
    uint32_t v = light_shift_at(lds, kShift512, light_shift_at(lds, kShift512, light_shift_at(lds, kShift512, c0) ^ c1) ^ c2) ^ c3;
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)light_shift<1>(lds, v), 0x111, 0xF, 0xF, false);  // row_shr:1
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)light_shift<2>(lds, v), 0x112, 0xF, 0xF, false);  // row_shr:2
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)light_shift<3>(lds, v), 0x114, 0xF, 0xF, false);  // row_shr:4
    // group g' = (lane >> 3) & 3 of the half: shift by 128 (3 - g') through light group table 8 + g'
    const uint32_t gq = (lane >> 3) & 3u;
    const uint32_t wv = light_shift_at(lds, kLtNib + kLtTab * (8u + min(gq, 2u)), v);
    v = gq < 3u ? wv : v;
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 (rows 1, 3)
    if (lp == 31u && (h ? lb : la)) emit(src, out, f0 + h, __builtin_bswap32(v), h ? fb : fa);
}

// The pair kernel's leftover waves (list[0 .. *left): wave indices, two fragments each) on a fixed grid: a
// workgroup stages the tables only if one of its waves has an entry.  Calls alternate between two counters:
// this one zeroes the other, which the stream's next call counts in (no workgroup ever waits for another).
template <class Src>
__global__ void __launch_bounds__(256) crc_light_pair_leftover_kernel(const Src src, size_t n,
                                                                      const uint32_t *__restrict__ img,
                                                                      uint32_t *__restrict__ out, const uint32_t *left,
                                                                      uint32_t *next_left,
                                                                      const uint32_t *__restrict__ list,
                                                                      uint32_t *shape_nhalf) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLtBytes / 4];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = __builtin_amdgcn_readfirstlane(t >> 6);
    const uint32_t c = __builtin_amdgcn_readfirstlane(__hip_atomic_load(left, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    // leftovers: the stream's batches are no longer all IB-sized -- tell the host's next call (the learned
    // shape's count of fragments <= 2 KiB, host-mapped) before the census would
    if (c != 0 && blockIdx.x == 0 && t == 0 && shape_nhalf) {
        *(volatile uint32_t *)shape_nhalf = 0u;
        __threadfence_system();
    }
    if (blockIdx.x * 4u < c) {
        constexpr uint32_t kNibPieces = kLightTables * kLightTableWords / 4;
        const u32x4 nib = reinterpret_cast<const u32x4 *>(img + kImgLightNib)[t];
        const uint32_t t2 = min(256u + t, kNibPieces - 1);
        const u32x4 nib2 = reinterpret_cast<const u32x4 *>(img + kImgLightNib)[t2];
        u32x4 bs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            bs[i] = reinterpret_cast<const u32x4 *>(img + kImgSliceBasis)[((t & 7u) >> 1) * 4 + i];
        build_slices_light(reinterpret_cast<char *>(lds), bs);
        reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds) + kLtNib)[t] = nib;
        reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(lds) + kLtNib)[t2] = nib2;
        __syncthreads();
        for (uint32_t e = blockIdx.x * 4u + w; e < c; e += gridDim.x * 4u)
            light_pair_fallback(src, (size_t)list[e] * 2, n, lds, lane, out);
    }
    if (blockIdx.x == 0 && t == 0) *next_left = 0u;  // the stream's next call counts there
}

// The fragments of more than one row group: value = XOR over the groups of group g shifted past the rows
// after it (normal domain, constant products), then emit (receive sources: the verdict).  G = min(64,
// pow2 >= W) lanes per fragment, lane j taking groups j, j + G, ... (each shift independent of the
// others: one thread walking 64 groups by Horner waited on 64 dependent rounds, ~25 us for 4 MiB
// fragments of 16-row groups; a whole wave per fragment of 4 groups cost 16 KiB copies 4 points).
template <class Src>
__global__ void __launch_bounds__(256) crc_light_group_join_kernel(const Src src, size_t n, uint32_t W, uint32_t G,
                                                                   const uint32_t *__restrict__ groups,
                                                                   uint32_t *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x, f = i / G;
    const uint32_t j = (uint32_t)(i & (G - 1u));
    if (f >= n) return;  // (the G lanes of a fragment leave or stay together)
    const FragInfo fi = src.get(f);
    const uint32_t R = (uint32_t)(((uint64_t)fi.len + kRowBytes - 1) / kRowBytes);
    const uint32_t *p = groups + f * W;
    if (fi.len < 16u || R <= 1u) {  // (one group: its value as it is)
        if (j == 0) emit(src, out, f, p[0], fi);
        return;
    }
    const uint32_t k = (R + W - 1) / W, ng = (R + k - 1) / k;
    uint32_t acc = 0;
    for (uint32_t g = j; g < ng; g += G) acc ^= shift_rows(p[g], R - min((g + 1u) * k, R));
    for (uint32_t o = G >> 1; o >= 1u; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, (int)o);
    if (j == 0) emit(src, out, f, acc, fi);
}

// workgroups of the leftover launch (four waves each; the leftover path is rare).  32 instead: the IB receive
// and the 4 KiB descriptor lines unchanged (60.6-60.9%, 80.9%: the empty launch costs nothing visible in-stream).
constexpr unsigned kLeftoverWgs = 256;

template <class Src>
static hipError_t launch_crc_light_pair_copy(const Src &src, size_t n, const uint32_t *img, uint32_t *out,
                                             hipStream_t s, uint32_t *shape_nhalf) {
    uint32_t *left = nullptr, *next_left = nullptr, *list = nullptr;
    static const int kWv = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_PAIR_WAVES");
        return e && e[0] == '1' ? 16 : e && e[0] == '4' ? 4 : 8;
    }();
    const size_t nwg = (n + 2 * kWv - 1) / (2 * kWv);
    bool pooled = false;
    // (one entry per wave at most: a batch whose shape changed since the census leaves every wave)
    hipError_t e = stream_scratch(s, nwg * kWv * sizeof(uint32_t), (void **)&list, &pooled);
    if (e != hipSuccess) return e;
    // the counter pair is taken only now: a failure before this point leaves it untouched
    e = pair_counters(s, &left, &next_left);
    if (e != hipSuccess) return scratch_done(s, list, pooled, e);
    if (kWv == 16)
        hipLaunchKernelGGL((crc_light_pair_copy_kernel<Src, 16>), dim3((unsigned)nwg), dim3(1024), 0, s, src, n, img, out,
                           left, list);
    else if (kWv == 8)
        hipLaunchKernelGGL((crc_light_pair_copy_kernel<Src, 8>), dim3((unsigned)nwg), dim3(512), 0, s, src, n, img, out,
                           left, list);
    else
        hipLaunchKernelGGL((crc_light_pair_copy_kernel<Src, 4>), dim3((unsigned)nwg), dim3(256), 0, s, src, n, img, out,
                           left, list);
    e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(crc_light_pair_leftover_kernel<Src>, dim3(kLeftoverWgs), dim3(256), 0, s, src, n, img, out,
                           (const uint32_t *)left, next_left, (const uint32_t *)list, shape_nhalf);
        e = hipGetLastError();
    }
    // a launch that failed left a counter unzeroed (the leftover kernel zeroes the next call's): zero both
    if (e != hipSuccess) reset_pair_counters(s);
    return scratch_done(s, list, pooled, e);
}

// waves per workgroup of the table-light copy kernels: four (the copy shape, four 36 KiB workgroups per CU).
// Eight (the same LDS, twice the waves per CU) lost 3-7 points on the copies and the read-only walk and was
// box-dependent on the receive step (profiles/r04/light_waves_ab.txt, recv_waves_ab.txt); with the
// single-row step (95 VGPRs) it lost there too: GM receive 72.2 against 69.0% (profiles/r04/last_row_ab.txt).
// A/B knob LAMPI_LIGHT_WAVES = 4, 8, 16.
static int light_waves(bool recv = false) {
    (void)recv;
    static const int w = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_LIGHT_WAVES");
        return e && e[0] == '1' ? 16 : e && e[0] == '8' ? 8 : 4;
    }();
    return w;
}

// W: row groups per fragment (1: one wave walks all the fragment's rows)
// the row groups a light launch runs with for a hint of W
static uint32_t light_groups(size_t n, uint32_t W) {
    W = min(W, 4096u);  // (the join: at most 64 groups per lane)
    while (W > 1 && (size_t)n * W > ((size_t)1 << 26)) W >>= 1;  // (grid: items * 64 threads < 2^32)
    return W;
}

template <class Src>
static hipError_t launch_crc_light_frag_copy(const Src &src, size_t n, const uint32_t *img, uint32_t *out,
                                             hipStream_t s, uint32_t W = 1) {
    W = light_groups(n, W);
    const int kWv = light_waves(IsRecv<Src>::value);
    auto launch = [&](size_t items, uint32_t *groups) {
        if (kWv == 16)
            hipLaunchKernelGGL((crc_light_frag_copy_kernel<Src, 16>), dim3((unsigned)((items + 15) / 16)), dim3(1024), 0,
                               s, src, n, img, out, W, groups);
        else if (kWv == 8)
            hipLaunchKernelGGL((crc_light_frag_copy_kernel<Src, 8>), dim3((unsigned)((items + 7) / 8)), dim3(512), 0, s,
                               src, n, img, out, W, groups);
        else
            hipLaunchKernelGGL((crc_light_frag_copy_kernel<Src, 4>), dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s,
                               src, n, img, out, W, groups);
    };
    if (W <= 1) {
        W = 1;
        launch(n, nullptr);
        return hipGetLastError();
    }
    uint32_t *groups = nullptr;
    bool pooled = false;
    hipError_t e = stream_scratch(s, n * W * sizeof(uint32_t), (void **)&groups, &pooled);
    if (e != hipSuccess) return e;
    launch(n * W, groups);
    e = hipGetLastError();
    if (e == hipSuccess) {
        uint32_t G = 1;
        while (G < W && G < 64u) G <<= 1;
        hipLaunchKernelGGL(crc_light_group_join_kernel<Src>, dim3((unsigned)((n * G + 255) / 256)), dim3(256), 0, s, src,
                           n, W, G, groups, out);
        e = hipGetLastError();
    }
    return scratch_done(s, groups, pooled, e);
}

// ---- CRC fast path: regular batches -------------------------------------------------------
// Fragment f = base + f*frag_len, frag_len = R*4096, base 16-byte aligned (P = 0, no masks).
// A wave checksums kChains of its fragments at once (independent lookup chains interleaved:
// with two waves per SIMD one chain's LDS latency, ~1 us per row, is too close to the
// ~1.3 us of HBM time per row).  Steps (kChains rows) flow through three register buffers
// -- two steps in flight while one is checksummed -- and the next loads are always issued
// (clamped to the last step), so the hot loop has no load-side branches.
struct GroupTask {
    uint32_t i, r;  // fragments kChains*i .. kChains*i + kChains-1 of this wave's list, row r
};

template <int K>
struct RowsK {
    Row x[K];
};

template <int N, int K>
__device__ __forceinline__ void wait_rows(RowsK<K> &b) {
    if constexpr (K == 1) {
        asm volatile("s_waitcnt vmcnt(%4) ; lampi-wait %0 %1 %2 %3"
                     : "+v"(b.x[0].q[0]), "+v"(b.x[0].q[1]), "+v"(b.x[0].q[2]), "+v"(b.x[0].q[3])
                     : "n"(N)
                     : "memory");
    } else if constexpr (K == 2) {
        asm volatile("s_waitcnt vmcnt(%8) ; lampi-wait %0 %1 %2 %3 %4 %5 %6 %7"
                     : "+v"(b.x[0].q[0]), "+v"(b.x[0].q[1]), "+v"(b.x[0].q[2]), "+v"(b.x[0].q[3]),
                       "+v"(b.x[1].q[0]), "+v"(b.x[1].q[1]), "+v"(b.x[1].q[2]), "+v"(b.x[1].q[3])
                     : "n"(N)
                     : "memory");
    } else {
        static_assert(K == 4, "kChains is 1, 2 or 4");
        asm volatile("s_waitcnt vmcnt(%16) ; lampi-wait %0 %1 %2 %3 %4 %5 %6 %7 %8 %9 %10 %11 %12 %13 %14 %15"
                     : "+v"(b.x[0].q[0]), "+v"(b.x[0].q[1]), "+v"(b.x[0].q[2]), "+v"(b.x[0].q[3]),
                       "+v"(b.x[1].q[0]), "+v"(b.x[1].q[1]), "+v"(b.x[1].q[2]), "+v"(b.x[1].q[3]),
                       "+v"(b.x[2].q[0]), "+v"(b.x[2].q[1]), "+v"(b.x[2].q[2]), "+v"(b.x[2].q[3]),
                       "+v"(b.x[3].q[0]), "+v"(b.x[3].q[1]), "+v"(b.x[3].q[2]), "+v"(b.x[3].q[3])
                     : "n"(N)
                     : "memory");
    }
}

// wait_rows with the count chosen at run time (sel, SGPR: 0 -> A, 1 -> B, else C) in one asm
// statement (see LAMPI_WAIT_SEL_ASM)
template <int A, int B, int C, int K>
__device__ __forceinline__ void wait_rows_sel(uint32_t sel, RowsK<K> &b) {
    if constexpr (K == 1) {
        asm volatile(LAMPI_WAIT_SEL_ASM("%0 %1 %2 %3")
                     : "+v"(b.x[0].q[0]), "+v"(b.x[0].q[1]), "+v"(b.x[0].q[2]), "+v"(b.x[0].q[3])
                     : [sel] "s"(sel), [a] "n"(A), [b] "n"(B), [c] "n"(C)
                     : "scc", "memory");
    } else if constexpr (K == 2) {
        asm volatile(LAMPI_WAIT_SEL_ASM("%0 %1 %2 %3 %4 %5 %6 %7")
                     : "+v"(b.x[0].q[0]), "+v"(b.x[0].q[1]), "+v"(b.x[0].q[2]), "+v"(b.x[0].q[3]),
                       "+v"(b.x[1].q[0]), "+v"(b.x[1].q[1]), "+v"(b.x[1].q[2]), "+v"(b.x[1].q[3])
                     : [sel] "s"(sel), [a] "n"(A), [b] "n"(B), [c] "n"(C)
                     : "scc", "memory");
    } else {
        static_assert(K == 4, "kChains is 1, 2 or 4");
        asm volatile(LAMPI_WAIT_SEL_ASM("%0 %1 %2 %3 %4 %5 %6 %7 %8 %9 %10 %11 %12 %13 %14 %15")
                     : "+v"(b.x[0].q[0]), "+v"(b.x[0].q[1]), "+v"(b.x[0].q[2]), "+v"(b.x[0].q[3]),
                       "+v"(b.x[1].q[0]), "+v"(b.x[1].q[1]), "+v"(b.x[1].q[2]), "+v"(b.x[1].q[3]),
                       "+v"(b.x[2].q[0]), "+v"(b.x[2].q[1]), "+v"(b.x[2].q[2]), "+v"(b.x[2].q[3]),
                       "+v"(b.x[3].q[0]), "+v"(b.x[3].q[1]), "+v"(b.x[3].q[2]), "+v"(b.x[3].q[3])
                     : [sel] "s"(sel), [a] "n"(A), [b] "n"(B), [c] "n"(C)
                     : "scc", "memory");
    }
}

__device__ __forceinline__ uint32_t row_word(const Row &r, int w) {
    const u32x4 v = r.q[w >> 2];
    return (w & 3) == 0 ? v.x : (w & 3) == 1 ? v.y : (w & 3) == 2 ? v.z : v.w;
}

// K registers through their 16-word pieces, chains interleaved
template <int K>
__device__ __forceinline__ void crc_pieces(const uint32_t *lds, const CrcLane &k, uint32_t (&C)[K],
                                           const RowsK<K> &b) {
    uint32_t X[K];
#pragma unroll
    for (int c = 0; c < K; ++c) X[c] = C[c] ^ row_word(b.x[c], 0);
#pragma unroll
    for (int w = 0; w < 15; ++w) {
        Look4 t[K];
#pragma unroll
        for (int c = 0; c < K; ++c) t[c] = look4(lds, k, X[c]);
#pragma unroll
        for (int c = 0; c < K; ++c) X[c] = xor3(xor3(t[c].t0, t[c].t1, t[c].t2), t[c].t3, row_word(b.x[c], w + 1));
    }
    Look4 t[K];
#pragma unroll
    for (int c = 0; c < K; ++c) t[c] = look4(lds, k, X[c]);
#pragma unroll
    for (int c = 0; c < K; ++c) C[c] = xor3(t[c].t0, t[c].t1, t[c].t2) ^ t[c].t3;
}

// Coalesced layout (fused copy): lane l holds the 16-byte chunks at 16l + 1024q of a row.
// Every chunk but the fragment's first is preceded by a 1008-byte Horner shift (the same step
// inside a row and across rows); the final per-lane shift is 16*(63-l).
template <int K>
__device__ __forceinline__ void crc_chunks(const uint32_t *lds, const CrcLane &k, uint32_t (&C)[K],
                                           const RowsK<K> &b, bool start, uint32_t init) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (start && q == 0) {
#pragma unroll
            for (int c = 0; c < K; ++c) C[c] = init;
        } else {
#pragma unroll
            for (int c = 0; c < K; ++c) C[c] = horner_shift(lds, C[c]);
        }
        uint32_t X[K];
#pragma unroll
        for (int c = 0; c < K; ++c) X[c] = C[c] ^ b.x[c].q[q].x;
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            Look4 t[K];
#pragma unroll
            for (int c = 0; c < K; ++c) t[c] = look4(lds, k, X[c]);
#pragma unroll
            for (int c = 0; c < K; ++c) {
                const uint32_t d = w == 1 ? b.x[c].q[q].y : w == 2 ? b.x[c].q[q].z : b.x[c].q[q].w;
                X[c] = xor3(xor3(t[c].t0, t[c].t1, t[c].t2), t[c].t3, d);
            }
        }
        Look4 t[K];
#pragma unroll
        for (int c = 0; c < K; ++c) t[c] = look4(lds, k, X[c]);
#pragma unroll
        for (int c = 0; c < K; ++c) C[c] = xor3(t[c].t0, t[c].t1, t[c].t2) ^ t[c].t3;
    }
}

// (Round 1's ablated variants -- loads only, lookups only -- ran as a template switch here until
// commit d95cfff: profiles/r01_ablation.txt.)
// kCopy: fused bcopy -- each row is also stored to dst + f*dst_stride (dst and dst_stride 4-byte
// aligned: asm global_store_dwordx4 at dword-aligned addresses, launch_msg_bcopy's gate) as soon
// as it arrives; per step the ring then carries 4K stores beside 4K loads, and the waits count
// them (first pass: 8K / 12K / 16K younger operations, then 16K).  Rows move in the coalesced
// layout (crc_chunks): lane-contiguous 64-byte stores run at 51% of the HBM roofline on
// MI355X against 71% for 1 KiB-per-instruction stores (profiles/r01_copy_patterns.txt).
// kV > 1 (read-only): every row is a whole 4 KiB fragment and rows are visited in the order of a
// kV*4096-byte fragment (launch with frag_len = kV*4096, n = fragments / kV): chain c of a wave
// reads kV consecutive fragments one after the other instead of one.
// kSum: the same schedule computes uicsum instead (no tables; the LDS stays allocated so the
// kernel keeps the two-workgroups-per-CU occupancy the schedule was measured at: without it, five
// workgroups per CU, config B SUM 78.7-80.4 -> 79.4-79.5%, with half the fragments per wave too
// 79.6-79.7%, 16 KiB fragments 79.1-79.2 -> 78.5%; profiles/r02_sum_regular/).
// kWv: waves per workgroup (the table builders use the first 256 threads); kCap > 0 asks the
// compiler for that many waves per SIMD.
// kDesc (read-only CRC; round 5): a descriptor batch of equal whole-row fragments on this schedule --
// `base` is the lampi_frag_desc array, each fragment with its own address and register.  kV = 2: 4 KiB
// fragments in pairs (n = pairs, lane 2j + r holds fragment 2 (f0 + kWv j) + r); kV = 1: fragments of
// R = frag_len / 4096 rows (n = fragments, lane j holds fragment f0 + kWv j).  A wave loads its
// descriptors into lanes (one vector load before the ring), takes each row's address and register by
// readlane, and checks every fragment: a pair (kV = 2) or fragment (kV = 1) that is not exactly
// frag_len / kV bytes at a 16-byte-aligned address is read at a dummy address (the table image: the
// ring's load counts stay fixed), not emitted, and listed (atomicAdd on *left) for
// crc_light_pair_leftover_kernel, which checksums fragments 2e and 2e + 1 of entry e on the table-light
// kernel (kV = 1 lists f / 2: its neighbour is checksummed again, to the same value).
// kSub < 64 (packed rows, round 6; messages of 64 * kSub-byte fragments, kSub = 1 .. 32): every 4 KiB row holds
// 64 / kSub whole fragments, lane l the 64-byte piece l % kSub of fragment l / kSub of the row.  The row's
// bytes and lookups are config B's; only the ends change: the register enters at every group's first lane,
// lane l shifts by 64 (kSub - 1 - l % kSub) bytes through the combine column of lane 64 - kSub + l % kSub
// (none for kSub = 1), the group's values meet by DPP (group_reduce) and the group's last lane stores
// out[row * 64 / kSub + l / kSub].  Launched with kV = 2 (every row a fragment end); read-only.
template <int kChains, bool kCopy = false, bool kCoal = kCopy, int kDepth = 3, int kV = 1,
          bool kSum = false, int kWv = kWaves, int kCap = 0, bool kDesc = false, int kSub = 64, bool kDiag = false>
__global__ void __launch_bounds__(64 * kWv) __attribute__((amdgpu_waves_per_eu(kCap > 0 ? kCap : 1)))
crc_regular_kernel(const uint8_t *__restrict__ base, uint32_t n, uint32_t fpw, size_t frag_len, uint32_t partial,
                   const uint32_t *__restrict__ img, uint32_t *__restrict__ out, uint8_t *__restrict__ dst,
                   size_t dst_stride, uint32_t *__restrict__ list = nullptr, uint32_t *left = nullptr) {
    constexpr int K = kChains;
    static_assert(kWv >= kWaves, "the table builders need 256 threads");
    static_assert(!kDesc || (kV <= 2 && !kCopy && !kSum), "descriptor batches: read-only CRC, kV = 1 or 2");
    static_assert(kSub == 64 || (kV == 2 && !kCopy && !kCoal && !kDesc), "packed rows: read-only, kV = 2");
    constexpr int kS = kCoal ? kRowBytes / 4 : 16;  // chunk stride of a lane
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
    const int lane = threadIdx.x & 63;
    if constexpr (kDiag) {  // timeline diagnostic (diag_regular_timeline): [0] entry, [8] HW_ID, [9] XCC_ID
        if (threadIdx.x == 0) {
            g_stream_diag[(size_t)blockIdx.x * 16] = __builtin_amdgcn_s_memrealtime();
            g_stream_diag[(size_t)blockIdx.x * 16 + 8] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (31 << 11));
            g_stream_diag[(size_t)blockIdx.x * 16 + 9] = (uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (31 << 11));
        }
    }
    const uint32_t R = (uint32_t)(frag_len / kRowBytes);
    const uint32_t f0 = uniform(blockIdx.x * kWv * fpw + (threadIdx.x >> 6));
    // fragments of this wave: f0 + kWv*j, j < nfr; processed in groups of K
    const uint32_t nfr = f0 < n ? min(fpw, (n - f0 + kWv - 1) / kWv) : 0u;
    const uint32_t ngrp = (nfr + K - 1) / K;
    const uint32_t lane_off = (uint32_t)lane * (kCoal ? kChunkBytes : kLaneBytes);
    uint32_t vinit = __builtin_bswap32(partial);
    // packed rows over a descriptor batch (read-only CRC; dst = the lampi_frag_desc array, base unused): a batch the
    // census saw as one contiguous run of equal fragments (fragment i = d[0].addr + i * L, L = 64 kSub, d[0]'s
    // register) runs as that message.  Each wave first checks the descriptors of its items (F = 128 / kSub
    // fragments each, one 16-byte load per lane and item, clamped so every load is issued): an item holding any
    // other fragment is read at a dummy address (the table image), not emitted, and its F / 2 fragment pairs are
    // listed for crc_light_pair_leftover_kernel -- no address outside the batch's own fragments is read.
    uint64_t pbad = 0u;
    const uint8_t *pbase = base;
    if constexpr (kSub < 64) {
        if (dst != nullptr) {  // (SUM: the register is ignored; the pairs go to sum_pair_leftover_kernel)
            const lampi_frag_desc *pd = reinterpret_cast<const lampi_frag_desc *>(dst);
            const uint64_t a0 = uniform64(pd[0].addr);
            const uint32_t p0 = uniform(pd[0].partial);
            constexpr uint32_t L = 64u * kSub, F = 128u / kSub, kPer = F > 64 ? 2 : 1;
            pbase = reinterpret_cast<const uint8_t *>(a0);
            vinit = __builtin_bswap32(p0);
            constexpr uint32_t kBatch = kPer == 2 ? 6u : 12u;  // items checked per round (12 x 4 VGPRs in flight)
            for (uint32_t j0 = 0; j0 < nfr; j0 += kBatch) {
                lampi_frag_desc x[kBatch][kPer];
#pragma unroll
                for (uint32_t jj = 0; jj < kBatch; ++jj)
#pragma unroll
                    for (uint32_t h = 0; h < kPer; ++h) {
                        const uint32_t j = min(j0 + jj, nfr - 1u), k = min(lane + 64u * h, F - 1u);
                        x[jj][h] = pd[(size_t)(f0 + kWv * j) * F + k];
                    }
#pragma unroll
                for (uint32_t jj = 0; jj < kBatch; ++jj) {
                    const uint32_t j = j0 + jj;
                    bool bad = false;
#pragma unroll
                    for (uint32_t h = 0; h < kPer; ++h) {
                        const uint64_t fi = (uint64_t)(f0 + kWv * min(j, nfr - 1u)) * F + min(lane + 64u * h, F - 1u);
                        bad |= x[jj][h].addr != a0 + fi * L || x[jj][h].length != L || (!kSum && x[jj][h].partial != p0);
                    }
                    if (j < nfr && __ballot(bad)) pbad |= 1ull << j;
                }
            }
            pbad = uniform64(pbad);
            for (uint64_t m = pbad; m; m &= m - 1) {  // list the item's fragment pairs
                const uint32_t item = f0 + kWv * (uint32_t)__builtin_ctzll(m);
                uint32_t e0 = 0u;
                if (lane == 0) e0 = atomicAdd(left, F / 2u);
                e0 = uniform(e0);
                if (lane < F / 2u) list[e0 + lane] = item * (F / 2u) + lane;
            }
        }
    }
    // kDesc: lane kV j + r holds fragment kV (f0 + kWv j) + r's descriptor; bad bit j: item j is listed
    // The descriptors are loaded here and checked (desc_check) after the slicing tables are built, so their
    // latency hides behind that build instead of delaying the workgroup's first rows.
    uint32_t da_lo = 0u, da_hi = 0u, dpart = 0u;
    uint64_t bad = 0u;
    lampi_frag_desc dx{};
    if constexpr (kDesc) {
        if (nfr) {  // every lane loads (clamped to the wave's last item)
            const lampi_frag_desc *descs = reinterpret_cast<const lampi_frag_desc *>(base);
            const uint32_t j = min((uint32_t)lane / kV, nfr - 1u);
            dx = descs[(size_t)(f0 + kWv * j) * kV + (kV == 2 ? (lane & 1) : 0)];
        }
    }
    auto desc_check = [&] {
      if constexpr (kDesc) {
        const uint32_t j = (uint32_t)lane / kV;
        const bool mine = j < nfr;
        uint32_t len = 0u;
        if (mine) {
            da_lo = (uint32_t)dx.addr;
            da_hi = (uint32_t)(dx.addr >> 32);
            len = dx.length;
            dpart = dx.partial;
        }
        const bool odd = mine && (len != (uint32_t)(frag_len / kV) || (da_lo & 15u) != 0u);
        const uint64_t lanes = __ballot(odd);
        if constexpr (kV == 2) {
            for (uint32_t q = 0; q < 32u; ++q) bad |= ((lanes >> (2u * q)) & 3ull) ? (1ull << q) : 0ull;
        } else {
            bad = lanes;
        }
        bad = uniform64(bad);
        if (bad && lane == 0) {
            for (uint64_t m = bad; m; m &= m - 1) {
                const uint32_t f = f0 + kWv * (uint32_t)__builtin_ctzll(m);
                list[atomicAdd(left, 1u)] = kV == 2 ? f : f >> 1;
            }
        }
      }
    };

    auto advance = [&](GroupTask t) -> GroupTask {
        if (t.r + 1 < R) return {t.i, t.r + 1};
        if (t.i + 1 < ngrp) return {t.i + 1, 0u};
        return t;
    };
    auto is_last = [&](const GroupTask &t) -> bool { return t.i + 1 >= ngrp && t.r + 1 >= R; };
    // fragment of slot s in group i; missing fragments (past nfr) re-read slot 0 (no output)
    auto frag = [&](uint32_t i, uint32_t s) -> uint32_t {
        const uint32_t j = K * i + s;
        return f0 + kWv * (j < nfr ? j : K * i);
    };
    auto row_ptr = [&](uint32_t f, uint32_t r) -> gbyte * {
        if constexpr (kDesc) {  // f = f0 + kWv j; kV = 2: row r is fragment 2f + r (lane 2j + r), kV = 1: lane j
            const uint32_t j = (f - f0) / kWv, L = kV == 2 ? 2u * j + r : j;
            // (readlane returns int: each half goes through uint32_t, or a low word >= 2^31 sign-extends
            // into the high one -- the illegal address of this path's first GPU run)
            const uint64_t a = (nfr && !((bad >> j) & 1u))
                                   ? ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(da_hi, L) << 32) |
                                         (uint64_t)(uint32_t)__builtin_amdgcn_readlane(da_lo, L)
                                   : (uint64_t)(uintptr_t)img;
            const uint64_t ro = kV == 2 || !(nfr && !((bad >> j) & 1u)) ? 0u : (uint64_t)r * kRowBytes;
            return (gbyte *)(a + ro + lane_off);
        }
        if constexpr (kSub < 64) {
            if (pbad >> ((f - f0) / kWv) & 1u) return (gbyte *)((const uint8_t *)img + lane_off);
        }
        return (gbyte *)(pbase + ((uint64_t)(nfr ? f : 0u) * frag_len + (uint64_t)r * kRowBytes + lane_off));
    };
    auto issue = [&](const GroupTask &t, RowsK<K> &b) {
#pragma unroll
        for (int c = 0; c < K; ++c) {
            issue_row<kS>(row_ptr(frag(t.i, c), t.r), b.x[c]);
        }
    };

    constexpr int D = kDepth;  // ring slots: D - 1 steps in flight while one is checksummed
    static_assert(D >= 2 && D <= 6, "ring depth");
    GroupTask t[D];
    RowsK<K> ring[D];
    t[0] = GroupTask{0u, 0u};
#pragma unroll
    for (int q = 1; q < D; ++q) t[q] = advance(t[q - 1]);
    auto issue_all = [&] {
#pragma unroll
        for (int q = 0; q < D; ++q) issue(t[q], ring[q]);
    };
    if constexpr (kSum) {
        issue_all();
        asm volatile("" ::"v"(lds) : "memory");  // the LDS array escapes: it stays allocated
    } else if (kWv == kWaves) {
        // every ring slot is in flight while the workgroup builds its tables
        if constexpr (kDesc) {
            auto checked_issue = [&] {
                desc_check();
                issue_all();
            };
            stage_tables<4 * K * D, decltype(checked_issue), 7, kCoal, true, true>(lds, img, checked_issue);
        } else {
            stage_tables<4 * K * D, decltype(issue_all), 7, kCoal>(lds, img, issue_all);
        }
    } else {
        desc_check();
        if (threadIdx.x < 64 * kWaves)
            stage_tables<4 * K * D, decltype(issue_all), 7, kCoal, false>(lds, img, issue_all);
        else
            issue_all();
        lds_barrier();
    }
    if constexpr (kDiag) {  // [1] tables staged
        if (threadIdx.x == 0) g_stream_diag[(size_t)blockIdx.x * 16 + 1] = __builtin_amdgcn_s_memrealtime();
    }
    if (nfr == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }
    const CrcLane k = make_lane(lane);
    // packed rows: the combine column of lane 64 - kSub + l % kSub (a shift by 64 (kSub - 1 - l % kSub) bytes)
    CrcLane ksub = k;
    if constexpr (kSub < 64) ksub.comb_base = make_lane(64 - kSub + (lane & (kSub - 1))).comb_base;
    uint32_t C[K];
#pragma unroll
    for (int c = 0; c < K; ++c) C[c] = 0;
    // a fragment's checksum waits in lane j kV + r of `res` (fragment kV (f0 + kWv j) + r) and the wave stores all of
    // them once, after its last row: a store inside the ring is one more operation each later wait counts
    // (CRC only: with kSum the compiler read a ring register before its wait -- tests/test_isa_guard.py)
    const bool late = !kSum && nfr * (uint32_t)kV <= 64u;
    uint32_t res = 0u;
    auto emit = [&](uint32_t j, uint32_t r, uint32_t v) {  // item j (K i + c) of this wave, row r (kV > 1)
        if (late) {
            res = (uint32_t)lane == j * kV + (kV > 1 ? r : 0u) ? v : res;
        } else if (lane == 0) {
            out[kV > 1 ? (f0 + kWv * j) * kV + r : f0 + kWv * j] = v;
        }
    };
    auto process = [&](RowsK<K> &b, const GroupTask &t) {
        if constexpr (kCopy) {
#pragma unroll
            for (int c = 0; c < K; ++c)
                if (K * t.i + c < nfr)
                    store_row<kS>(
                        (gwbyte *)(dst + (uint64_t)frag(t.i, c) * dst_stride + (uint64_t)t.r * kRowBytes + lane_off),
                        b.x[c]);
        }
        if constexpr (kSum) {  // uicsum: 32-bit LE words of the fragment, summed mod 2^32
#pragma unroll
            for (int c = 0; c < K; ++c) {
                uint32_t y = (kV > 1 || t.r == 0) ? 0u : C[c];
#pragma unroll
                for (int w = 0; w < 16; ++w) y += row_word(b.x[c], w);
                C[c] = y;
            }
            if constexpr (kSub < 64) {  // packed rows: every group of kSub lanes is a fragment
                uint32_t x[K];
#pragma unroll
                for (int c = 0; c < K; ++c) x[c] = group_reduce<kSub, true>(C[c]);
                if ((lane & (kSub - 1)) == kSub - 1) {
#pragma unroll
                    for (int c = 0; c < K; ++c)
                        if (K * t.i + c < nfr && !((pbad >> (K * t.i + c)) & 1u))
                            out[(frag(t.i, c) * kV + t.r) * (64u / kSub) + lane / kSub] = x[c];
                }
                return;
            }
            if (kV > 1 || t.r + 1 == R) {
                uint32_t x[K];
#pragma unroll
                for (int c = 0; c < K; ++c) x[c] = wave_add(C[c]);
#pragma unroll
                for (int c = 0; c < K; ++c)
                    if (K * t.i + c < nfr) emit(K * t.i + c, t.r, x[c]);
            }
            return;
        }
        if constexpr (kCoal) {
            crc_chunks<K>(lds, k, C, b, t.r == 0, (lane == 0) ? vinit : 0u);
        } else {
            if (kDesc && (kV > 1 || t.r == 0)) {  // a fragment's first row: its own register
#pragma unroll
                for (int c = 0; c < K; ++c) {
                    const uint32_t j = (frag(t.i, c) - f0) / kWv, L = kV == 2 ? 2u * j + t.r : j;
                    const uint32_t v = __builtin_bswap32((uint32_t)__builtin_amdgcn_readlane(dpart, L));
                    C[c] = (lane == 0) ? v : 0u;
                }
            } else if (kV > 1 || t.r == 0) {
#pragma unroll
                for (int c = 0; c < K; ++c) C[c] = (lane & (kSub - 1)) == 0 ? vinit : 0u;
            } else {
#pragma unroll
                for (int c = 0; c < K; ++c) C[c] = horner_shift(lds, C[c]);
            }
            crc_pieces<K>(lds, k, C, b);
        }
        if constexpr (kSub < 64) {  // packed rows: lane l to its fragment's end, the group's XOR, its last lane stores
            uint32_t x[K];
#pragma unroll
            for (int c = 0; c < K; ++c) x[c] = kSub > 1 ? lane_combine(lds, ksub, C[c]) : C[c];
#pragma unroll
            for (int c = 0; c < K; ++c) x[c] = group_reduce<kSub, false>(x[c]);
            if ((lane & (kSub - 1)) == kSub - 1) {
#pragma unroll
                for (int c = 0; c < K; ++c)
                    if (K * t.i + c < nfr && !((pbad >> (K * t.i + c)) & 1u))
                        out[(frag(t.i, c) * kV + t.r) * (64u / kSub) + lane / kSub] = __builtin_bswap32(x[c]);
            }
            return;
        }
        if (kV > 1 || t.r + 1 == R) {
            uint32_t x[K];
#pragma unroll
            for (int c = 0; c < K; ++c) x[c] = lane_combine(lds, k, C[c]);
#pragma unroll
            for (int c = 0; c < K; ++c) x[c] = wave_xor(x[c]);
#pragma unroll
            for (int c = 0; c < K; ++c)
                if (K * t.i + c < nfr && !(kDesc && ((bad >> (K * t.i + c)) & 1u)))
                    emit(K * t.i + c, t.r, __builtin_bswap32(x[c]));
        }
    };
    // steady state: slot S is waited for, checksummed (and stored) and refilled with the task
    // after the most recently issued one.  vmcnt counts loads and stores in issue order: the
    // operations younger than slot S's loads are (D-1)*kL loads, plus with kCopy the stores
    // in between -- (D-1+S)*kL on the first pass, 2(D-1)*kL after.
    constexpr int kL = 4 * K;  // loads (and, with kCopy, stores) per step
    bool first = true;
    // a wave whose fragment count is not a multiple of K skips the stores of its missing chain
    // in the last group: fewer younger operations than the counts assume, so those steps drain
    const bool short_tail = kCopy && (nfr % K) != 0;
#define LAMPI_RING_STEP(S)                                                  \
    if constexpr ((S) < D) {                                                \
        if constexpr (kCopy) { /* one asm statement: see wait_rows_sel */  \
            const uint32_t sel_ = uniform((short_tail && t[(S) % D].i + 1 >= ngrp) ? 0u : (first ? 1u : 2u)); \
            wait_rows_sel<0, (D - 1 + (S)) * kL, 2 * (D - 1) * kL, K>(sel_, ring[(S) % D]); \
        } else {                                                            \
            wait_rows<(D - 1) * kL, K>(ring[(S) % D]);                      \
        }                                                                   \
        process(ring[(S) % D], t[(S) % D]);                                 \
        if (is_last(t[(S) % D])) break;                                     \
        t[(S) % D] = advance(t[((S) + D - 1) % D]);                         \
        issue(t[(S) % D], ring[(S) % D]);                                   \
    }
    for (;;) {
        LAMPI_RING_STEP(0)
        LAMPI_RING_STEP(1)
        LAMPI_RING_STEP(2)
        LAMPI_RING_STEP(3)
        LAMPI_RING_STEP(4)
        LAMPI_RING_STEP(5)
        first = false;
    }
#undef LAMPI_RING_STEP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the clamped re-loads before exit
    if constexpr (kSub == 64) {
        const uint32_t j = (uint32_t)lane / kV;
        if (late && j < nfr && !(kDesc && ((bad >> j) & 1u)))
            out[kV > 1 ? (f0 + kWv * j) * kV + (uint32_t)lane % kV : f0 + kWv * j] = res;
    }
    if constexpr (kDiag) {  // [2 + w] wave w done
        if (lane == 0) g_stream_diag[(size_t)blockIdx.x * 16 + 2 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime();
    }
}

// ---- SUM -------------------------------------------------------------------------------
// SUM fused copies (bcopy_uicsum descriptors, the receive step, ragged message fragments and the
// rows of longer ones) in the textbook copy shape: one short-lived 128-thread workgroup per
// fragment, thread t the 16-byte chunk at 16t of each 2 KiB row (unaligned loads and stores, any
// alignment: the memory pipeline splits them at line boundaries; 1 KiB per wave-instruction both
// ways), non-temporal stores, the next row loaded before this one is stored.  The sum is
// order-free and every chunk starts on the fragment's word grid.  Copy shape: 4 KiB rows 78-81% of
// read + write against 72-74% for one fragment per wave (tools/microbench/copy5.hip).
typedef __attribute__((address_space(1))) const uint32_t __attribute__((aligned(1))) gu32_a1;
typedef __attribute__((address_space(1))) uint32_t __attribute__((aligned(1))) gwu32_a1;

// The last 1-15 bytes of a fragment (chunk at o, n < 16 bytes): whole words by unaligned dword
// loads, the last 1-3 bytes one by one, zero-padded (the reference's partial last word).
__device__ __forceinline__ u32x4 load_tail16(gbyte *p, uint32_t n) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t b = 4u * k;
        w[k] = 0u;
        if (b + 4u <= n) {
            w[k] = *(gu32_a1 *)(p + b);
        } else if (b < n) {
            for (uint32_t c = b; c < n; ++c) w[k] |= (uint32_t)p[c] << (8u * (c - b));
        }
    }
    return u32x4{w[0], w[1], w[2], w[3]};
}

// the first n < 16 bytes of a chunk: whole words by (unaligned) dword stores, then bytes
__device__ __forceinline__ void store_head16(gwbyte *q, const u32x4 &v, uint32_t n) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t b = 4u * k;
        if (b + 4u <= n) {
            *(gwu32_a1 *)(q + b) = w[k];
        } else if (b < n) {
            for (uint32_t c = b; c < n; ++c) q[c] = (uint8_t)(w[k] >> (8u * (c - b)));
        }
    }
}

// Threads per workgroup (one fragment each), same-box A/B (profiles/r02_sumcopy/ab_wgT/, ab_row/):
// 128 against 256: 4 KiB descriptors 74.4 -> 79.1-79.2%, +8 sources 74 -> 79.6%, the receive step
// 72 -> 75-77%, fragments of 64 B-2 KiB 1.5-2x faster (1 GiB of 1,976-byte fragments 0.80 ->
// 0.53 ms, now ahead of sum_rows_kernel's 0.61 at every size), 16 KiB / 65,456-byte descriptors
// 71.5 / 61.4 -> 69.9 / 58.1%; 64 threads: small fragments faster still (64 B 3.4x) but +8 and +1
// destinations 66%; 192: 75.7%.  The row kernel keeps 256 (128 / 64: GM slots 75 -> 71 / 64%).
constexpr int kSumWgThreads = 128;

// One fragment's copy and partial sum on kT threads (thread t of them): returns the thread's sum.
template <int kT, class Src>
__device__ __forceinline__ uint32_t sum_copy_frag(const FragInfo &fi, uint32_t t) {
    gbyte *p = (gbyte *)uniform64((uint64_t)(uintptr_t)fi.addr);
    gwbyte *q = (gwbyte *)uniform64((uint64_t)(uintptr_t)fi.dst);
    const uint32_t len = uniform(fi.len), clen = uniform(fi.copylen);  // clen <= len
    const uint32_t nfull = len / 16u, cfull = clen / 16u;  // whole 16-byte chunks
    const uint32_t R = (nfull + kT - 1) / kT;
    // the loop moves whole chunks only (chunk c = kT r + t); the chunk the copy ends inside is kept (vc) and
    // the fragment's partial last chunk is read after the loop
    uint32_t acc = 0;
    u32x4 v = {0u, 0u, 0u, 0u}, vc = {0u, 0u, 0u, 0u};
    if (t < nfull) v = ld16u((gu32x4_a1 *)(p + 16u * t));
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t c = kT * r + t;
        u32x4 nv = {0u, 0u, 0u, 0u};
        if (c + kT < nfull) nv = ld16u((gu32x4_a1 *)(p + 16u * (c + kT)));
        if constexpr (Src::kCopy) {
            if (c < cfull)
                st16u((gwu32x4_a1 *)(q + 16u * c), v);
            else if (c == cfull)
                vc = v;
        }
        acc += v.x + v.y + v.z + v.w;
        v = nv;
    }
    if ((len & 15u) && t == nfull % kT) {  // the fragment's last 1-15 bytes
        const u32x4 w = load_tail16(p + 16u * nfull, len & 15u);
        acc += w.x + w.y + w.z + w.w;
        if (cfull == nfull) vc = w;
    }
    if constexpr (Src::kCopy)
        if ((clen & 15u) && t == cfull % kT) store_head16(q + 16u * cfull, vc, clen & 15u);
    return acc;
}

// SUM messages of fragments of L = 64 .. 1024 bytes (a power of two; round 6): one short-lived 128-thread workgroup
// per 4 KiB of the message, thread t the 16-byte chunks at 16 t and 2048 + 16 t, non-temporal -- config B SUM's shape
// (sum_copy_wg_kernel) over 4096 / L fragments at once.  A fragment's chunks sit in kG = L / 16 consecutive lanes of
// one wave: summed by DPP (group_reduce; a whole wave for 1 KiB), the group's last lane stores.  Whole words only:
// every chunk is on its fragment's word grid (L is a multiple of 16).
template <int kG>
__global__ void __launch_bounds__(128) sum_row4k_kernel(const uint8_t *__restrict__ base, uint32_t *__restrict__ out) {
    constexpr uint32_t L = 16u * kG, F = (uint32_t)kRowBytes / L;  // fragment bytes, fragments per 4 KiB
    static_assert(kG >= 4 && kG <= 64 && (kG & (kG - 1)) == 0, "64 B .. 1 KiB fragments");
    const uint32_t t = threadIdx.x;
    gbyte *p = (gbyte *)(base + (size_t)blockIdx.x * kRowBytes + 16u * t);
    const u32x4 a = ld16u((gu32x4_a1 *)p), b = ld16u((gu32x4_a1 *)(p + kRowBytes / 2));
    uint32_t s0 = a.x + a.y + a.z + a.w, s1 = b.x + b.y + b.z + b.w;
    if constexpr (kG == 64) {
        s0 = wave_add(s0);
        s1 = wave_add(s1);
    } else {
        s0 = group_reduce<kG, true>(s0);
        s1 = group_reduce<kG, true>(s1);
    }
    if ((t & (kG - 1u)) == kG - 1u) {
        const size_t f = (size_t)blockIdx.x * F + (16u * t) / L;
        out[f] = s0;
        out[f + F / 2] = s1;
    }
}

// The same over a descriptor batch of equal L-byte fragments (round 6): workgroup b takes fragments b F .. b F + F - 1
// (F = 4096 / L), each thread loading the descriptors of its two chunks' fragments first and reading its chunks at their
// own addresses -- a fragment of another length is read as zeros (the table image's zero chunk), not emitted, and its
// pair listed for sum_pair_leftover_kernel (the pair counters), so nothing outside the batch's fragments is read.
template <int kG>
__global__ void __launch_bounds__(128) sum_row4k_desc_kernel(const lampi_frag_desc *__restrict__ d,
                                                             const uint32_t *__restrict__ img, uint32_t *__restrict__ out,
                                                             uint32_t *__restrict__ list, uint32_t *left) {
    constexpr uint32_t L = 16u * kG, F = (uint32_t)kRowBytes / L;
    static_assert(kG >= 4 && kG <= 64 && (kG & (kG - 1)) == 0, "64 B .. 1 KiB fragments");
    const uint32_t t = threadIdx.x, j0 = (16u * t) / L, o = 16u * t - j0 * L;  // chunk 0: fragment j0, offset o
    const size_t f0 = (size_t)blockIdx.x * F;
    const lampi_frag_desc x0 = d[f0 + j0], x1 = d[f0 + j0 + F / 2];
    const bool ok0 = x0.length == L, ok1 = x1.length == L;
    gbyte *zero = (gbyte *)(img + kImgZero);
    const u32x4 a = ld16u((gu32x4_a1 *)(ok0 ? (gbyte *)(uintptr_t)x0.addr + o : zero));
    const u32x4 b = ld16u((gu32x4_a1 *)(ok1 ? (gbyte *)(uintptr_t)x1.addr + o : zero));
    uint32_t s0 = a.x + a.y + a.z + a.w, s1 = b.x + b.y + b.z + b.w;
    if constexpr (kG == 64) {
        s0 = wave_add(s0);
        s1 = wave_add(s1);
    } else {
        s0 = group_reduce<kG, true>(s0);
        s1 = group_reduce<kG, true>(s1);
    }
    if ((t & (kG - 1u)) == kG - 1u) {
        const size_t fa = f0 + j0, fb = fa + F / 2;
        if (ok0) out[fa] = s0;
        else list[atomicAdd(left, 1u)] = (uint32_t)(fa >> 1);
        if (ok1) out[fb] = s1;
        else list[atomicAdd(left, 1u)] = (uint32_t)(fb >> 1);
    }
}

// The fused copy of such a message (bcopy_uicsum per fragment, lampi_msg_bcopy): the same workgroups, each chunk
// also stored (non-temporal) at dst + f * dst_stride + its offset in fragment f.
template <int kG>
__global__ void __launch_bounds__(128) sum_row4k_copy_kernel(const uint8_t *__restrict__ base, uint8_t *__restrict__ dst,
                                                             size_t dst_stride, uint32_t *__restrict__ out) {
    constexpr uint32_t L = 16u * kG, F = (uint32_t)kRowBytes / L;
    static_assert(kG >= 4 && kG <= 64 && (kG & (kG - 1)) == 0, "64 B .. 1 KiB fragments");
    const uint32_t t = threadIdx.x, j0 = (16u * t) / L, o = 16u * t - j0 * L;
    gbyte *p = (gbyte *)(base + (size_t)blockIdx.x * kRowBytes + 16u * t);
    const u32x4 a = ld16u((gu32x4_a1 *)p), b = ld16u((gu32x4_a1 *)(p + kRowBytes / 2));
    const size_t fa = (size_t)blockIdx.x * F + j0, fb = fa + F / 2;
    st16u((gwu32x4_a1 *)(dst + fa * dst_stride + o), a);
    st16u((gwu32x4_a1 *)(dst + fb * dst_stride + o), b);
    uint32_t s0 = a.x + a.y + a.z + a.w, s1 = b.x + b.y + b.z + b.w;
    if constexpr (kG == 64) {
        s0 = wave_add(s0);
        s1 = wave_add(s1);
    } else {
        s0 = group_reduce<kG, true>(s0);
        s1 = group_reduce<kG, true>(s1);
    }
    if ((t & (kG - 1u)) == kG - 1u) {
        out[fa] = s0;
        out[fb] = s1;
    }
}

// Fused copies of a descriptor batch of equal 64 B .. 1 KiB fragments (lampi_frag_bcopy_batch SUM; the census saw equal
// lengths): the descriptor kernel's workgroups, each chunk read at its fragment's source and stored at its destination;
// a descriptor of another shape (copylen != L or csumlen > L) is left to sum_copy_list_kernel (its index listed).
template <int kG>
__global__ void __launch_bounds__(128) sum_row4k_copy_desc_kernel(const lampi_copy_desc *__restrict__ d,
                                                                  const uint32_t *__restrict__ img,
                                                                  uint32_t *__restrict__ out, uint32_t *__restrict__ list,
                                                                  uint32_t *left) {
    constexpr uint32_t L = 16u * kG, F = (uint32_t)kRowBytes / L;
    static_assert(kG >= 4 && kG <= 64 && (kG & (kG - 1)) == 0, "64 B .. 1 KiB fragments");
    const uint32_t t = threadIdx.x, j0 = (16u * t) / L, o = 16u * t - j0 * L;
    const size_t fa = (size_t)blockIdx.x * F + j0, fb = fa + F / 2;
    const lampi_copy_desc x0 = d[fa], x1 = d[fb];
    const bool ok0 = x0.copylen == L && x0.csumlen <= L, ok1 = x1.copylen == L && x1.csumlen <= L;
    gbyte *zero = (gbyte *)(img + kImgZero);
    const u32x4 a = ld16u((gu32x4_a1 *)(ok0 ? (gbyte *)(uintptr_t)x0.src + o : zero));
    const u32x4 b = ld16u((gu32x4_a1 *)(ok1 ? (gbyte *)(uintptr_t)x1.src + o : zero));
    if (ok0) st16u((gwu32x4_a1 *)((uint8_t *)(uintptr_t)x0.dst + o), a);
    if (ok1) st16u((gwu32x4_a1 *)((uint8_t *)(uintptr_t)x1.dst + o), b);
    uint32_t s0 = a.x + a.y + a.z + a.w, s1 = b.x + b.y + b.z + b.w;
    if constexpr (kG == 64) {
        s0 = wave_add(s0);
        s1 = wave_add(s1);
    } else {
        s0 = group_reduce<kG, true>(s0);
        s1 = group_reduce<kG, true>(s1);
    }
    if ((t & (kG - 1u)) == kG - 1u) {
        if (ok0) out[fa] = s0;
        else list[atomicAdd(left, 1u)] = (uint32_t)fa;
        if (ok1) out[fb] = s1;
        else list[atomicAdd(left, 1u)] = (uint32_t)fb;
    }
}

template <class Src, int kT = kSumWgThreads>
__global__ void __launch_bounds__(kT) sum_copy_wg_kernel(Src src, size_t n, uint32_t *__restrict__ out) {
    static_assert(!Src::kPhase, "word-grid sources only (read-only ones: row groups of read-only SUM batches)");
    constexpr uint32_t kW = kT / 64;
    __shared__ uint32_t part[2][kW];  // by iteration parity: one barrier per fragment
    const uint32_t t = threadIdx.x;
    uint32_t it = 0;
    // a grid has at most 2^32 - 1 threads: beyond kMaxWgGrid fragments a workgroup takes several
    for (size_t f = blockIdx.x; f < n; f += gridDim.x, it ^= 1u) {
        if constexpr (IsGroupRecv<Src>::value)  // (row groups of the receive step: the join gives the verdicts)
            if (t == 0 && f % src.W == 0) zero_verdict_words(src.src, f / src.W);
        const FragInfo fi = src.get(f);
        uint32_t acc = wave_add(sum_copy_frag<kT, Src>(fi, t));
        if constexpr (kW == 1) {
            if (t == 0) emit(src, out, f, acc, fi);
        } else {
            if ((t & 63) == 0) part[it][t >> 6] = acc;
            __syncthreads();
            if (t == 0) {
                uint32_t sm = 0;
#pragma unroll
                for (uint32_t w = 0; w < kW; ++w) sm += part[it][w];
                emit(src, out, f, sm, fi);
            }
        }
    }
}

// The copy descriptors sum_row4k_copy_desc_kernel listed (list[0 .. *left)): one 128-thread workgroup per entry on a
// fixed grid (sum_copy_wg_kernel's fragment walk, any length); zeroes the stream's other counter (the pair counters).
__global__ void __launch_bounds__(128) sum_copy_list_kernel(const lampi_copy_desc *__restrict__ d, const uint32_t *left,
                                                            uint32_t *next_left, const uint32_t *__restrict__ list,
                                                            uint32_t *__restrict__ out) {
    __shared__ uint32_t part[2][2];
    const uint32_t t = threadIdx.x;
    const uint32_t c = __builtin_amdgcn_readfirstlane(__hip_atomic_load(left, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    uint32_t it = 0;
    for (uint32_t e = blockIdx.x; e < c; e += gridDim.x, it ^= 1u) {
        const size_t f = list[e];
        const FragInfo fi = CopySource{d}.get(f);
        const uint32_t acc = wave_add(sum_copy_frag<128, CopySource>(fi, t));
        if ((t & 63u) == 0) part[it][t >> 6] = acc;
        __syncthreads();
        if (t == 0) out[f] = part[it][0] + part[it][1];
    }
    if (blockIdx.x == 0 && t == 0) *next_left = 0u;
}

// Fragments of at most 2 KiB (IB's payloads; the learned batch shape picks it): one fragment per wave, four
// to a workgroup -- one workgroup per 1,976-byte fragment made the grid's dispatch the bound (522K
// workgroups per GiB).  Exact for any length.
template <class Src>
__global__ void __launch_bounds__(256) sum_copy_waves_kernel(Src src, size_t n, uint32_t *__restrict__ out) {
    static_assert(!Src::kPhase, "word-grid sources only");
    const uint32_t lane = threadIdx.x & 63u;
    for (size_t f = (size_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); f < n;
         f += (size_t)gridDim.x * 4) {
        const FragInfo fi = src.get(f);
        const uint32_t acc = wave_add(sum_copy_frag<64, Src>(fi, lane));
        if (lane == 0) emit(src, out, f, acc, fi);
    }
}

// The leftovers of SUM packed rows over descriptors (launch_sum_desc_packed): entry e of the list = fragments 2 list[e]
// and 2 list[e] + 1, one wave per fragment through sum_copy_frag (any length, any alignment); the entry count is the
// pair kernel's counter, the next call's zeroed here (as crc_light_pair_leftover_kernel).
__global__ void __launch_bounds__(256) sum_pair_leftover_kernel(const lampi_frag_desc *__restrict__ d, size_t n,
                                                                uint32_t *__restrict__ out, const uint32_t *left,
                                                                uint32_t *next_left, const uint32_t *__restrict__ list) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t c = __builtin_amdgcn_readfirstlane(__hip_atomic_load(left, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    for (size_t e = (size_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); e < 2 * (size_t)c;
         e += (size_t)gridDim.x * 4) {
        const size_t f = 2 * (size_t)list[e >> 1] + (e & 1u);
        if (f >= n) continue;
        const FragInfo fi = DescSource{d}.get(f);
        const uint32_t acc = wave_add(sum_copy_frag<64, DescSource>(fi, lane));
        if (lane == 0) out[f] = acc;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *next_left = 0u;
}

// SUM row groups: out[f] = the sum of fragment f's W group sums, then emit (receive sources: the verdict).
// G = min(64, pow2 >= W) lanes per fragment, lane j adding groups j, j + G, ... (one thread walking a
// fragment's 4,096 one-row groups waited on 4,096 loads in turn).
template <class Src>
__global__ void __launch_bounds__(256) sum_group_join_kernel(const Src src, size_t n, uint32_t W, uint32_t G,
                                                             const uint32_t *__restrict__ groups,
                                                             uint32_t *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x, f = i / G;
    const uint32_t j = (uint32_t)(i & (G - 1u));
    if (f >= n) return;  // (the G lanes of a fragment leave or stay together)
    const uint32_t *p = groups + f * W;
    uint32_t sm = 0;
    for (uint32_t g = j; g < W; g += G) sm += p[g];
    for (uint32_t o = G >> 1; o >= 1u; o >>= 1) sm += (uint32_t)__shfl_xor((int)sm, (int)o);
    if (j == 0) emit(src, out, f, sm, src.get(f));
}

// Acc = uint32_t: uicsum (32-bit words); Acc = uint64_t: csum (64-bit words, ref
// MemFunctions.cc:142-516, 913-1071).  Phase (kPhase sources) is taken mod the word size.
template <class Src, class Acc = uint32_t, int kWv = kWaves>
__global__ void __launch_bounds__(64 * kWv) sum_rows_kernel(Src src, size_t n, uint32_t fpw, Acc *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    __shared__ __attribute__((aligned(16))) uint32_t stage[Src::kCopy ? kWv * 1024 / 4 : 1];  // per-wave copy staging
    const size_t f0 = uniform(blockIdx.x * kWv * fpw + (threadIdx.x >> 6));
    const size_t fend = f0 + (size_t)kWv * fpw;  // exclusive, stride kWv
    uint32_t *area = stage + (threadIdx.x >> 6) * (1024 / 4);

    // a fragment's frame: `ph` = the byte phase of its first byte in the word grid (chained
    // pieces); the frame starts ph bytes early and those bytes read as zero
    struct Frame {
        FragInfo fi;
        gbyte *fb;
        uint8_t *db;
        uint32_t ph, span, R, s16, dm;
    };
    auto open = [&](size_t x, Frame &t) -> size_t {  // next non-empty fragment (empty ones: 0)
        for (; x < n && x < fend; x += kWv) {
            FragInfo fi = src.get(x);
            fi.addr = (gbyte *)uniform64((uint64_t)(uintptr_t)fi.addr);
            fi.len = uniform(fi.len);
            if constexpr (Src::kCopy) {
                fi.dst = (uint8_t *)uniform64((uint64_t)(uintptr_t)fi.dst);
                fi.copylen = uniform(fi.copylen);
            }
            if (fi.len) {
                t.fi = fi;
                t.ph = Src::kPhase ? (uniform(fi.partial) & (uint32_t)(sizeof(Acc) - 1)) : 0u;
                t.fb = fi.addr - t.ph;
                t.span = fi.len + t.ph;
                t.R = (uint32_t)(((uint64_t)fi.len + t.ph + (kRowBytes - 1)) / kRowBytes);
                t.s16 = (uint32_t)((uintptr_t)t.fb & 15u);
                t.db = fi.dst - t.ph;
                t.dm = (uint32_t)((uintptr_t)t.db & 15u);
                return x;
            }
            if (lane == 0) emit(src, out, x, (Acc)0, fi);
        }
        return n;
    };
    // interior rows load coalesced (16 bytes at 16l + 1024q, one 1 KiB run per instruction,
    // unaligned sources included): every chunk starts on the fragment's word grid and the sum is
    // order-free, so only a copy to a destination that is not dword aligned needs the lane-contiguous
    // pieces (rows_to_pieces).  Edge rows (a phase in front, a partial last row) load lane-contiguous
    // and masked.  Returns whether the row was loaded coalesced.
    auto load = [&](const Frame &t, uint32_t r, uint32_t(&d)[16]) -> bool {
        const bool mask = (r == 0 && t.ph != 0) || (r + 1 == t.R && t.span % kRowBytes != 0);
        if (mask) {
            load64(t.fb, (long long)r * kRowBytes + lane * kLaneBytes, t.ph, (long long)t.span, true, t.s16, d);
            return false;
        }
        gbyte *p = t.fb + (uint64_t)r * kRowBytes + 16 * lane;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32x4 v = *(gu32x4_a1 *)(p + 1024 * q);
            d[4 * q + 0] = v.x;
            d[4 * q + 1] = v.y;
            d[4 * q + 2] = v.z;
            d[4 * q + 3] = v.w;
        }
        return true;
    };

    Frame cur;
    size_t f = open(f0, cur);
    if (f >= n) return;
    uint32_t r = 0;
    uint32_t d[16];
    bool coal = load(cur, 0, d);
    Acc acc = 0;
    uint32_t carry = 0;
    for (;;) {
        // prefetch the next row (of this fragment, or the first of the wave's next one)
        Frame nt = cur;
        size_t nf = f;
        uint32_t nr = r + 1;
        if (nr >= cur.R) {
            nf = open(f + kWv, nt);
            nr = 0;
        }
        const bool more = nf < n;
        uint32_t nd[16];
        bool ncoal = false;
        if (more) ncoal = load(nt, nr, nd);

        if constexpr (Src::kCopy) {
            const FragInfo &fi = cur.fi;
            const long long row0 = (long long)r * kRowBytes, lo = cur.ph, hi = (long long)fi.copylen + cur.ph;
            bool stored = false;
            if (coal && fi.copylen) {
                if (row0 >= lo && row0 + kRowBytes <= hi && (cur.dm & 3u) == 0) {
                    gwbyte *q = (gwbyte *)(cur.db + row0) + 16 * lane;
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        st16((gwu32x4_a4 *)(q + 1024 * c), u32x4{d[4 * c], d[4 * c + 1], d[4 * c + 2], d[4 * c + 3]});
                    stored = true;
                } else {
                    rows_to_pieces(area, d, lane);
                }
            }
            if (fi.copylen && !stored) {
                // whole rows inside the copy: staged 1 KiB-coalesced stores at the dword-aligned
                // db + row0 - m (as in crc_rows_kernel); edge rows: word/byte stores
                const long long o = row0 + lane * kLaneBytes;
                const uint32_t m = cur.dm & 3u;
                if (r == 0) carry = 0;
                const uint32_t prev = m ? prev_lane_top(d[15], carry, lane) : 0u;
                if (row0 >= lo && row0 + kRowBytes <= hi) {
                    if (m == 0) {
                        store_row_coalesced<1024>(area, cur.db + row0, d, lane);
                    } else {
                        const uint32_t sh = 4u - m;
                        uint32_t v[16];
                        v[0] = __builtin_amdgcn_alignbyte(d[0], prev, sh);
#pragma unroll
                        for (int w = 1; w < 16; ++w) v[w] = __builtin_amdgcn_alignbyte(d[w], d[w - 1], sh);
                        const bool skip0 = row0 < lo + 4;
                        store_row_coalesced<1024>(area, cur.db + row0 - m, v, lane, skip0);
                        if (skip0 && lane == 0) store_word(cur.db, row0 - (long long)m, v[0], lo, hi);
                        if (lane == 63 && r + 1 == cur.R)
                            store_word(cur.db, row0 - (long long)m + kRowBytes, __builtin_amdgcn_alignbyte(0u, d[15], sh),
                                       lo, hi);
                    }
                } else if (m == 0) {
                    store_row_coalesced_masked(area, cur.db, row0, d, lane, lo, hi);
                } else {
                    store64(cur.db, o, d, cur.ph, hi, m, false, prev, lane == 63 && r + 1 == cur.R);
                }
                carry = __builtin_amdgcn_readlane(d[15], 63);
            }
        }
        if constexpr (sizeof(Acc) == 4) {
#pragma unroll
            for (int w = 0; w < 16; ++w) acc += d[w];
        } else {  // 64-bit words: the frame is 8-byte aligned to the fragment's word grid
#pragma unroll
            for (int w = 0; w < 16; w += 2) acc += (uint64_t)d[w] | ((uint64_t)d[w + 1] << 32);
        }
        if (r + 1 == cur.R) {
            if constexpr (sizeof(Acc) == 4) {
                acc = wave_add(acc);
            } else {
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
            }
            if (lane == 0) emit(src, out, f, acc, cur.fi);
            acc = 0;
        }
        if (!more) break;
#pragma unroll
        for (int w = 0; w < 16; ++w) d[w] = nd[w];
        coal = ncoal;
        cur = nt;
        f = nf;
        r = nr;
    }
}

// SUM fused copy (bcopy_uicsum) of messages whose fragments are >= 4 KiB and a multiple of 16
// bytes long, from a 16-byte-aligned base to dword-aligned destinations: the textbook copy shape --
// one short-lived 256-thread workgroup per 4 KiB row, one 16-byte chunk per thread, non-temporal
// stores -- which copies at 78-81% of read + write against 72-74% for one fragment per wave
// (tools/microbench/copy5.hip, profiles/r02_copy5.txt); 1-2 points above sum_copy_wg_kernel on the
// same rows (profiles/r02_ab_recv/).  The row's sum goes to out[f] (a one-row fragment) or is
// added atomically into out[f], zeroed beforehand (the sum is order-free and a row starts on the
// fragment's word grid).  Fragment f spans [f*frag_len, min(.., msg_len)); a workgroup takes rows
// blockIdx.x + k*gridDim.x (one, unless there are more than kMaxWgGrid).
constexpr int kSumRowThreads = 256;
template <int kT = kSumRowThreads>
__global__ void __launch_bounds__(kT) sum_copy_row_kernel(const uint8_t *__restrict__ base, size_t msg_len,
                                                          size_t frag_len, uint32_t rpf, uint32_t nrows,
                                                          uint32_t *__restrict__ out, uint8_t *__restrict__ dst,
                                                          size_t dst_stride) {
    constexpr int kS = kRowBytes / 16 / kT;  // chunks per thread per row
    constexpr uint32_t kW = kT / 64;
    __shared__ uint32_t part[2][kW];  // by iteration parity: one barrier per row
    uint32_t it = 0;
    for (uint32_t i = blockIdx.x; i < nrows; i += gridDim.x, it ^= 1u) {
        const uint32_t f = uniform(i / rpf), r = uniform(i - f * rpf);
        const uint64_t fo = (uint64_t)f * frag_len;
        const uint64_t flen = msg_len - fo < frag_len ? msg_len - fo : frag_len;
        u32x4 v[kS];
#pragma unroll
        for (int k = 0; k < kS; ++k) {  // flen % 16 == 0: a chunk is wholly inside or wholly outside
            const uint64_t o = (uint64_t)r * kRowBytes + 16u * (threadIdx.x + k * kT);
            v[k] = o < flen ? ld16u((gu32x4_a1 *)(base + fo + o)) : u32x4{0u, 0u, 0u, 0u};
        }
        uint32_t a = 0;
#pragma unroll
        for (int k = 0; k < kS; ++k) {
            const uint64_t o = (uint64_t)r * kRowBytes + 16u * (threadIdx.x + k * kT);
            if (o < flen) st16((gwu32x4_a4 *)(dst + (uint64_t)f * dst_stride + o), v[k]);
            a += v[k].x + v[k].y + v[k].z + v[k].w;
        }
        a = wave_add(a);
        uint32_t sm = a;
        if constexpr (kW > 1) {
            if ((threadIdx.x & 63) == 0) part[it][threadIdx.x >> 6] = a;
            __syncthreads();
            sm = 0;
#pragma unroll
            for (uint32_t w = 0; w < kW; ++w) sm += part[it][w];
        }
        if (threadIdx.x == 0) {
            if (rpf == 1)
                out[f] = sm;
            else
                atomicAdd(out + f, sm);
        }
    }
}

// ---- headers and receive-side verification -----------------------------------------------
// Headers are small (68-128 B): one thread per header, slicing-by-4 in the swapped domain
// from a 4 KiB LDS copy of the tables (S_j[i] at j*256 + i), byte steps C = (C >> 8) ^
// S_3[(C ^ b) & 255] for a ragged tail.  Header addresses are 4-byte aligned (host-checked).
__device__ __forceinline__ uint32_t thread_crc(const uint32_t *S, gbyte *p, uint32_t len, uint32_t partial) {
    uint32_t C = __builtin_bswap32(partial);
    uint32_t i = 0;
    for (; i + 4 <= len; i += 4) {
        const uint32_t X = C ^ *(guint *)(p + i);
        C = S[X & 255u] ^ S[256 + ((X >> 8) & 255u)] ^ S[512 + ((X >> 16) & 255u)] ^ S[768 + (X >> 24)];
    }
    for (; i < len; ++i) C = (C >> 8) ^ S[768 + ((C ^ p[i]) & 255u)];
    return __builtin_bswap32(C);
}

__device__ __forceinline__ void stage_slices(uint32_t *S, const uint32_t *__restrict__ img) {
    for (uint32_t t = threadIdx.x; t < 1024; t += blockDim.x) S[(t & 3u) * 256 + (t >> 2)] = img[kImgSliceT + t];
    __syncthreads();
}

// BasePath_t::headerChecksum (ref src/path/common/path.h:280-314): CRC mode bswap(uicrc(h, crclen))
// (so that CRC(header || stored) == 0), SUM mode the sum of word_count 32-bit words.
__global__ void __launch_bounds__(256) header_csum_kernel(const uint8_t *__restrict__ hdrs, uint32_t n, size_t stride,
                                                          uint32_t crclen, uint32_t word_count, int mode,
                                                          const uint32_t *__restrict__ img, uint8_t *out,
                                                          size_t out_stride) {
    __shared__ uint32_t S[1024];
    if (mode == LAMPI_CSUM_CRC32) stage_slices(S, img);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    gbyte *h = (gbyte *)(hdrs + (size_t)i * stride);
    uint32_t v = 0;
    if (mode == LAMPI_CSUM_CRC32) {
        v = __builtin_bswap32(thread_crc(S, h, crclen, kCrcInit));
    } else {
        for (uint32_t w = 0; w < word_count; ++w) v += *(guint *)(h + 4 * w);
    }
    // (out_stride = stride, out = hdrs + 68: the sender's `headerp->checksum = headerChecksum(...)` in place,
    // ref src/path/gm/sendFrag.cc:218-225 -- this thread read its header's bytes above, no other thread does)
    *(uint32_t *)(out + (size_t)i * out_stride) = v;
}

// One bit per fragment, set when it FAILS (wave ballot -> two mask words), plus a count.
__device__ __forceinline__ void emit_mask(uint32_t i, uint32_t n, bool bad, uint32_t *mask, uint32_t *nbad) {
    const uint64_t b = __ballot(bad && i < n);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w0 = (i - lane) / 32;  // first mask word of this wave (i - lane is a multiple of 64)
    if (lane == 0 && i < n) mask[w0] = (uint32_t)b;
    if (lane == 32 && i < n) mask[w0 + 1] = (uint32_t)(b >> 32);
    if (lane == 0 && b) atomicAdd(nbad, (uint32_t)__popcll(b));
}

// Receiver header check (ref src/path/gm/path.cc:364-393): CRC mode accepts iff
// uicrc(header, hdr_bytes) == 0 over the whole header including the stored checksum; SUM mode
// iff the sum of word_count words == 2 x the stored checksum (at csum_offset).
__global__ void __launch_bounds__(256) header_check_kernel(const uint8_t *__restrict__ hdrs, uint32_t n, size_t stride,
                                                           uint32_t hdr_bytes, uint32_t word_count,
                                                           uint32_t csum_offset, int mode,
                                                           const uint32_t *__restrict__ img, uint32_t *mask,
                                                           uint32_t *nbad) {
    __shared__ uint32_t S[1024];
    if (mode == LAMPI_CSUM_CRC32) stage_slices(S, img);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    if (i < n) {
        gbyte *h = (gbyte *)(hdrs + (size_t)i * stride);
        if (mode == LAMPI_CSUM_CRC32) {
            bad = thread_crc(S, h, hdr_bytes, kCrcInit) != 0u;
        } else {
            uint32_t v = 0;
            for (uint32_t w = 0; w < word_count; ++w) v += *(guint *)(h + 4 * w);
            const uint32_t stored = *(guint *)(h + csum_offset);
            bad = v != stored + stored;
        }
    }
    emit_mask(i, n, bad, mask, nbad);
}

// The IB variant (ref src/path/ib/path.cc:652-680; senders src/path/ib/sendFrag.cc:306-314, ACKs
// :327-335): the sender stores uicrc(h, crclen) / uicsum(h, crclen) as it is (not byte-swapped) and
// the receiver recomputes it over the same crclen bytes and compares it with the stored word.
// uicsum of a fresh state: little-endian words, a 1-3 byte tail zero-padded in its high bytes.
__global__ void __launch_bounds__(256) header_compare_kernel(const uint8_t *__restrict__ hdrs, uint32_t n,
                                                             size_t stride, uint32_t crclen, uint32_t csum_offset,
                                                             int mode, const uint32_t *__restrict__ img,
                                                             uint32_t *mask, uint32_t *nbad) {
    __shared__ uint32_t S[1024];
    if (mode == LAMPI_CSUM_CRC32) stage_slices(S, img);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    if (i < n) {
        gbyte *h = (gbyte *)(hdrs + (size_t)i * stride);
        uint32_t v = 0;
        if (mode == LAMPI_CSUM_CRC32) {
            v = thread_crc(S, h, crclen, kCrcInit);
        } else {
            uint32_t w = 0;
            for (; w + 4 <= crclen; w += 4) v += *(guint *)(h + w);
            for (uint32_t b = 0; w + b < crclen; ++b) v += (uint32_t)h[w + b] << (8 * b);
        }
        bad = v != *(guint *)(h + csum_offset);
    }
    emit_mask(i, n, bad, mask, nbad);
}

// CheckData (ref src/path/gm/recvFrag.h:213-257): fragment i is corrupt iff its length is
// nonzero and calc[i] != expected; expected values and lengths are read through byte strides
// (e.g. straight out of an array of headers: dataChecksum @64, dataLength @20).
__global__ void __launch_bounds__(256) check_data_kernel(const uint32_t *__restrict__ calc, const uint8_t *expected,
                                                         size_t exp_stride, const uint8_t *lengths, size_t len_stride,
                                                         uint32_t n, uint32_t *mask, uint32_t *nbad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    if (i < n) {
        const uint32_t len = lengths ? *(guint *)(lengths + (size_t)i * len_stride) : 1u;
        bad = len != 0 && calc[i] != *(guint *)(expected + (size_t)i * exp_stride);
    }
    emit_mask(i, n, bad, mask, nbad);
}

// Checksums into records: dst + i*stride gets vals[i] (e.g. gmHeaderData.dataChecksum @64 of a
// 72-byte header array, SURVEY.md 8(b) optional strided output).
__global__ void __launch_bounds__(256) scatter_u32_kernel(const uint32_t *__restrict__ vals, uint32_t n, uint8_t *dst,
                                                          size_t stride) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) *(uint32_t *)(dst + (size_t)i * stride) = vals[i];
}

// ---- chained checksums over typemap pieces ------------------------------------------------
// Fragment f = pieces first[f] .. first[f+1]-1 concatenated (ref src/path/gm/sendFrag.cc:157-217,
// src/path/common/BaseDesc.cc:72-163).  Pass 1 (SUM only): byte phase of every piece.  Pass 2:
// per-piece values, large pieces one wavefront each (crc_rows_kernel / sum_rows_kernel over
// PieceSource), small ones one thread each (below).  Pass 3: one wavefront per fragment folds
// them: CRC (C, len) pairs combine as (a, la) . (b, lb) = (shift_lb(a) ^ b, la + lb) --
// associative, so lanes fold contiguous runs of pieces and a DPP-free shuffle tree joins the
// lanes -- and the caller's register enters as shift_total(partial); SUM values just add.
__global__ void __launch_bounds__(256) chain_phase_kernel(const lampi_copy_desc *__restrict__ d,
                                                          const uint32_t *__restrict__ first, uint32_t nfrags,
                                                          uint32_t *__restrict__ phase) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nfrags) return;
    uint32_t off = 0;
    for (uint32_t k = first[f]; k < first[f + 1]; ++k) {
        phase[k] = off & 3u;
        const uint32_t len = d[k].copylen > d[k].csumlen ? d[k].copylen : d[k].csumlen;
        off += len;
    }
}

// pieces of at most `small` bytes: byte / aligned-word loops in one thread
__global__ void __launch_bounds__(256) chain_small_kernel(const lampi_copy_desc *__restrict__ d, uint32_t npieces,
                                                          const uint32_t *__restrict__ phase, uint32_t small, int mode,
                                                          const uint32_t *__restrict__ img, uint32_t *__restrict__ vals) {
    __shared__ uint32_t S[1024];
    if (mode == LAMPI_CSUM_CRC32) stage_slices(S, img);
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npieces) return;
    const lampi_copy_desc x = d[k];
    const uint32_t len = x.copylen > x.csumlen ? x.copylen : x.csumlen;
    if (len > small) return;
    gbyte *p = (gbyte *)(uintptr_t)x.src;
    gwbyte *q = (gwbyte *)(uintptr_t)x.dst;
    for (uint32_t i = 0; i < x.copylen; ++i) q[i] = p[i];
    if (mode == LAMPI_CSUM_CRC32) {
        uint32_t C = 0;  // swapped domain, zero register
        uint32_t i = 0;
        for (; i < len && (((uintptr_t)(p + i)) & 3u); ++i) C = (C >> 8) ^ S[768 + ((C ^ p[i]) & 255u)];
        for (; i + 4 <= len; i += 4) {
            const uint32_t X = C ^ *(guint *)(p + i);
            C = S[X & 255u] ^ S[256 + ((X >> 8) & 255u)] ^ S[512 + ((X >> 16) & 255u)] ^ S[768 + (X >> 24)];
        }
        for (; i < len; ++i) C = (C >> 8) ^ S[768 + ((C ^ p[i]) & 255u)];
        vals[k] = __builtin_bswap32(C);
    } else {
        const uint32_t ph = phase[k];
        uint32_t acc = 0, i = 0;
        for (; i < len && (((uintptr_t)(p + i)) & 3u); ++i) acc += (uint32_t)p[i] << (8 * ((ph + i) & 3u));
        for (; i + 4 <= len; i += 4) {  // a whole word lands rotated by its phase
            const uint32_t w = *(guint *)(p + i);
            const uint32_t r = 8 * ((ph + i) & 3u);
            acc += r ? (w << r) | (w >> (32 - r)) : w;
        }
        for (; i < len; ++i) acc += (uint32_t)p[i] << (8 * ((ph + i) & 3u));
        vals[k] = acc;
    }
}

// RecvDesc_t::CopyToApp's non-contiguous branch over a chain batch (ref src/path/common/BaseDesc.cc:326-340:
// non_contiguous_copy, then CheckData(checkSum, len_copied)): with `copied` set, fragment f's verdict --
// copied[f] = the bytes it copied, or -1 when they were copied but the checksum differs from the expected value
// at expected + f * exp_stride; mask bit / nbad as lampi_copy_to_app_batch.  init: CRC from
// CRC_INITIAL_REGISTER (nonContigCopyFunction's firstCall, gm/recvFrag.h:198-200) instead of the first piece's
// partial; nocheck: checksumming off (copy only, checksum 0, every fragment DataOK).
// (ChainVerdict: frag_csum_kernels.h)
__device__ __forceinline__ void chain_result(const ChainVerdict &v, uint32_t f, uint32_t csum, uint64_t copied,
                                             uint32_t *out) {
    out[f] = csum;
    if (!v.copied) return;
    const bool bad = !v.nocheck && copied != 0 && csum != *(const guint *)(v.expected + (size_t)f * v.exp_stride);
    v.copied[f] = bad ? -1ll : (int64_t)copied;
    if (bad) {
        atomicOr(v.mask + (f >> 5), 1u << (f & 31u));
        atomicAdd(v.nbad, 1u);
    }
}

// C after `len` zero bytes (normal domain), T[e*128 + p*16 + v] = shift_{2^e}(v << 4p)
__device__ __forceinline__ uint32_t shift_by(const uint32_t *T, uint32_t C, uint32_t len) {
    while (len) {
        const uint32_t e = __builtin_ctz(len);
        len &= len - 1;
        const uint32_t *t = T + e * 128;
        uint32_t r = 0;
#pragma unroll
        for (int p = 0; p < 8; ++p) r ^= t[p * 16 + ((C >> (4 * p)) & 15u)];
        C = r;
    }
    return C;
}

__global__ void __launch_bounds__(256) chain_fold_kernel(const lampi_copy_desc *__restrict__ d,
                                                         const uint32_t *__restrict__ first, uint32_t nfrags,
                                                         const uint32_t *__restrict__ vals, int mode,
                                                         const uint32_t *__restrict__ img, uint32_t *__restrict__ out,
                                                         const ChainVerdict v) {
    __shared__ uint32_t T[32 * 128];  // 16 KiB: nibble tables of shift by 2^e bytes
    if (mode == LAMPI_CSUM_CRC32) {
        for (uint32_t t = threadIdx.x; t < 32 * 128; t += blockDim.x) {
            const uint32_t e = t >> 7, p = (t >> 4) & 7u, v = t & 15u;
            const uint32_t *col = img + kImgPow2Cols + e * 32 + 4 * p;
            uint32_t x = 0;
            if (v & 1) x ^= col[0];
            if (v & 2) x ^= col[1];
            if (v & 4) x ^= col[2];
            if (v & 8) x ^= col[3];
            T[t] = x;
        }
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t f = uniform(blockIdx.x * kWaves + (threadIdx.x >> 6));
    if (f >= nfrags) return;
    const uint32_t k0 = first[f], k1 = first[f + 1];
    const uint32_t np = k1 > k0 ? k1 - k0 : 0u;
    const uint32_t per = (np + 63) / 64;  // contiguous run of pieces per lane
    const uint32_t a = k0 + min(np, lane * per), b = k0 + min(np, (lane + 1) * per);
    // non_contiguous_copy's length: the bytes copied into the typemap pieces (BaseDesc.cc:160-161)
    uint64_t copied = 0;
    if (v.copied) {
        for (uint32_t k = a; k < b; ++k) copied += d[k].copylen;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)copied, o), hi = (uint32_t)__shfl_xor((int)(uint32_t)(copied >> 32), o);
            copied += ((uint64_t)hi << 32) | lo;
        }
    }
    if (mode != LAMPI_CSUM_CRC32) {
        uint32_t acc = 0;
        for (uint32_t k = a; k < b; ++k) acc += vals[k];
        acc = wave_add(acc);
        if (lane == 0) chain_result(v, f, v.nocheck ? 0u : acc, copied, out);
        return;
    }
    uint32_t C = 0, L = 0;
    for (uint32_t k = a; k < b; ++k) {
        const uint32_t len = d[k].copylen > d[k].csumlen ? d[k].copylen : d[k].csumlen;
        C = shift_by(T, C, len) ^ vals[k];
        L += len;
    }
    // ordered tree: at distance s, lane l (l % 2s == 0) absorbs lane l + s
#pragma unroll
    for (uint32_t s = 1; s < 64; s <<= 1) {
        const uint32_t oc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane + s) & 63u) * 4), (int)C);
        const uint32_t ol = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane + s) & 63u) * 4), (int)L);
        if ((lane & (2 * s - 1)) == 0) {
            C = shift_by(T, C, ol) ^ oc;
            L += ol;
        }
    }
    if (lane == 0) {
        const uint32_t partial = np && !v.init ? d[k0].partial : kCrcInit;
        chain_result(v, f, shift_by(T, partial, L) ^ C, copied, out);
    }
}

// ---- 64-bit csum over a chained stream -----------------------------------------------------
// Host path of csum / bcopy_csum: the pieces' phase-shifted sums add up to the increment; the
// new (lastPartialLong, lastPartialLength) is the trailing partial word of the virtual stream
// [old partial bytes | the len new bytes].  out3 = {sum, plong, plen}.
__global__ void sum64_finish_kernel(const uint64_t *__restrict__ vals, uint32_t nv, const uint8_t *__restrict__ src,
                                    uint64_t len, uint64_t plong, uint64_t plen, uint64_t *__restrict__ out3,
                                    uint64_t *sig, uint64_t seq) {
    uint64_t acc = 0;
    for (uint32_t i = threadIdx.x; i < nv; i += blockDim.x) acc += vals[i];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
    __shared__ uint64_t part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x != 0) return;
    uint64_t total = 0;
    for (uint32_t w = 0; w < (blockDim.x + 63) / 64; ++w) total += part[w];
    const uint64_t end = plen + len;  // virtual stream length
    const uint64_t nl = end & 7u;
    uint64_t np = 0;
    for (uint64_t b = end - nl; b < end; ++b) {
        const uint64_t byte = b < plen ? (plong >> (8 * b)) & 0xFFu : src[b - plen];
        np |= byte << (8 * (b & 7u));
    }
    out3[0] = total;
    out3[1] = np;
    out3[2] = nl;
    signal_host(sig, seq);
}

// ---- synthetic stream fill ----------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}
__device__ __forceinline__ uint64_t stream_word(uint64_t seed, uint64_t i) {
    return mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
}

__global__ void __launch_bounds__(256) fill_stream_kernel(uint8_t *dst, size_t nbytes, uint64_t seed,
                                                          uint64_t byte_off) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint32_t s = (uint32_t)(byte_off & 7u);
    const uint64_t w0 = byte_off >> 3;
    const size_t nfull = nbytes / 16;
    const bool aligned16 = (((uintptr_t)dst) & 15u) == 0;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < nfull; t += stride) {
        uint64_t a = stream_word(seed, w0 + 2 * t);
        uint64_t b = stream_word(seed, w0 + 2 * t + 1);
        uint64_t lo = a, hi = b;
        if (s) {
            uint64_t c = stream_word(seed, w0 + 2 * t + 2);
            lo = (a >> (8 * s)) | (b << (64 - 8 * s));
            hi = (b >> (8 * s)) | (c << (64 - 8 * s));
        }
        if (aligned16) {
            reinterpret_cast<ulonglong2 *>(dst)[t] = make_ulonglong2(lo, hi);
        } else {
            for (int j = 0; j < 8; ++j) dst[16 * t + j] = (uint8_t)(lo >> (8 * j));
            for (int j = 0; j < 8; ++j) dst[16 * t + 8 + j] = (uint8_t)(hi >> (8 * j));
        }
    }
    // tail bytes
    const size_t tail0 = nfull * 16;
    for (size_t i = tail0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += stride) {
        uint64_t pos = byte_off + i;
        dst[i] = (uint8_t)(stream_word(seed, pos >> 3) >> (8 * (pos & 7u)));
    }
}

// ---- CRC combine over equal-size pieces ---------------------------------------------------
// vals[0..n): crc(s_k, piece_k) of consecutive pieces of a front-padded message, each
// piece B bytes (the first may be shorter: leading zeros are free).  Tree over a
// power-of-two frame padded with zero pieces in front:  (A, B) -> shift_B(A) ^ B.
// tabs[lvl*128 + p*16 + v]: normal-domain nibble tables of shift by B * 2^lvl.
__global__ void __launch_bounds__(1024) crc_combine_kernel(const uint32_t *__restrict__ vals, uint32_t n,
                                                           const uint32_t *__restrict__ tabs, uint32_t npow,
                                                           uint32_t *__restrict__ out, uint64_t *sig, uint64_t seq) {
    extern __shared__ __attribute__((aligned(16))) uint32_t v[];  // 2 * npow words: ping-pong
    const uint32_t pad = npow - n;
    for (uint32_t i = threadIdx.x; i < npow; i += blockDim.x) v[i] = (i < pad) ? 0u : vals[i - pad];
    __syncthreads();
    uint32_t *src = v, *dst = v + npow;
    uint32_t lvl = 0;
    for (uint32_t m = npow; m > 1; m >>= 1, ++lvl) {
        const uint32_t *t = tabs + lvl * 128;
        for (uint32_t i = threadIdx.x; i < m / 2; i += blockDim.x) {
            const uint32_t a = src[2 * i];
            uint32_t r = src[2 * i + 1];
#pragma unroll
            for (int p = 0; p < 8; ++p) r ^= t[p * 16 + ((a >> (4 * p)) & 15u)];
            dst[i] = r;
        }
        __syncthreads();
        uint32_t *tmp = src;
        src = dst;
        dst = tmp;
    }
    if (threadIdx.x == 0) {
        out[0] = src[0];
        signal_host(sig, seq);
    }
}

// ---- SUM over a chained stream ------------------------------------------------------------
// The body [t, t + 4*nb) was summed by sum_rows_kernel in word-aligned pieces (partials);
// this adds the head (completing the caller's partial word) and the tail partial word and
// produces the new (pint, plen) state.  out3 = {sum, pint, plen}.  partials == nullptr (small
// host calls, one kernel in all): the workgroup sums the body words of src itself -- aligned
// dwords funnel-shifted by the body's byte offset, consecutive lanes on consecutive words, eight
// loads in flight per thread (host memory: each load is a PCIe round trip).
__global__ void sum_stream_finish_kernel(const uint32_t *__restrict__ partials, uint32_t npart,
                                         const uint8_t *__restrict__ src, uint64_t len, uint32_t pint,
                                         uint32_t plen, uint32_t *__restrict__ out3, uint64_t *sig, uint64_t seq) {
    __shared__ uint32_t red[1024];
    uint32_t acc = 0;
    if (partials != nullptr) {
        for (uint32_t i = threadIdx.x; i < npart; i += blockDim.x) acc += partials[i];
    } else {
        const uint32_t k0 = plen >= 4 ? 0u : plen;
        const uint64_t take = k0 ? (4u - k0 < len ? 4u - k0 : len) : 0u;
        if (!(k0 && k0 + take < 4)) {  // otherwise every byte completes the partial word
            const uint64_t nw = (len - take) >> 2;  // body words
            const uintptr_t b0 = (uintptr_t)(src + take);
            const uint32_t sh = (uint32_t)(b0 & 3u);
            const uint32_t *a = (const uint32_t *)(b0 - sh);
            for (uint64_t i0 = threadIdx.x; i0 < nw; i0 += 8ull * blockDim.x) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint64_t i = i0 + (uint64_t)u * blockDim.x;
                    v[u] = i < nw ? (sh ? __builtin_amdgcn_alignbyte(a[i + 1], a[i], sh) : a[i]) : 0u;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += v[u];
            }
        }
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t s = blockDim.x / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    uint32_t sum = red[0];
    uint32_t k = plen >= 4 ? 0u : plen;
    uint64_t pos = 0;
    if (k) {
        uint32_t w = pint;
        uint64_t take = 4 - k;
        if (take > len) take = len;
        for (uint64_t j = 0; j < take; ++j) {
            const uint32_t sh = 8u * (uint32_t)(k + j);
            w = (w & ~(0xFFu << sh)) | ((uint32_t)src[j] << sh);
        }
        sum += w - pint;
        pos = take;
        if (k + take < 4) {
            out3[0] = sum;
            out3[1] = w;
            out3[2] = k + (uint32_t)take;
            signal_host(sig, seq);
            return;
        }
    }
    const uint64_t body = (len - pos) & ~3ull;
    const uint64_t r = (len - pos) & 3ull;
    uint32_t tail = 0;
    for (uint64_t j = 0; j < r; ++j) tail |= (uint32_t)src[pos + body + j] << (8 * j);
    out3[0] = sum + tail;
    out3[1] = tail;
    out3[2] = (uint32_t)r;
    signal_host(sig, seq);
}

// Fragment-strided stream: fragment i of dst (frag_len bytes, frag_len % 8 == 0) holds stream
// bytes [(k0 + i*kstep) * frag_len, +frag_len) -- a round-robin shard of a global batch.
__global__ void __launch_bounds__(256) fill_frags_kernel(uint64_t *dst, size_t n, uint64_t frag_words,
                                                         uint64_t seed, uint64_t k0, uint64_t kstep) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t total = n * frag_words;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        const uint64_t i = t / frag_words, j = t - i * frag_words;
        dst[t] = stream_word(seed, (k0 + i * kstep) * frag_words + j);
    }
}

}  // namespace

// ---- launchers ---------------------------------------------------------------------------
int crc_grid(int device) {
    static int cu[64] = {0};
    if (device < 0 || device >= 64) device = 0;
    if (!cu[device]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0) v = 256;
        cu[device] = v;
    }
    return cu[device];
}

// fragments per wave for the non-persistent grids: enough work per workgroup to amortise the
// 64.5 KiB table staging, small enough to keep the chip's read window compact
static uint32_t pick_fpw(size_t n, uint32_t R) {
    // measured on MI355X (profiles/r01_ablation*.txt): 4 KiB fragments fpw 32, >= 16 KiB fpw 12
    uint32_t fpw = R >= 4 ? 12u : 32u;
    while (fpw > 1 && (size_t)kWaves * fpw * 512 > n) fpw >>= 1;  // small batches: more workgroups
    return fpw;
}

// Large fragments of a known length (messages; descriptor batches pass frag_len 0): halve the
// fragments per wave while the grid has fewer than 2048 workgroups (4 per resident slot) and a
// workgroup of kWv waves would carry more than 512 KiB -- a 1 GiB message of 65,456-byte
// fragments otherwise runs as ~500 workgroups of 2-3 MiB, most of the chip idle in the tail.
static uint32_t spread_fpw(uint32_t fpw, size_t n, int kWv, size_t frag_len) {
    while (frag_len > 0 && fpw > 1 && (n + (size_t)kWv * fpw - 1) / ((size_t)kWv * fpw) < 2048 &&
           (size_t)kWv * fpw * frag_len > (512u << 10))
        fpw >>= 1;
    return fpw;
}

constexpr int kRegularChains = 2;

// crc_rows_kernel with a fused copy: 8-wave workgroups (16 waves/CU, one row in flight each),
// half the fragments per wave of the 4-wave schedule so a workgroup covers the same span
template <class Src>
static void launch_crc_rows_copy(const Src &src, size_t n, uint32_t R, const uint32_t *img, uint32_t *out,
                                 hipStream_t s, size_t frag_len = 0) {
    static_assert(Src::kCopy, "the staging area is for the fused copy");
    // 10-wave workgroups (20 waves/CU): 61% against 69% (4M x 4 KiB); with half the fragments per
    // wave, 4 / 6 waves: descriptors 62-64 / 52% against 74-75% (profiles/r02_crc_copy_fpw/waves/)
    constexpr int kWv = 2 * kWaves;
    // a quarter of the read kernel's fragments per wave: half for the 8-wave workgroup (the same span),
    // half again for the copy (shorter-lived workgroups, profiles/r02_crc_copy_fpw/: +2-3 points)
    const uint32_t fpw = spread_fpw(std::max(1u, pick_fpw(n, R) / 4), n, kWv, frag_len);
    const dim3 grid((unsigned)((n + (size_t)kWv * fpw - 1) / ((size_t)kWv * fpw)));
    hipLaunchKernelGGL((crc_rows_kernel<Src, kWv>), grid, dim3(64 * kWv), 0, s, src, n, fpw, img, out);
}

// fragments per workgroup of crc_stream_kernel: 96 (measured: tools/microbench/frags_sweep.hip,
// 12-wave workgroups -- 96 beat 64/128/192/256 on config C and on 4 KiB descriptors: shorter
// workgroups shrink the end-of-kernel tail, and 96 uniform 4 KiB fragments are 8 rows per chain),
// halved for small batches until they give one workgroup per CU (a 16 MiB chunk of 65,456-byte
// fragments is only 256 fragments).  Every workgroup stages ~77 KiB of LDS tables, so more
// workgroups than CUs only repeat that prologue: 4,096 x 4 KiB took 21.9 us at >= 2048
// workgroups, 14.6 us at >= 512, 9.95 us at >= 256 (bench.py --latency); config C unchanged.
// With the fragment length known (messages), large fragments are spread as in spread_fpw
// (16,404 x 65,456 bytes: 6 fragments per workgroup, not 48: CRC 55 -> 62%, SUM 62 -> 74%;
// profiles/r02_bigfrag_ab.txt).
constexpr uint32_t kCrcFpg = 96;
static uint32_t frags_per_wg(size_t n, size_t frag_len = 0) {
    static const uint32_t fpg_env = [] {  // (A/B knob LAMPI_STREAM_FPG: fragments per workgroup, <= 256)
        const char *e = LAMPI_AB_ENV("LAMPI_STREAM_FPG");
        return e ? (uint32_t)std::min(256, std::max(1, std::atoi(e))) : 0u;
    }();
    uint32_t fpg = fpg_env ? fpg_env : kCrcFpg;
    while (fpg > 3 && n / fpg < 256) fpg >>= 1;
    return spread_fpw(fpg, n, 1, frag_len);
}

// crc_stream_kernel: ring depth and chains per wave (measured, tools/microbench/frags_sweep.hip)
constexpr int kStreamD = 2, kStreamK = 1, kStreamWv = 12, kStreamCap = 6;
// the SUM piece streams (no tables, so no per-workgroup staging to amortise): waves per
// workgroup, waves per SIMD and fragments per workgroup.  Same-box A/B (profiles/r02_sum_stream/,
// two rounds): 48 fragments per 768-thread workgroup config C SUM 74.2-76.8 -> 78.1-78.3%, 4 KiB
// descriptors 78.9 -> 79.1-80.3%; 24 / 32 / 64 fragments 71 / 76.5 / 77.5%; 8-wave workgroups 76.6%;
// 256-thread workgroups of 8 / 16 / 32 fragments 78.2-78.9 / 77.5-77.9 / 76.4% (4 KiB descriptors
// 74 / 80 / 77%); 8 waves per SIMD spills (scratch next to the asm load ring: not run).
constexpr int kSumWv = 12, kSumCap = 6;
constexpr uint32_t kSumFpg = 48;
static uint32_t sum_frags_per_wg(size_t n, size_t frag_len = 0) {
    uint32_t fpg = kSumFpg;
    while (fpg > 3 && n / fpg < 256) fpg >>= 1;
    return spread_fpw(fpg, n, 1, frag_len);
}

static dim3 frags_grid(size_t n, uint32_t fpg) { return dim3((unsigned)((n + fpg - 1) / fpg)); }

static dim3 grid_for(size_t n, uint32_t fpw) { return dim3((unsigned)((n + (size_t)kWaves * fpw - 1) / ((size_t)kWaves * fpw))); }

// Descriptor batches of up to kPlanMax fragments with LAMPI_CSUM_BY_BYTES run byte-balanced (plan_kernel,
// then the piece streams over its segments): the host cannot see the lengths, and a count split leaves
// a batch of few large fragments to a few workgroups (1 GiB of 4 MiB descriptors: 34% of the roofline).
// Not the default: the plan launch adds ~10 us to every call (1 x 4 KiB: 7.8 -> 20 us, 4,096 x 4 KiB:
// 10.6 -> 23 us; profiles/r03/bigdesc_ab.txt).  Larger batches keep the count split.
// Device scratch for a launch sequence on stream s (the byte-balanced plan, the light copy's group
// values): one grow-only buffer per (calling thread, device, stream), reused in stream order -- a
// call's kernels finish with it before the same thread's next call on that stream starts.  Keyed by
// thread as well, so two threads calling on one stream (torch's default stream, handle 0) never share
// a buffer: their producer and join launches may interleave on the stream, each pair reading only its
// own values.  Per-call hipMallocAsync / hipFreeAsync put a ~6 us gap before the next kernel on the
// stream (profiles/r03/light_join_gap.txt).  Growing first synchronizes s (this thread's earlier
// launches on it are the only users of the old buffer), then frees it.  The thread's buffers are
// freed at thread exit, by lampi_host_release() and, per stream, when the host pipeline destroys its
// streams (release_stream_scratch); lampi_device_scratch_bytes() counts them for leak checks.
// While s is being captured into a graph the graph gets its own allocation (hipMallocAsync; *pooled
// set: release it with scratch_done), so no replay depends on a buffer a later call may replace.
namespace {
std::atomic<int64_t> g_scratch_bytes{0};

// What the census kernel records about a batch (BatchShape, below): host-mapped, one per entry-point kind.
struct BatchShape {
    uint32_t seq;      // written last; 0: nothing recorded yet
    uint32_t sampled;  // descriptors sampled (up to 64, spread over the batch)
    uint32_t rmin, rmax;  // fewest / most rows (4 KiB) among them
    uint32_t nhalf;    // how many were at most 2 KiB
    uint32_t nwhole;   // how many were whole 4 KiB rows (> 0 bytes) at a 16-byte-aligned address
    uint32_t nmis;     // how many were 1-2 KiB and ended off the 16-byte grid
    uint32_t n12k;     // how many were 1-2 KiB
    uint32_t n1k;      // how many were at most 1 KiB
    uint32_t ncontig;  // how many lay where a contiguous run of equal fragments from fragment 0 puts them (fragment i
                       // at d[0].addr + i * d[0].length, the same length and register; d[0].addr 16-byte aligned)
    uint32_t len0;     // fragment 0's length
    uint32_t pad;
};
constexpr int kShapeSlots = 8;  // shape records per (thread, device, stream): descriptor arrays remembered
constexpr int64_t kLeftBytes = 256;

struct ScratchTable {
    struct Slot {
        void *p = nullptr;
        size_t cap = 0;
        // learned batch shapes, one record per (entry-point kind, descriptor array): a stream that
        // alternates batches from different arrays (GM's and IB's receive rings) keeps one shape each
        struct ShapeRec {
            const void *key = nullptr;  // the batch's descriptor array
            int kind = -1;
            BatchShape *rec = nullptr;  // host-mapped (coherent), lazily allocated; reused on eviction
            uint32_t calls = 0;
            uint64_t used = 0;          // the slot's call count at its last use (least recently used: evicted)
        };
        ShapeRec shapes[kShapeSlots];
        uint64_t shape_tick = 0;
        uint32_t *left = nullptr;  // the pair kernel's two leftover counters (device, zeroed at creation)
        uint32_t left_calls = 0;
        bool pair_broken = false;  // the counters could not be re-zeroed after a failed launch
    };
    std::map<std::pair<int, hipStream_t>, Slot> slots;
    ScratchTable() = default;
    ScratchTable(const ScratchTable &) = delete;
    ScratchTable &operator=(const ScratchTable &) = delete;
    ~ScratchTable();

    // Free the slots whose key satisfies pred, each on its own device after its stream drained;
    // errors are ignored (this also runs at thread exit).
    template <class Pred>
    void release_if(Pred pred) {
        int cur = -1;
        const bool have_cur = hipGetDevice(&cur) == hipSuccess;
        int set = cur;
        for (auto it = slots.begin(); it != slots.end();) {
            if (!pred(it->first)) {
                ++it;
                continue;
            }
            if (it->first.first != set && hipSetDevice(it->first.first) == hipSuccess) set = it->first.first;
            (void)hipStreamSynchronize(it->first.second);
            (void)hipFree(it->second.p);
            g_scratch_bytes.fetch_sub((int64_t)it->second.cap, std::memory_order_relaxed);
            if (it->second.left) {
                (void)hipFree(it->second.left);
                g_scratch_bytes.fetch_sub(kLeftBytes, std::memory_order_relaxed);
            }
            for (auto &r : it->second.shapes)
                if (r.rec) {
                    (void)hipHostFree(r.rec);
                    g_scratch_bytes.fetch_sub((int64_t)sizeof(BatchShape), std::memory_order_relaxed);
                    r.rec = nullptr;
                }
            it = slots.erase(it);
        }
        if (have_cur && set != cur) (void)hipSetDevice(cur);
    }
};
thread_local ScratchTable t_scratch;
// Set once this thread's t_scratch has been destroyed.  Thread-local objects are destroyed in
// reverse order of construction, so the host pipeline's (host_msg.cc, t_pipe) may run after this one and
// call release_stream_scratch(): that must not touch the destroyed map.  A trivially destructible
// thread_local stays readable until the thread ends.
thread_local bool t_scratch_dead = false;
ScratchTable::~ScratchTable() {
    release_if([](const std::pair<int, hipStream_t> &) { return true; });
    t_scratch_dead = true;
}
}  // namespace

static hipError_t stream_scratch(hipStream_t s, size_t bytes, void **out, bool *pooled) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipError_t ce = hipStreamIsCapturing(s, &cs);
    if (ce != hipSuccess) return ce;
    *pooled = cs != hipStreamCaptureStatusNone;
    if (*pooled) return hipMallocAsync(out, bytes, s);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    ScratchTable::Slot &slot = t_scratch.slots[{dev, s}];
    if (slot.cap < bytes) {
        if (slot.p) {
            e = hipStreamSynchronize(s);  // this thread's earlier launches on s still read the old buffer
            if (e == hipSuccess) e = hipFree(slot.p);
            if (e != hipSuccess) return e;  // the old buffer stays in the slot, still valid
            g_scratch_bytes.fetch_sub((int64_t)slot.cap, std::memory_order_relaxed);
            // only the buffer goes: the learned shapes, the pair counters and their state are not tied to its
            // size (`slot = {}` here leaked the host-mapped shape records and the counters)
            slot.p = nullptr;
            slot.cap = 0;
        }
        const size_t want = std::max<size_t>(bytes + bytes / 4, 1u << 20);
        e = hipMalloc(&slot.p, want);
        if (e != hipSuccess) {
            slot.p = nullptr;
            slot.cap = 0;
            return e;
        }
        slot.cap = want;
        g_scratch_bytes.fetch_add((int64_t)want, std::memory_order_relaxed);
    }
    *out = slot.p;
    return hipSuccess;
}

// The pair kernel's leftover counters for stream s (this thread's): two, zeroed on the stream when created;
// calls alternate between them, each call's leftover kernel zeroing the next call's.
static hipError_t pair_counters(hipStream_t s, uint32_t **cur, uint32_t **next) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    ScratchTable::Slot &slot = t_scratch.slots[{dev, s}];
    if (!slot.left) {
        void *p = nullptr;
        e = hipMalloc(&p, kLeftBytes);
        if (e != hipSuccess) return e;
        e = hipMemsetAsync(p, 0, kLeftBytes, s);
        if (e != hipSuccess) {
            (void)hipFree(p);
            return e;
        }
        slot.left = (uint32_t *)p;
        g_scratch_bytes.fetch_add(kLeftBytes, std::memory_order_relaxed);
    }
    if (slot.pair_broken) return hipErrorNotReady;  // (learned_rows_hint no longer picks pairs here)
    const uint32_t par = slot.left_calls++ & 1u;
    *cur = slot.left + par;
    *next = slot.left + (par ^ 1u);
    return hipSuccess;
}

// After a failed pair launch: both counters back to zero on the stream (a failing memset too: the pair
// schedule is then retired for this stream, since a stale count could index past the leftover list).
static void reset_pair_counters(hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    auto it = t_scratch.slots.find({dev, s});
    if (it == t_scratch.slots.end() || !it->second.left) return;
    if (hipMemsetAsync(it->second.left, 0, 2 * sizeof(uint32_t), s) != hipSuccess) {
        (void)hipGetLastError();
        it->second.pair_broken = true;
    }
}

// Whether stream s may still take the pair counters (false once reset_pair_counters could not re-zero them):
// schedules that list leftovers through them check this before they are chosen.
static bool pair_counters_ok(hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    auto it = t_scratch.slots.find({dev, s});
    return it == t_scratch.slots.end() || !it->second.pair_broken;
}

void release_stream_scratch(hipStream_t s) {
    if (t_scratch_dead) return;  // everything was released when the table went
    t_scratch.release_if([s](const std::pair<int, hipStream_t> &k) { return k.second == s; });
}

void release_thread_scratch() {
    if (t_scratch_dead) return;
    t_scratch.release_if([](const std::pair<int, hipStream_t> &) { return true; });
}

int64_t device_scratch_bytes() { return g_scratch_bytes.load(std::memory_order_relaxed); }

static hipError_t scratch_done(hipStream_t s, void *p, bool pooled, hipError_t e) {
    const hipError_t f = pooled ? hipFreeAsync(p, s) : hipSuccess;
    return e != hipSuccess ? e : f;
}

// ---- Batch shapes learned on the device ----------------------------------------------------------
// A descriptor batch's lengths live on the device, so the host cannot size a one-row-per-wave grid for
// it (LAMPI_CSUM_ROWS_HINT is the caller's way to say it).  Without a hint the library learns the shape
// from the stream's earlier batches: every kShapeEvery-th call of an entry point on a stream (and its
// first) launches census_kernel ahead of the batch's kernels -- one wave reading up to 64 descriptors
// spread over the batch, recording the fewest / most rows among them into a host-mapped BatchShape --
// and a later call on that stream reads the record (no synchronization: whatever has landed) and, when
// the sampled fragments were all of 8 or more rows within a factor of two of each other, runs as if
// the caller had passed LAMPI_CSUM_ROWS_HINT(most rows); CRC copies and receives whose sampled
// fragments were all at most 2 KiB (IB's payloads) run two fragments to a wave
// (crc_light_pair_copy_kernel).  The results never depend on it (every
// schedule is exact for any lengths); the first batches of a stream, mixed batches (config C), batches
// under kShapeMin fragments and graph captures keep the given schedule.  LAMPI_CSUM_NO_SHAPES=1
// turns it off.
constexpr size_t kShapeMin = 256;
constexpr uint32_t kShapeEvery = 16;
constexpr uint32_t kShapeRows = 8;  // fewest rows of a learned hint (CRC 16 KiB copies: hint 4 no better, receive worse)
constexpr uint32_t kShapeRowsSum = 4;  // SUM copies and receives: 16 KiB with hint 4 72 -> 78%, receive 68 -> 75%

template <class Src>
__global__ void __launch_bounds__(64) census_kernel(const Src src, size_t n, BatchShape *rec, uint32_t seq) {
    const uint32_t l = threadIdx.x;
    const uint32_t m = (uint32_t)min<size_t>(n, 64);
    uint32_t rmin = 0xFFFFFFFFu, rmax = 0u, half = 0u, full = 0u, mis = 0u, k12 = 0u, k1 = 0u, contig = 0u;
    const FragInfo f0i = src.get(0);  // (sample 0 is fragment 0: the run's start)
    if (l < m) {
        const size_t idx = (size_t)l * n / m;
        const FragInfo fi = src.get(idx);
        contig = fi.len == f0i.len && fi.partial == f0i.partial && ((uintptr_t)f0i.addr & 15u) == 0 &&
                         (uint64_t)(uintptr_t)fi.addr == (uint64_t)(uintptr_t)f0i.addr + (uint64_t)idx * f0i.len
                     ? 1u : 0u;
        const uint32_t R = (uint32_t)(((uint64_t)fi.len + kRowBytes - 1) / kRowBytes);
        rmin = R;
        rmax = R;
        half = fi.len <= (uint32_t)kRowBytes / 2u ? 1u : 0u;
        full = fi.len != 0u && fi.len % (uint32_t)kRowBytes == 0u && ((uintptr_t)fi.addr & 15u) == 0 ? 1u : 0u;
        k12 = fi.len > 1024u && fi.len <= 2048u ? 1u : 0u;
        k1 = fi.len <= 1024u ? 1u : 0u;
        mis = k12 && (((uintptr_t)fi.addr + fi.len) & 15u) != 0 ? 1u : 0u;
    }
    for (int o = 32; o >= 1; o >>= 1) {
        rmin = min(rmin, (uint32_t)__shfl_xor((int)rmin, o));
        rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, o));
        half += (uint32_t)__shfl_xor((int)half, o);
        full += (uint32_t)__shfl_xor((int)full, o);
        mis += (uint32_t)__shfl_xor((int)mis, o);
        k12 += (uint32_t)__shfl_xor((int)k12, o);
        k1 += (uint32_t)__shfl_xor((int)k1, o);
        contig += (uint32_t)__shfl_xor((int)contig, o);
    }
    if (l == 0) {
        volatile BatchShape *r = rec;
        r->sampled = m;
        r->rmin = rmin;
        r->rmax = rmax;
        r->nhalf = half;
        r->nwhole = full;
        r->nmis = mis;
        r->n12k = k12;
        r->n1k = k1;
        r->ncontig = contig;
        r->len0 = f0i.len;
        __threadfence_system();
        r->seq = seq;
    }
}

static bool shapes_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("LAMPI_CSUM_NO_SHAPES");
        return !(e && e[0] == '1');
    }();
    return on;
}

// The rows hint to run this batch with: the caller's, or the one learned from the stream's earlier
// batches of this kind (launching the census for later ones when due).
template <class Src>
static uint32_t learned_rows_hint(const Src &src, size_t n, hipStream_t s, int kind, uint32_t rows_hint,
                                  bool *pairs = nullptr, uint32_t **nhalf_dev = nullptr,
                                  uint32_t min_rows = kShapeRows, bool *one_row = nullptr,
                                  bool *full_rows = nullptr, bool pairs_misaligned_only = false,
                                  bool *all_half = nullptr, bool *all_1k = nullptr, uint32_t *contig_len = nullptr) {
    if (contig_len) *contig_len = 0u;
    if (all_half) *all_half = false;
    if (all_1k) *all_1k = false;
    if (pairs) *pairs = false;
    if (one_row) *one_row = false;
    if (full_rows) *full_rows = false;
    if (rows_hint > 1 || n < kShapeMin || !shapes_enabled()) return rows_hint;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return rows_hint;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return rows_hint;
    ScratchTable::Slot &slot = t_scratch.slots[{dev, s}];
    // this batch's record: the one of its descriptor array, else the least recently used one, reset
    static const bool keyed = [] {  // (A/B knob LAMPI_SHAPES_UNKEYED=1: one record per kind, as in round 4)
        const char *e = LAMPI_AB_ENV("LAMPI_SHAPES_UNKEYED");
        return !(e && e[0] == '1');
    }();
    const void *key = keyed ? (const void *)src.d : nullptr;
    ScratchTable::Slot::ShapeRec *sr = nullptr, *lru = &slot.shapes[0];
    for (auto &r : slot.shapes) {
        if (r.key == key && r.kind == kind) {
            sr = &r;
            break;
        }
        if (r.used < lru->used) lru = &r;
    }
    if (!sr) {
        sr = lru;
        sr->key = key;
        sr->kind = kind;
        sr->calls = 0;
        if (sr->rec) std::memset(sr->rec, 0, sizeof(BatchShape));  // (a census still in flight only costs speed)
    }
    sr->used = ++slot.shape_tick;
    BatchShape *&rec = sr->rec;
    if (!rec) {
        void *p = nullptr;
        if (hipHostMalloc(&p, sizeof(BatchShape), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            (void)hipGetLastError();
            return rows_hint;
        }
        std::memset(p, 0, sizeof(BatchShape));
        rec = (BatchShape *)p;
        g_scratch_bytes.fetch_add((int64_t)sizeof(BatchShape), std::memory_order_relaxed);
    }
    // the last record that landed (seq read before and after the fields: a record being written is skipped)
    const volatile BatchShape *v = rec;
    uint32_t W = rows_hint;
    const uint32_t q0 = v->seq;
    std::atomic_thread_fence(std::memory_order_acquire);  // the fields are read after the first seq ...
    const uint32_t sampled = v->sampled, rmin = v->rmin, rmax = v->rmax, nhalf = v->nhalf, nwhole = v->nwhole,
                   nmis = v->nmis, n12k = v->n12k, n1k = v->n1k, ncontig = v->ncontig, len0 = v->len0;
    std::atomic_thread_fence(std::memory_order_acquire);  // ... and before the second (a seqlock read)
    if (q0 != 0 && v->seq == q0 && sampled > 0) {
        if (rmin >= min_rows && rmax <= 2 * rmin) W = rmax;
        if (one_row && rmin == 1u && rmax == 1u) *one_row = true;  // every sampled fragment one row (17 B-4 KiB)
        // every sampled fragment the same whole number of rows at a 16-byte-aligned address (*full_rows: the
        // rows, W the most rows as above)
        // (the whole-row path lists off-shape fragments through the pair counters: not on a stream whose counters
        // could not be re-zeroed)
        if (full_rows && nwhole == sampled && rmin == rmax && !slot.pair_broken) *full_rows = true;
        if (all_half && nhalf == sampled) *all_half = true;  // every sampled fragment at most 2 KiB
        if (all_1k && n1k == sampled) *all_1k = true;        // ... at most 1 KiB
        // every sampled fragment where one contiguous run of equal fragments puts it (packed rows; the pair counters
        // list the items that are not, so not on a stream whose counters are broken)
        if (contig_len && ncontig == sampled && !slot.pair_broken) *contig_len = len0;
        if (pairs && nhalf == sampled && !slot.pair_broken &&
            (!pairs_misaligned_only || (n12k == sampled && 4 * nmis >= sampled))) {  // every sampled fragment at
            // most 2 KiB: two per wave (read-only: 1-2 KiB each, a quarter or more ending off the 16-byte grid)
            void *dp = nullptr;
            if (nhalf_dev && hipHostGetDevicePointer(&dp, rec, 0) == hipSuccess) {
                *pairs = true;
                *nhalf_dev = &((BatchShape *)dp)->nhalf;
            } else {
                (void)hipGetLastError();
            }
        }
    }
    const uint32_t c = sr->calls++;
    if (c % kShapeEvery == 0) {
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, rec, 0) == hipSuccess) {
            hipLaunchKernelGGL(census_kernel<Src>, dim3(1), dim3(64), 0, s, src, n, (BatchShape *)dp, c + 1);
            (void)hipGetLastError();
        } else {
            (void)hipGetLastError();
        }
    }
    return W;
}

template <bool kSum, int kWv, int kCap>
static hipError_t launch_planned(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img,
                                 hipStream_t s) {
    // byte windows at most: ~4 workgroups per resident slot for large batches, fewer for small ones
    // (every window the plan cannot fill is a workgroup that starts and exits)
    const uint32_t gb = (uint32_t)std::min<size_t>(2048, std::max<size_t>(64, 16 * n));
    const size_t cap = n + gb;                                                            // segments at most
    const size_t gmax = 2 + (cap + kPlanF - 1) / kPlanF + gb;                             // workgroups at most
    const size_t seg_bytes = (cap * sizeof(SegDesc) + 255) & ~(size_t)255;
    uint8_t *scratch = nullptr;
    bool pooled = false;
    hipError_t e = stream_scratch(s, seg_bytes + (gmax + 2) * sizeof(uint32_t), (void **)&scratch, &pooled);
    if (e != hipSuccess) return e;
    SegDesc *segs = (SegDesc *)scratch;
    uint32_t *plan = (uint32_t *)(scratch + seg_bytes);
    if (n <= 64)
        hipLaunchKernelGGL((plan_kernel<64, 64>), dim3(1), dim3(64), 0, s, d, (uint32_t)n, kSum ? 1 : 0, gb, segs,
                           plan, out);
    else if (n <= 2048)
        hipLaunchKernelGGL((plan_kernel<256, 2048>), dim3(1), dim3(256), 0, s, d, (uint32_t)n, kSum ? 1 : 0, gb, segs,
                           plan, out);
    else
        hipLaunchKernelGGL((plan_kernel<1024, kPlanMax>), dim3(1), dim3(1024), 0, s, d, (uint32_t)n, kSum ? 1 : 0, gb,
                           segs, plan, out);
    e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL((crc_stream_kernel<SegSource, kStreamD, kStreamK, kSum, kWv, kCap>), dim3((unsigned)gmax),
                           dim3(64 * kWv), 0, s, SegSource{segs, d}, cap, 0u, img, out, (const uint32_t *)plan);
        e = hipGetLastError();
    }
    return scratch_done(s, scratch, pooled, e);
}

// LAMPI_CSUM_ROWS_HINT(r) on a read-only descriptor batch (fragments of about r rows): the count split
// sizes workgroups by that length (spread_fpw, as for messages: 16,404 x 65,456 B in workgroups of 6,
// not 48), and fragments longer than kSegRows rows run as W = ceil(r / kSegRows) row segments each
// (RowSegSource, out zeroed first: split fragments accumulate into it) -- segments of ~64 KiB, so the
// per-segment join (a constant-product shift past the later rows) stays small against its rows.
constexpr uint32_t kSegRows = 16;
constexpr uint32_t kLightDescRows = 8;  // read-only CRC with LAMPI_CSUM_ROWS_HINT(r >= 8): table-light kernel
constexpr uint32_t kLightRoRows = 8;
template <bool kSum, int kWv, int kCap>
static hipError_t launch_row_segments(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img,
                                      hipStream_t s, uint32_t rows_hint) {
    const uint32_t W = (rows_hint + kSegRows - 1) / kSegRows;
    if (W <= 1) {
        const size_t frag = (size_t)rows_hint * kRowBytes;
        const uint32_t fpg = kSum ? sum_frags_per_wg(n, frag) : frags_per_wg(n, frag);
        hipLaunchKernelGGL((crc_stream_kernel<DescSource, kStreamD, kStreamK, kSum, kWv, kCap>), frags_grid(n, fpg),
                           dim3(64 * kWv), 0, s, DescSource{d}, n, fpg, img, out, nullptr);
        return hipGetLastError();
    }
    const hipError_t e = hipMemsetAsync(out, 0, n * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const size_t items = n * W, seg = (size_t)kSegRows * kRowBytes;
    const uint32_t fpg = kSum ? sum_frags_per_wg(items, seg) : frags_per_wg(items, seg);
    hipLaunchKernelGGL((crc_stream_kernel<RowSegSource, kStreamD, kStreamK, kSum, kWv, kCap>), frags_grid(items, fpg),
                       dim3(64 * kWv), 0, s, RowSegSource{d, W, kSum ? 1 : 0}, items, fpg, img, out, nullptr);
    return hipGetLastError();
}

// The two-launch size split for read-only CRC descriptor batches without a hint (SplitDescSource), for
// batches of kSplitMin..kSplitMax fragments.  Same box (profiles/r04/split_ab.txt): 16,404 x 65,456 B
// 55.6 -> 75.7-76.5%, 16,404 x 40,000 B 54 -> 72-75%, config C and 1 MiB fragments unchanged (outside /
// not of the light class).  The light launch costs a dead workgroup per four fragments of the other class
// (a vote before the table staging): 4,096 x 4 KiB 10.2 -> 12.8 us per call, 65,536 x 4 KiB 52.6 -> 71 us;
// so smaller batches (latency) and larger ones (config C's 659,114 fragments: 74.6 -> 40.9%, its 8-16-row
// fragments run on the light kernel only after the piece streams) keep one launch.  Running the two
// launches concurrently on a forked stream measured worse (GM 67-68%).
constexpr size_t kSplitMin = 1024, kSplitMax = 65536;

// Read-only CRC descriptor batches the census saw as equal whole-row fragments (R rows) at 16-byte-aligned
// addresses: crc_regular_kernel<kDesc> on config B's schedule -- 4 KiB fragments in pairs (two chains per
// wave, each reading a pair in turn; an odd last fragment on the table-light kernel), longer ones one per
// chain row by row -- the items holding any other fragment listed by the kernel and checksummed by
// crc_light_pair_leftover_kernel (the pair kernel's counters and leftover launch).
constexpr size_t kRegDescMinPairs = 2048;
constexpr size_t kPackedMinRows = 256;
constexpr size_t kSumRow4kMinRows = 256;  // sum_row4k_kernel: smaller messages keep the other schedules  // packed rows: smaller batches keep the other schedules (one launch)
static uint32_t pick_regular_fpw(size_t n, size_t span);
static hipError_t launch_crc_desc_whole(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img,
                                        hipStream_t s, uint32_t R) {
    const size_t items = R == 1 ? n / 2 : n;  // pairs of 4 KiB fragments, or fragments
    const size_t span = R == 1 ? 2 * kRowBytes : (size_t)R * kRowBytes;
    if (items > 0xFFFFFFFFull) return hipErrorInvalidValue;
    static const uint32_t fpw_env = [] {  // (A/B knob LAMPI_DESC_FPW: items per wave)
        const char *e = LAMPI_AB_ENV("LAMPI_DESC_FPW");
        return e ? (uint32_t)std::atoi(e) : 0u;
    }();
    uint32_t fpw = pick_regular_fpw(items, span);
    if (fpw_env) {
        fpw = fpw_env;
        while (fpw > 1 && (size_t)kWaves * fpw * 512 > items) fpw >>= 1;
    }
    if (fpw > (R == 1 ? 32u : 64u)) return hipErrorInvalidValue;  // (a wave's descriptors live in its 64 lanes)
    uint32_t *list = nullptr, *left = nullptr, *next_left = nullptr;
    bool pooled = false;
    hipError_t e = stream_scratch(s, (items + 1) * sizeof(uint32_t), (void **)&list, &pooled);
    if (e != hipSuccess) return e;
    e = pair_counters(s, &left, &next_left);
    if (e != hipSuccess) return scratch_done(s, list, pooled, e);
    if (R == 1)
        hipLaunchKernelGGL((crc_regular_kernel<kRegularChains, false, false, 3, 2, false, kWaves, 0, true>),
                           grid_for(items, fpw), dim3(kBlock), 0, s, reinterpret_cast<const uint8_t *>(d),
                           (uint32_t)items, fpw, span, 0u, img, out, nullptr, (size_t)0, list, left);
    else
        hipLaunchKernelGGL((crc_regular_kernel<kRegularChains, false, false, 3, 1, false, kWaves, 0, true>),
                           grid_for(items, fpw), dim3(kBlock), 0, s, reinterpret_cast<const uint8_t *>(d),
                           (uint32_t)items, fpw, span, 0u, img, out, nullptr, (size_t)0, list, left);
    e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(crc_light_pair_leftover_kernel<DescSource>, dim3(kLeftoverWgs), dim3(256), 0, s,
                           DescSource{d}, n, img, out, (const uint32_t *)left, next_left, (const uint32_t *)list,
                           (uint32_t *)nullptr);
        e = hipGetLastError();
    }
    if (e != hipSuccess) reset_pair_counters(s);
    e = scratch_done(s, list, pooled, e);
    if (e == hipSuccess && R == 1 && (n & 1u))
        e = launch_crc_light_frag_copy(DescSource{d + n - 1}, 1, img, out + n - 1, s);
    return e;
}

// Read-only CRC descriptor batches the census saw as one contiguous run of equal L-byte fragments (L = 64 B .. 2 KiB,
// a power of two; config A's shape as descriptors): the message's packed rows (crc_regular_kernel<kSub>) over the
// whole 8 KiB items from d[0].addr, each wave checking its items' descriptors first; items holding anything else are
// listed by fragment pairs for crc_light_pair_leftover_kernel; the last fragments (past the whole items) on the
// count split.
template <bool kSum, int kSub>
static hipError_t launch_packed_desc_k(const lampi_frag_desc *d, size_t nv, uint32_t *out, const uint32_t *img,
                                       hipStream_t s, uint32_t *list, uint32_t *left) {
    const uint32_t fpw = pick_regular_fpw(nv, 2 * kRowBytes);
    hipLaunchKernelGGL((crc_regular_kernel<kRegularChains, false, false, 3, 2, kSum, kWaves, 0, false, kSub>),
                       grid_for(nv, fpw), dim3(kBlock), 0, s, (const uint8_t *)nullptr, (uint32_t)nv, fpw,
                       2 * kRowBytes, 0u, img, out, (uint8_t *)const_cast<lampi_frag_desc *>(d), (size_t)0, list, left);
    return hipGetLastError();
}
template <bool kSum>
static hipError_t launch_desc_packed(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img,
                                     hipStream_t s, uint32_t L, size_t *done) {
    *done = 0;
    const size_t F = 2 * kRowBytes / L, nv = n / F;
    if (nv * 2 < kPackedMinRows || nv > 0xFFFFFFFFull || nv * F / 2 > 0xFFFFFFFFull) return hipSuccess;
    uint32_t *list = nullptr, *left = nullptr, *next_left = nullptr;
    bool pooled = false;
    hipError_t e = stream_scratch(s, (nv * F / 2 + 1) * sizeof(uint32_t), (void **)&list, &pooled);
    if (e != hipSuccess) return e;
    e = pair_counters(s, &left, &next_left);
    if (e != hipSuccess) return scratch_done(s, list, pooled, e);
    switch (L) {
        case 64: e = launch_packed_desc_k<kSum, 1>(d, nv, out, img, s, list, left); break;
        case 128: e = launch_packed_desc_k<kSum, 2>(d, nv, out, img, s, list, left); break;
        case 256: e = launch_packed_desc_k<kSum, 4>(d, nv, out, img, s, list, left); break;
        case 512: e = launch_packed_desc_k<kSum, 8>(d, nv, out, img, s, list, left); break;
        case 1024: e = launch_packed_desc_k<kSum, 16>(d, nv, out, img, s, list, left); break;
        default: e = launch_packed_desc_k<kSum, 32>(d, nv, out, img, s, list, left); break;
    }
    if (e == hipSuccess) {
        if constexpr (kSum)
            hipLaunchKernelGGL(sum_pair_leftover_kernel, dim3(kLeftoverWgs), dim3(256), 0, s, d, nv * F, out,
                               (const uint32_t *)left, next_left, (const uint32_t *)list);
        else
            hipLaunchKernelGGL(crc_light_pair_leftover_kernel<DescSource>, dim3(kLeftoverWgs), dim3(256), 0, s,
                               DescSource{d}, nv * F, img, out, (const uint32_t *)left, next_left,
                               (const uint32_t *)list, (uint32_t *)nullptr);
        e = hipGetLastError();
    }
    if (e != hipSuccess) reset_pair_counters(s);
    e = scratch_done(s, list, pooled, e);
    if (e == hipSuccess) *done = nv * F;
    return e;
}

// SUM descriptor batches of equal 64 B .. 1 KiB fragments (the census saw one contiguous run): sum_row4k_desc_kernel
// over the whole 4 KiB rows' worth of fragments (*done), the leftovers on sum_pair_leftover_kernel.
static hipError_t launch_sum_desc_row4k(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img,
                                        hipStream_t s, uint32_t L, size_t *done) {
    *done = 0;
    const size_t F = kRowBytes / L, nrow = n / F;
    if (nrow < kSumRow4kMinRows || nrow > 0xFFFFFFFFull || nrow * F > 0xFFFFFFFFull) return hipSuccess;
    uint32_t *list = nullptr, *left = nullptr, *next_left = nullptr;
    bool pooled = false;
    hipError_t e = stream_scratch(s, (nrow * F + 1) * sizeof(uint32_t), (void **)&list, &pooled);
    if (e != hipSuccess) return e;
    e = pair_counters(s, &left, &next_left);
    if (e != hipSuccess) return scratch_done(s, list, pooled, e);
    const dim3 g((unsigned)nrow);
    switch (L) {
        case 64: hipLaunchKernelGGL(sum_row4k_desc_kernel<4>, g, dim3(128), 0, s, d, img, out, list, left); break;
        case 128: hipLaunchKernelGGL(sum_row4k_desc_kernel<8>, g, dim3(128), 0, s, d, img, out, list, left); break;
        case 256: hipLaunchKernelGGL(sum_row4k_desc_kernel<16>, g, dim3(128), 0, s, d, img, out, list, left); break;
        case 512: hipLaunchKernelGGL(sum_row4k_desc_kernel<32>, g, dim3(128), 0, s, d, img, out, list, left); break;
        default: hipLaunchKernelGGL(sum_row4k_desc_kernel<64>, g, dim3(128), 0, s, d, img, out, list, left); break;
    }
    e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(sum_pair_leftover_kernel, dim3(kLeftoverWgs), dim3(256), 0, s, d, nrow * F, out,
                           (const uint32_t *)left, next_left, (const uint32_t *)list);
        e = hipGetLastError();
    }
    if (e != hipSuccess) reset_pair_counters(s);
    e = scratch_done(s, list, pooled, e);
    if (e == hipSuccess) *done = nrow * F;
    return e;
}

// Read-only descriptor batches under the learned-shape minimum (kShapeMin fragments) without a rows hint.
// The lengths are on the device only: the count split gave a whole fragment to one workgroup (16 x 16 MiB
// 2.3 ms, 1.5% of the roofline; one 64 MiB fragment 3 ms).  Every fragment runs as W row groups instead
// (k = ceil(R / W) rows each, groups past a fragment's rows empty; CRC: the table-light kernel, a workgroup
// of four empty waves leaving before its table staging), W the power of two bringing the launch to ~4,096
// items: 16 x 16 MiB 2,284 -> 60 us (CRC), 1,348 -> 46 us (SUM); 200 x 1 MiB 155 -> 43 / 91 -> 37 us; batches of
// small fragments pay the join launch, 200 x 4 KiB 8.3 -> 11.3 us (tools/microbench/small_batch.py,
// profiles/r05/small_batch_ab.txt).  A shape learned per descriptor array would save that join but a stale
// one-row shape would bring the 100x case back; the caller's LAMPI_CSUM_ROWS_HINT picks the best schedule
// (one 64 MiB fragment: 168 us as groups, 55 us with the hint).  A/B knob LAMPI_SMALL_BATCH = the item
// target (0: the count split).
static uint32_t small_batch_groups(size_t n, hipStream_t s) {
    static const size_t target = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SMALL_BATCH");
        return e ? (size_t)std::atoll(e) : (size_t)4096;
    }();
    // graph captures keep the count split: the groups' scratch would be a pooled allocation inside the graph
    // (bench.py --latency: a replayed one-descriptor call 6.9 -> 32 us)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return 1u;
    uint32_t W = 1;
    while ((size_t)n * W < target && W < 4096u) W <<= 1;
    return W;
}

hipError_t launch_crc_desc(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img, int grid,
                           hipStream_t s, bool plan, uint32_t rows_hint) {  // (defaults: frag_csum_kernels.h)
    (void)grid;
    if (n == 0) return hipSuccess;
    if (plan && n <= kPlanMax) return launch_planned<false, kStreamWv, kStreamCap>(d, n, out, img, s);
    if (rows_hint == 0 && n < kShapeMin) {  // (1: the caller's pieces, count split)
        const uint32_t W = small_batch_groups(n, s);
        if (W > 1) return launch_crc_light_frag_copy(SparseDescSource{{d}}, n, img, out, s, W);
    }
    bool whole = false, pairs = false;
    uint32_t *nhalf = nullptr;
    const uint32_t given = rows_hint;
    // read-only: two fragments per wave only for 1-2 KiB fragments ending off the 16-byte grid (IB's 1,976 B), where
    // the piece streams take their five-load variant (profiles/r05/crc_ro_pairs_ab.txt)
    bool small = false;
    uint32_t contig = 0;
    rows_hint = learned_rows_hint(DescSource{d}, n, s, 0, rows_hint, &pairs, &nhalf, 1u, nullptr, &whole, true, &small,
                                  nullptr, &contig);
    // one contiguous run of equal 64 B .. 2 KiB fragments (a message as descriptors): packed rows, the rest after it
    static const bool packed_desc = [] {  // (A/B knob LAMPI_PACKED_DESC=0: off)
        const char *e = LAMPI_AB_ENV("LAMPI_PACKED_DESC");
        return !(e && e[0] == '0');
    }();
    if (packed_desc && contig >= 64 && contig <= kRowBytes / 2 && (contig & (contig - 1)) == 0) {
        size_t done = 0;
        const hipError_t e = launch_desc_packed<false>(d, n, out, img, s, contig, &done);
        if (e != hipSuccess) return e;
        if (done) return done >= n ? hipSuccess : launch_crc_desc(d + done, n - done, out + done, img, grid, s, false, 1u);
    }
    static const bool ro_pairs = [] {  // (A/B knob LAMPI_CRC_RO_PAIRS=0: read-only IB-sized batches on the piece streams)
        const char *e = LAMPI_AB_ENV("LAMPI_CRC_RO_PAIRS");
        return !(e && e[0] == '0');
    }();
    if (pairs && ro_pairs) return launch_crc_light_pair_copy(DescSource{d}, n, img, out, s, nhalf);
    // batches of equal whole-row fragments of 1-7 rows on the regular kernel (profiles/r05/crc_desc_pairs_ab.txt:
    // 4 KiB 76.4-77.8 -> 80.3-80.4%, 8 KiB 74.3 -> 77.8%, 16 KiB 74.7 -> 79.2%, 28 KiB 70.4 -> 75.4%; from 8 rows
    // the table-light kernel stays ahead, 32 KiB 81 against 73%, 64 KiB 80 against 67%).  A/B knob
    // LAMPI_CRC_DESC_REGULAR = the most rows taken (0: never).
    static const uint32_t reg_desc = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_CRC_DESC_REGULAR");
        return e ? (uint32_t)std::atoi(e) : 7u;
    }();
    if (whole && rows_hint >= 1u && rows_hint <= reg_desc && n >= 2 * kRegDescMinPairs)
        return launch_crc_desc_whole(d, n, out, img, s, rows_hint);
    if (given <= 1 && rows_hint < kShapeRows) rows_hint = given;  // (learned hints under 8 rows: as before)
    if (rows_hint >= kLightDescRows)  // one wave per kSegRows rows of a fragment, read-only
        return launch_crc_light_frag_copy(DescSource{d}, n, img, out, s,
                                          rows_hint <= kSegRows ? 1u : (rows_hint + kLightRoRows - 1) / kLightRoRows);
    if (rows_hint > 1 && n * ((rows_hint + kSegRows - 1) / kSegRows) <= 0xFFFFFFFFull)
        return launch_row_segments<false, kStreamWv, kStreamCap>(d, n, out, img, s, rows_hint);
    if (n >= kSplitMin && n <= kSplitMax && !small) {  // both size classes, one launch each (SplitDescSource)
        const uint32_t fpg = frags_per_wg(n);
        hipLaunchKernelGGL((crc_stream_kernel<SplitDescSource<false>, kStreamD, kStreamK, false, kStreamWv, kStreamCap>),
                           frags_grid(n, fpg), dim3(64 * kStreamWv), 0, s, SplitDescSource<false>{d}, n, fpg, img, out,
                           nullptr);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        return launch_crc_light_frag_copy(SplitDescSource<true>{d}, n, img, out, s, 1u);
    }
    // batches of fragments of at most 2 KiB: the most fragments per workgroup, 256 (the table staging over more
    // fragments; profiles/r05/stream_fpg_ab.txt: 64 B 5.4 -> 13.0%, 256 B 17.9 -> 36.3%, 1 KiB 50.8 -> 64.1%)
    const uint32_t fpg = small && kFragsPerWg >= 256 && n / 256 >= 256 ? 256u : frags_per_wg(n);
    hipLaunchKernelGGL((crc_stream_kernel<DescSource, kStreamD, kStreamK, false, kStreamWv, kStreamCap>),
                       frags_grid(n, fpg), dim3(64 * kStreamWv), 0, s, DescSource{d}, n, fpg, img, out, nullptr);
    return hipGetLastError();
}

// Timeline diagnostic of the read-only CRC piece streams (tools/microbench/stream_timeline.py): the
// product's grid and schedule, the kDiag instantiation stamping 16 words per workgroup into `stamps`
// (>= 16 * workgroups words); returns the workgroup count in *nwg.  Not on any product path.
hipError_t diag_stream_timeline(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img,
                                uint64_t *stamps, hipStream_t s, uint32_t *nwg) {
    const uint32_t fpg = frags_per_wg(n);
    const dim3 wgs = frags_grid(n, fpg);
    *nwg = wgs.x;
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_stream_diag), &stamps, sizeof(stamps), 0,
                                          hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((crc_stream_kernel<DescSource, kStreamD, kStreamK, false, kStreamWv, kStreamCap, true>), wgs,
                       dim3(64 * kStreamWv), 0, s, DescSource{d}, n, fpg, img, out, nullptr);
    return hipGetLastError();
}

// Timeline diagnostic of config B's kernel (tools/microbench/regular_timeline.py): a read-only CRC message of 4 KiB
// fragments on launch_regular's grid and schedule (pairs, pick_regular_fpw), the kDiag instantiation stamping 16
// words per workgroup into `stamps`; returns the workgroup count in *nwg.  Not on any product path.
hipError_t diag_regular_timeline(const uint8_t *base, size_t n, uint32_t *out, const uint32_t *img, uint64_t *stamps,
                                 hipStream_t s, uint32_t *nwg) {
    const size_t nv = n / 2;
    if (nv == 0 || (n & 1u) || nv > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const uint32_t fpw = pick_regular_fpw(nv, 2 * kRowBytes);
    const dim3 g = grid_for(nv, fpw);
    *nwg = g.x;
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_stream_diag), &stamps, sizeof(stamps), 0,
                                          hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((crc_regular_kernel<kRegularChains, false, false, 3, 2, false, kWaves, 0, false, 64, true>), g,
                       dim3(kBlock), 0, s, base, (uint32_t)nv, fpw, (size_t)2 * kRowBytes, 0xFFFFFFFFu, img, out,
                       nullptr, (size_t)0);
    return hipGetLastError();
}

// The north_star's one-wavefront-per-fragment schedule for descriptor batches (hard
// part 3: reported beside the piece streams): crc_rows_kernel (a wave walks its fragments row by
// row, one row prefetched) / sum_rows_kernel.
hipError_t launch_desc_per_wave(const lampi_frag_desc *d, size_t n, uint32_t *out, int mode, const uint32_t *img,
                                hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t fpw = pick_fpw(n, 1);
    if (mode == LAMPI_CSUM_CRC32)
        hipLaunchKernelGGL((crc_rows_kernel<DescSource>), grid_for(n, fpw), dim3(kBlock), 0, s, DescSource{d}, n, fpw,
                           img, out);
    else
        hipLaunchKernelGGL(sum_rows_kernel<DescSource>, grid_for(n, fpw), dim3(kBlock), 0, s, DescSource{d}, n, fpw,
                           out);
    return hipGetLastError();
}

template <bool kSum>
static hipError_t launch_packed(const uint8_t *base, size_t msg_len, size_t frag_len, uint32_t partial, uint32_t *out,
                                const uint32_t *img, hipStream_t s, size_t *done);

hipError_t launch_crc_msg(const uint8_t *base, size_t msg_len, size_t frag_len, uint32_t partial, size_t n,
                          uint32_t *out, const uint32_t *img, int grid, hipStream_t s) {
    (void)grid;
    if (n == 0) return hipSuccess;
    // the read-only table-light kernel (tools/microbench/msg_light.py, profiles/r03/msg_light_ab.txt):
    // fragments of 8-16 rows (GM's 65,456-byte payloads, 64 KiB) one wave each -- 4 GiB of 64 KiB
    // fragments 67.7 -> 78.4%, of 65,456 B 76.9 -> 78.3% -- and longer ones as 8-row groups joined.
    // Since round 5 at every message length (profiles/r05/crc_light_msg_ab.txt): 4 GiB messages of
    // 128 KiB-2 MiB fragments on the regular kernel 73-74 -> 80.7-83.4%, 4 MiB 40.9 -> 80.7%, 16 MiB
    // 10.5 -> 80.9% (the regular kernel's chains are fragments: 256 of them starve the grid), and of
    // non-whole-row 65,552-131,056 B on the framed regular kernel (removed) 71-76.5 -> 76-82%.
    // fragments of 64 B .. 2 KiB (powers of two) in packed rows of config B's kernel; the rest of the message
    // (its last fragments) through the schedules below
    static const bool packed = [] {  // (A/B knob LAMPI_PACKED=0: off)
        const char *e = LAMPI_AB_ENV("LAMPI_PACKED");
        return !(e && e[0] == '0');
    }();
    if (packed) {
        size_t done = 0;
        const hipError_t e = launch_packed<false>(base, msg_len, frag_len, partial, out, img, s, &done);
        if (e != hipSuccess || done == 0) {
            if (e != hipSuccess) return e;
        } else {
            if (done >= n) return hipSuccess;
            return launch_crc_msg(base + done * frag_len, msg_len - done * frag_len, frag_len, partial, n - done,
                                  out + done, img, grid, s);
        }
    }
    const size_t R = (frag_len + kRowBytes - 1) / kRowBytes;
    static const bool ro_pairs = [] {  // (A/B knob LAMPI_CRC_RO_PAIRS=0, as launch_crc_desc)
        const char *e = LAMPI_AB_ENV("LAMPI_CRC_RO_PAIRS");
        return !(e && e[0] == '0');
    }();
    if (ro_pairs && frag_len > 1024 && frag_len <= kRowBytes / 2 && (frag_len & 15u) != 0 && n >= kShapeMin &&
        pair_counters_ok(s))
        return launch_crc_light_pair_copy(MsgSource{base, msg_len, frag_len, partial}, n, img, out, s, nullptr);
    if (crc_light_msg(frag_len, msg_len))
        return launch_crc_light_frag_copy(MsgSource{base, msg_len, frag_len, partial}, n, img, out, s,
                                          R <= kSegRows ? 1u : (uint32_t)((R + kLightRoRows - 1) / kLightRoRows));
    // fragments of at most 2 KiB: 256 per workgroup (as launch_crc_desc)
    const uint32_t fpg = frag_len <= kRowBytes / 2 && n / 256 >= 256 ? 256u : frags_per_wg(n, frag_len);
    hipLaunchKernelGGL((crc_stream_kernel<MsgSource, kStreamD, kStreamK, false, kStreamWv, kStreamCap>), frags_grid(n, fpg), dim3(64 * kStreamWv), 0, s,
                       MsgSource{base, msg_len, frag_len, partial}, n, fpg, img, out, nullptr);
    return hipGetLastError();
}

// Read-kernel schedule, measured on MI355X (tools/microbench/crc_sweep.hip, profiles/r01_sweep.txt):
// a workgroup covers ~384 KiB (fpw * span = 96 KiB per wave) and its waves walk fragments row by
// row.  4 KiB fragments are visited in the order of 8 KiB ones (kV = 2: chain c reads two
// consecutive fragments in turn): 81.4-82.4% of the HBM roofline at every batch offset measured
// (0, 4 KiB .. 1.5 MiB) against 79.4-79.8% for the previous fpw = 32 fragment-order schedule and
// 77-79% for the same 384 KiB in fragment order; the 16 KiB order (kV = 4, fpw 6) matched it
// except at a 64 KiB batch offset (79.8%).  16 KiB fragments: fpw 6, 80.3-82.3% (fpw 12: 78.6%).
// fpw stays even (two chains, no duplicate ring slots).
static uint32_t pick_regular_fpw(size_t n, size_t span) {
    uint32_t fpw = (uint32_t)std::max<size_t>(2, (96u * 1024u / span) & ~(size_t)1);
    while (fpw > 1 && (size_t)kWaves * fpw * 512 > n) fpw >>= 1;  // small batches: more workgroups
    return fpw;
}

template <bool kSum>
static hipError_t launch_regular(const uint8_t *base, size_t n, size_t frag_len, uint32_t partial, uint32_t *out,
                                 const uint32_t *img, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;
    constexpr int kV = 2;
    size_t done = 0;
    if (frag_len == (size_t)kRowBytes && n >= (size_t)kV) {
        const size_t nv = n / kV;
        const uint32_t fpw = pick_regular_fpw(nv, kV * frag_len);
        hipLaunchKernelGGL((crc_regular_kernel<kRegularChains, false, false, 3, kV, kSum>), grid_for(nv, fpw),
                           dim3(kBlock), 0, s, base, (uint32_t)nv, fpw, kV * frag_len, partial, img, out, nullptr,
                           (size_t)0);
        done = nv * kV;
        if (done == n) return hipGetLastError();
    }
    const size_t m = n - done;  // fragment-order schedule (and the last n % kV fragments of a 4 KiB batch)
    const uint32_t fpw = pick_regular_fpw(m, frag_len);
    hipLaunchKernelGGL((crc_regular_kernel<kRegularChains, false, false, 3, 1, kSum>), grid_for(m, fpw),
                       dim3(kBlock), 0, s, base + done * frag_len, (uint32_t)m, fpw, frag_len, partial, img, out + done,
                       nullptr, (size_t)0);
    return hipGetLastError();
}

// Packed rows (crc_regular_kernel<kSub < 64>): a message of 64 * kSub-byte fragments (kSub = 1 .. 32: 64 B ..
// 2 KiB) at a 16-byte-aligned base on config B's schedule, 64 / kSub fragments per 4 KiB row, two rows per
// chain item (kV = 2).  Takes the first *done fragments -- whole pairs of rows -- and leaves the rest (fewer
// than 128 / kSub plus the message's last, possibly short, fragment) to the caller.
template <bool kSum, int kSub>
static hipError_t launch_packed_k(const uint8_t *base, size_t nv, uint32_t partial, uint32_t *out, const uint32_t *img,
                                  hipStream_t s) {
    static const uint32_t fpw_env = [] {  // (A/B knob LAMPI_PACKED_FPW: items per wave)
        const char *e = LAMPI_AB_ENV("LAMPI_PACKED_FPW");
        return e ? (uint32_t)std::atoi(e) : 0u;
    }();
    // (config B's choice, 12 items per wave; 1 GiB of 1 KiB fragments: 16 items 71.4%, 8 70.6%, 6 70.5-70.9%, 4 66%;
    // a balanced grid of whole rounds of resident workgroups 68.6-71.1%, profiles/r06/packed_fpw.txt; a tapered grid
    // ending on 512-2,048 workgroups of 2-6 items 68-72%, profiles/r06/packed_taper.txt)
    const uint32_t fpw = fpw_env ? fpw_env : pick_regular_fpw(nv, 2 * kRowBytes);
    hipLaunchKernelGGL((crc_regular_kernel<kRegularChains, false, false, 3, 2, kSum, kWaves, 0, false, kSub>),
                       grid_for(nv, fpw), dim3(kBlock), 0, s, base, (uint32_t)nv, fpw, 2 * kRowBytes, partial, img, out,
                       nullptr, (size_t)0);
    return hipGetLastError();
}
template <bool kSum>
static hipError_t launch_packed(const uint8_t *base, size_t msg_len, size_t frag_len, uint32_t partial, uint32_t *out,
                                const uint32_t *img, hipStream_t s, size_t *done) {
    *done = 0;
    if (((uintptr_t)base & 15u) != 0 || frag_len < 64 || frag_len > kRowBytes / 2 || (frag_len & (frag_len - 1)) != 0)
        return hipSuccess;
    const size_t rows = msg_len / kRowBytes, nv = rows / 2;  // whole 8 KiB items: every fragment in them is full
    if (rows < kPackedMinRows || nv > 0xFFFFFFFFull) return hipSuccess;
    hipError_t e = hipErrorInvalidValue;
    switch (frag_len) {
        case 64: e = launch_packed_k<kSum, 1>(base, nv, partial, out, img, s); break;
        case 128: e = launch_packed_k<kSum, 2>(base, nv, partial, out, img, s); break;
        case 256: e = launch_packed_k<kSum, 4>(base, nv, partial, out, img, s); break;
        case 512: e = launch_packed_k<kSum, 8>(base, nv, partial, out, img, s); break;
        case 1024: e = launch_packed_k<kSum, 16>(base, nv, partial, out, img, s); break;
        case 2048: e = launch_packed_k<kSum, 32>(base, nv, partial, out, img, s); break;
        default: return hipSuccess;
    }
    if (e == hipSuccess) *done = nv * 2 * (kRowBytes / frag_len);
    return e;
}

hipError_t launch_crc_regular(const uint8_t *base, size_t n, size_t frag_len, uint32_t partial, uint32_t *out,
                              const uint32_t *img, int grid, hipStream_t s) {
    (void)grid;
    return launch_regular<false>(base, n, frag_len, partial, out, img, s);
}

hipError_t launch_crc_regular_copy(const uint8_t *base, size_t n, size_t frag_len, uint32_t partial, uint8_t *dst,
                                   size_t dst_stride, uint32_t *out, const uint32_t *img, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;
// fused CRC copies: half the read-only kernels' fragments per wave (same-box A/B,
// profiles/r02_crc_copy_fpw/: message 69.8 -> 72.2%, descriptors 72.1 -> 74.4%, +8 sources
// 71.8 -> 74.2%, +8 destinations 67.4 -> 69.5-70.4%, the receive step 71.2 -> 72%; a quarter:
// about the same, +1 destinations 2 points lower; twice: no change; 3/4: 2 points lower)
    const uint32_t fpw = std::max(1u, pick_fpw(n, (uint32_t)(frag_len / kRowBytes)) / 2);  // half the read kernel's
    // (one chain per wave and / or a two-deep ring: within a point of this, profiles/r02_crc_copy_fpw/chains/)
    hipLaunchKernelGGL((crc_regular_kernel<kRegularChains, true>), grid_for(n, fpw), dim3(kBlock), 0, s, base,
                       (uint32_t)n, fpw, frag_len, partial, img, out, dst, dst_stride);
    return hipGetLastError();
}

// Fused-copy SUM (bcopy_uicsum, LA-MPI's default mode): sum_copy_wg_kernel, one short-lived
// workgroup per fragment (the textbook copy shape).
template <class Src>
static void launch_sum_copy(const Src &src, size_t n, uint32_t *out, hipStream_t s, bool small = false) {
    if (small)
        hipLaunchKernelGGL(sum_copy_waves_kernel<Src>, dim3((unsigned)std::min<size_t>((n + 3) / 4, kMaxWgGrid)),
                           dim3(256), 0, s, src, n, out);
    else
        hipLaunchKernelGGL(sum_copy_wg_kernel<Src>, dim3((unsigned)std::min<size_t>(n, kMaxWgGrid)), dim3(kSumWgThreads),
                           0, s, src, n, out);
}

// With LAMPI_CSUM_ROWS_HINT (W > 1): each fragment as W row-group workgroups, their sums joined.
static uint32_t sum_groups(size_t n, uint32_t W) {
    while (W > 1 && (size_t)n * W > ((size_t)1 << 31)) W >>= 1;
    return W;
}

template <class Src>
static hipError_t launch_sum_copy_groups(const Src &src, size_t n, uint32_t *out, hipStream_t s, uint32_t W,
                                         bool small = false) {
    W = sum_groups(n, W);
    if (W <= 1) {
        launch_sum_copy(src, n, out, s, small);
        return hipGetLastError();
    }
    uint32_t *groups = nullptr;
    bool pooled = false;
    hipError_t e = stream_scratch(s, n * W * sizeof(uint32_t), (void **)&groups, &pooled);
    if (e != hipSuccess) return e;
    // (128 threads per group measured against 256 -- GM receive 72.5 -> 63% -- and a wave per group, four to a
    // workgroup -- 72.5 -> 62.4%)
    // (two or four groups per workgroup, grid-stride: GM receive 72.5 -> 71.2 / 69.6%)
    launch_sum_copy(GroupSource<Src>{src, W}, n * W, groups, s);
    e = hipGetLastError();
    if (e == hipSuccess) {
        uint32_t G = 1;
        while (G < W && G < 64u) G <<= 1;
        hipLaunchKernelGGL(sum_group_join_kernel<Src>, dim3((unsigned)((n * G + 255) / 256)), dim3(256), 0, s, src, n, W,
                           G, groups, out);
        e = hipGetLastError();
    }
    return scratch_done(s, groups, pooled, e);
}

// SUM message copies of fragments of R rows: the row groups to run (1: sum_copy_row_kernel's row items).
// Row groups of one row each (GroupSource<MsgCopySource> on sum_copy_wg_kernel, joined by
// sum_group_join_kernel) instead of row items whose sums meet in one atomicAdd per row on the fragment's
// word -- 256+ same-address atomics per fragment serialize at L2 -- for fragments of whole rows and for any
// of >= 64 rows (profiles/r05/sum_msg_copy_ab.txt): 16 KiB 77.4 -> 79.9%, 128 KiB 76.7 -> 79.5%, 512 KiB
// 65.7 -> 79.2%, 1 MiB 60.2 -> 78.7%, 4 MiB 49.0 -> 76.0%, 16 MiB 32.2 -> 67%.  GM's 65,456-byte fragments
// (rows off the 16-byte grid) stay on the row items (77.2% against 71.3%).  A/B knobs LAMPI_SUM_CP_GRP_MIN
// (fewest rows for fragments that are not whole rows, 0 = never groups), LAMPI_SUM_CP_GRP_ROWS (rows per group).
static uint32_t sum_copy_groups(uint32_t R, bool whole_rows) {
    static const uint32_t grp_min = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_CP_GRP_MIN");
        return e ? (uint32_t)std::atoi(e) : 64u;
    }();
    static const uint32_t grp_rows = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_CP_GRP_ROWS");
        return e ? (uint32_t)std::max(1, std::atoi(e)) : 1u;
    }();
    if (!grp_min || R < 2 || (!whole_rows && R < grp_min)) return 1u;
    return (R + grp_rows - 1) / grp_rows;
}


hipError_t launch_bcopy_desc(const lampi_copy_desc *d, size_t n, uint32_t *out, int mode, const uint32_t *img,
                             hipStream_t s, uint32_t rows_hint) {
    if (n == 0) return hipSuccess;
    if (!img) return hipErrorInvalidValue;  // the tables (CRC)
    bool pairs = false;
    uint32_t *nhalf = nullptr;
    if (mode == LAMPI_CSUM_NONE) {  // copies only (out: the caller's scratch), the SUM copy schedules
        rows_hint = learned_rows_hint(CopyOnlySource{d}, n, s, 3, rows_hint, &pairs, &nhalf, kShapeRowsSum);
        return launch_sum_copy_groups(CopyOnlySource{d}, n, out, s, rows_hint, pairs);
    }
    const bool crc = mode == LAMPI_CSUM_CRC32;
    uint32_t contig = 0;
    const uint32_t given = rows_hint;
    rows_hint = learned_rows_hint(CopySource{d}, n, s, 1, rows_hint, &pairs, &nhalf, crc ? kShapeRows : kShapeRowsSum,
                                  nullptr, nullptr, false, nullptr, nullptr, &contig);
    // SUM copies of equal 64 B .. 1 KiB fragments: one short-lived workgroup per 4 KiB of them (sum_row4k_copy_desc_kernel),
    // the rest after them.  Same box, interleaved (profiles/r06/sum_row4k_cd_ab.txt), of read + write: 1 KiB 69.0 ->
    // 77.3%, 256 B 23.7 -> 77.7%, 64 B 6.9 -> 63.0% (to + 8 / + 1 destinations 58-74%).  A/B knob
    // LAMPI_SUM_ROW4K_COPY_DESC=0: off
    static const bool row4k_cd = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_ROW4K_COPY_DESC");
        return !(e && e[0] == '0');
    }();
    if (!crc && row4k_cd && given <= 1 && contig >= 64 && contig <= 1024 && (contig & (contig - 1)) == 0) {
        const size_t F = kRowBytes / contig, nrow = n / F;
        if (nrow >= kSumRow4kMinRows && nrow * F <= 0xFFFFFFFFull) {
            uint32_t *list = nullptr, *left = nullptr, *next_left = nullptr;
            bool pooled = false;
            hipError_t e = stream_scratch(s, (nrow * F + 1) * sizeof(uint32_t), (void **)&list, &pooled);
            if (e != hipSuccess) return e;
            e = pair_counters(s, &left, &next_left);
            if (e != hipSuccess) return scratch_done(s, list, pooled, e);
            const dim3 g((unsigned)nrow);
            switch (contig) {
                case 64: hipLaunchKernelGGL(sum_row4k_copy_desc_kernel<4>, g, dim3(128), 0, s, d, img, out, list, left); break;
                case 128: hipLaunchKernelGGL(sum_row4k_copy_desc_kernel<8>, g, dim3(128), 0, s, d, img, out, list, left); break;
                case 256: hipLaunchKernelGGL(sum_row4k_copy_desc_kernel<16>, g, dim3(128), 0, s, d, img, out, list, left); break;
                case 512: hipLaunchKernelGGL(sum_row4k_copy_desc_kernel<32>, g, dim3(128), 0, s, d, img, out, list, left); break;
                default: hipLaunchKernelGGL(sum_row4k_copy_desc_kernel<64>, g, dim3(128), 0, s, d, img, out, list, left); break;
            }
            e = hipGetLastError();
            if (e == hipSuccess) {
                hipLaunchKernelGGL(sum_copy_list_kernel, dim3(kLeftoverWgs), dim3(128), 0, s, d, (const uint32_t *)left,
                                   next_left, (const uint32_t *)list, out);
                e = hipGetLastError();
            }
            if (e != hipSuccess) reset_pair_counters(s);
            e = scratch_done(s, list, pooled, e);
            if (e != hipSuccess) return e;
            const size_t done = nrow * F;
            return done >= n ? hipSuccess : launch_bcopy_desc(d + done, n - done, out + done, mode, img, s, 1u);
        }
    }
    if (crc && pairs) return launch_crc_light_pair_copy(CopySource{d}, n, img, out, s, nhalf);
    if (crc) return launch_crc_light_frag_copy(CopySource{d}, n, img, out, s, rows_hint);
    return launch_sum_copy_groups(CopySource{d}, n, out, s, rows_hint, pairs);  // (pairs: a wave per fragment)
}

// The receive step's mask words and bad count, zeroed in one launch (two memsets were two ~5 us stream
// operations per call, 2.5% of a GiB of GM receives)
__global__ void __launch_bounds__(256) zero_verdicts_kernel(uint32_t *__restrict__ mask, size_t nwords,
                                                            uint32_t *__restrict__ nbad) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < nwords) mask[i] = 0u;
    if (i == 0) *nbad = 0u;
}

hipError_t launch_copy_to_app(const lampi_recv_desc *d, size_t n, const uint8_t *expected, size_t exp_stride,
                              int64_t *copied, uint32_t *csum, uint32_t *mask, uint32_t *nbad, int mode,
                              const uint32_t *img, hipStream_t s, uint32_t rows_hint) {
    if (n == 0) return hipMemsetAsync(nbad, 0, sizeof(uint32_t), s);
    if (!img) return hipErrorInvalidValue;
    const bool crc = mode == LAMPI_CSUM_CRC32;
    const RecvSource src{d, crc ? 0xFFFFFFFFu : 0u, expected, exp_stride, copied, mask, nbad};
    if (mode == LAMPI_CSUM_NONE) {  // copy only, every fragment DataOK: the SUM copy schedules without the sums
        const size_t nwords = (n + 31) / 32;
        hipLaunchKernelGGL(zero_verdicts_kernel, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, s, mask, nwords,
                           nbad);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        RecvCopyOnlySource co;
        static_cast<RecvSource &>(co) = src;
        bool small = false;  // (fragments of at most 2 KiB: a wave each, as SUM)
        uint32_t *nh = nullptr;
        rows_hint = learned_rows_hint(co, n, s, 2, rows_hint, &small, &nh, kShapeRowsSum);
        return launch_sum_copy_groups(co, n, csum, s, rows_hint, small);
    }
    bool pairs = false;
    uint32_t *nhalf = nullptr;
    rows_hint = learned_rows_hint(src, n, s, 2, rows_hint, &pairs, &nhalf, crc ? kShapeRows : kShapeRowsSum);
    // row groups: the first launch zeroes the verdicts (zero_verdict_words), the join gives them; otherwise
    // the fragments' own waves give them, after this
    const bool groups = crc ? !pairs && light_groups(n, rows_hint) > 1 : sum_groups(n, rows_hint) > 1;
    if (!groups) {
        const size_t nwords = (n + 31) / 32;
        hipLaunchKernelGGL(zero_verdicts_kernel, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, s, mask, nwords,
                           nbad);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (crc && pairs) return launch_crc_light_pair_copy(src, n, img, csum, s, nhalf);
    if (crc) return launch_crc_light_frag_copy(src, n, img, csum, s, rows_hint);
    return launch_sum_copy_groups(src, n, csum, s, rows_hint, pairs);  // (pairs: a wave per fragment)
}

hipError_t launch_sum64_desc(const lampi_frag_desc *d, size_t n, uint64_t *out, bool phased, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t fpw = pick_fpw(n, 1);
    if (phased)
        hipLaunchKernelGGL((sum_rows_kernel<PhaseDescSource, uint64_t>), grid_for(n, fpw), dim3(kBlock), 0, s,
                           PhaseDescSource{d}, n, fpw, out);
    else
        hipLaunchKernelGGL((sum_rows_kernel<DescSource, uint64_t>), grid_for(n, fpw), dim3(kBlock), 0, s, DescSource{d},
                           n, fpw, out);
    return hipGetLastError();
}

hipError_t launch_sum64_finish(const uint64_t *vals, uint32_t nv, const uint8_t *src, uint64_t len, uint64_t plong,
                               uint64_t plen, uint64_t *out3, hipStream_t s, uint64_t *sig, uint64_t seq) {
    hipLaunchKernelGGL(sum64_finish_kernel, dim3(1), dim3(256), 0, s, vals, nv, src, len, plong, plen, out3, sig, seq);
    return hipGetLastError();
}

// Read-only SUM batches of fragments of R > 1 rows (descriptors: the caller's or learned hint; messages:
// the fragment length): 1 = one fragment per short-lived 128-thread workgroup (sum_copy_wg_kernel), W > 1 =
// W row groups per fragment joined by sum_group_join_kernel, ~0u = neither (the row segments).
//  - R <= 8 in batches of >= 4096 fragments: one per workgroup.  Same box, interleaved
//    (profiles/r05/sum_ro_sched_ab.txt), against the piece streams / eight one-row groups before: 8 KiB
//    77.5 -> 88.8%, 16 KiB 76.7 -> 89.1%, 32 KiB 77.4 -> 88.0%.
//  - otherwise min(R, 8) groups, doubled while each group keeps >= 2 rows and the launch has under 65,536
//    workgroups: 1 MiB x 1,024 72.9 -> 83.9%, 2 MiB x 1,024 74.6 -> 83+%, 4 MiB x 2,048 81.1 -> 87.0%,
//    16 MiB x 256 77.1 -> 84.6%; GM's 65,456 B and 1 MiB x 4,096 unchanged (86.5, 85%).  One workgroup
//    per fragment above 8 rows loses wherever the grid needs more than one round of workgroups (512 KiB
//    x 8,192 86.9 -> 75.4%, GM 86.7 -> 84.8%).
//  - fragments over 256 rows were row segments before (2 MiB x 4,096 76.6 -> 84.8% as groups).
// A/B knobs: LAMPI_SUM_RO_ONEWG = fewest fragments for one per workgroup (0: never), LAMPI_SUM_RO_WGS = the
// workgroup target, LAMPI_SUM_RO_GROUPS=0 = the round-4 schedules (groups of <= 8 up to 256 rows, segments above).
static uint32_t sum_ro_groups(size_t n, uint32_t R) {
    static const size_t onewg = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_RO_ONEWG");
        return e ? (size_t)std::atoll(e) : (size_t)4096;
    }();
    static const size_t wgs = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_RO_WGS");
        return e ? (size_t)std::atoll(e) : (size_t)65536;
    }();
    static const bool r5 = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_RO_GROUPS");
        return !(e && e[0] == '0');
    }();
    if (!r5) return R <= 256u && sum_groups(n, min(R, 8u)) > 1 ? min(R, 8u) : 0xFFFFFFFFu;
    if (onewg && R <= 8u && n >= onewg) return 1u;
    uint32_t W = min(R, 8u);
    while (W < R / 2 && (size_t)n * W < wgs) W *= 2;
    W = sum_groups(n, W);
    return W > 1 ? W : 0xFFFFFFFFu;
}

hipError_t launch_sum_desc(const lampi_frag_desc *d, size_t n, uint32_t *out, const uint32_t *img, int grid,
                           hipStream_t s, bool plan, uint32_t rows_hint) {
    (void)grid;
    if (n == 0) return hipSuccess;
    if (img && plan && n <= kPlanMax) return launch_planned<true, kSumWv, kSumCap>(d, n, out, img, s);
    if (img && rows_hint == 0 && n < kShapeMin) {  // (small batches: as launch_crc_desc)
        const uint32_t W = small_batch_groups(n, s);
        if (W > 1) return launch_sum_copy_groups(DescSource{d}, n, out, s, W);
    }
    bool one_row = false;
    bool half = false;  // (every sampled fragment at most 2 KiB)
    uint32_t *nh = nullptr;
    bool tiny = false;  // (every sampled fragment at most 1 KiB)
    uint32_t contig = 0;  // (one contiguous run of equal fragments: their length)
    if (img)
        rows_hint = learned_rows_hint(DescSource{d}, n, s, 0, rows_hint, &half, &nh, 2u, &one_row, nullptr, false,
                                      nullptr, &tiny, &contig);
    // one contiguous run of equal 64 B .. 1 KiB fragments: packed rows, as launch_crc_desc (2 KiB: one per wave reads
    // faster, as for messages)
    static const bool packed_desc = [] {  // (A/B knob LAMPI_PACKED_DESC=0: off, as launch_crc_desc)
        const char *e = LAMPI_AB_ENV("LAMPI_PACKED_DESC");
        return !(e && e[0] == '0');
    }();
    // ... on short-lived 4 KiB workgroups (sum_row4k_desc_kernel; profiles/r06/sum_row4k_desc_ab.txt, against the packed
    // rows: 1 KiB 72.0 -> 79.9%, 256 B 63.6 -> 75.5%, 64 B 50.5-56.0 -> 60.4-64.3%).  A/B knob LAMPI_SUM_ROW4K_DESC=0: off
    static const bool row4k_desc = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_ROW4K_DESC");
        return !(e && e[0] == '0');
    }();
    if (img && row4k_desc && rows_hint <= 1 && contig >= 64 && contig <= 1024 && (contig & (contig - 1)) == 0) {
        size_t done = 0;
        const hipError_t e = launch_sum_desc_row4k(d, n, out, img, s, contig, &done);
        if (e != hipSuccess) return e;
        if (done) return done >= n ? hipSuccess : launch_sum_desc(d + done, n - done, out + done, img, grid, s, false, 1u);
    }
    if (img && packed_desc && rows_hint <= 1 && contig >= 64 && contig <= 1024 && (contig & (contig - 1)) == 0) {
        size_t done = 0;
        const hipError_t e = launch_desc_packed<true>(d, n, out, img, s, contig, &done);
        if (e != hipSuccess) return e;
        if (done) return done >= n ? hipSuccess : launch_sum_desc(d + done, n - done, out + done, img, grid, s, false, 1u);
    }
    static const bool sum_tiny = [] {  // (A/B knob LAMPI_SUM_TINY=0, as launch_sum_msg)
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_TINY");
        return !(e && e[0] == '0');
    }();
    if (img && sum_tiny && tiny && rows_hint <= 1 && n / 256 >= 256) {  // (as launch_sum_msg: 256 per workgroup)
        hipLaunchKernelGGL((crc_stream_kernel<DescSource, kStreamD, kStreamK, true, kSumWv, kSumCap>),
                           frags_grid(n, 256), dim3(64 * kSumWv), 0, s, DescSource{d}, n, 256u, img, out, nullptr);
        return hipGetLastError();
    }
    // batches the census saw as all <= 2 KiB fragments: one fragment per wave, four to a workgroup
    // (sum_copy_waves_kernel, IB's SUM copies' schedule; profiles/r05/sum_ro_waves_ab.txt: 1,976 B 45.5 -> 69.5%,
    // 1 KiB 35.6 -> 64.3%, 2 KiB 58.5 -> 80.4%, 256 B 10.2 -> 20.8%).  A/B knob LAMPI_SUM_RO_WAVES=0: off.
    static const bool ro_waves = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_RO_WAVES");
        return !(e && e[0] == '0');
    }();
    if (img && ro_waves && half && rows_hint <= 1) {
        launch_sum_copy(DescSource{d}, n, out, s, true);
        return hipGetLastError();
    }
    if (img && rows_hint > 1) {
        const uint32_t W = sum_ro_groups(n, rows_hint);
        if (W <= 1) {
            launch_sum_copy(DescSource{d}, n, out, s);
            return hipGetLastError();
        }
        if (W < 0xFFFFFFFFu) return launch_sum_copy_groups(DescSource{d}, n, out, s, W);
    }
    if (img && rows_hint > 1 && n * ((rows_hint + kSegRows - 1) / kSegRows) <= 0xFFFFFFFFull)
        return launch_row_segments<true, kSumWv, kSumCap>(d, n, out, img, s, rows_hint);
    // batches of one-row fragments (the census: every sampled fragment 1-4096 bytes) on short-lived 128-thread
    // workgroups of two fragments each (profiles/r04/sum_ro_wg_ab.txt: 4 KiB descriptors 79.6 -> 86.3%; one per
    // workgroup 83.2%, four 82.7%; config C's mixed sizes lost 0.5 on it and keep the piece streams).  A/B knob
    // LAMPI_SUM_RO_WG = fragments per workgroup (0: off).
    static const uint32_t ro_wg = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_RO_WG");
        return e ? (uint32_t)std::atoi(e) : 2u;
    }();
    if (img && ro_wg && one_row && rows_hint <= 1) {
        hipLaunchKernelGGL(sum_copy_wg_kernel<DescSource>,
                           dim3((unsigned)std::min<size_t>((n + ro_wg - 1) / ro_wg, kMaxWgGrid)), dim3(kSumWgThreads), 0,
                           s, DescSource{d}, n, out);
        return hipGetLastError();
    }
    if (img) {  // piece streams (img: the zero chunk)
        const uint32_t fpg = sum_frags_per_wg(n);
        hipLaunchKernelGGL((crc_stream_kernel<DescSource, kStreamD, kStreamK, true, kSumWv, kSumCap>),
                           frags_grid(n, fpg), dim3(64 * kSumWv), 0, s, DescSource{d}, n, fpg, img, out, nullptr);
        return hipGetLastError();
    }
    const uint32_t fpw = pick_fpw(n, 1);
    hipLaunchKernelGGL(sum_rows_kernel<DescSource>, grid_for(n, fpw), dim3(kBlock), 0, s, DescSource{d}, n, fpw, out);
    return hipGetLastError();
}

hipError_t launch_sum_msg(const uint8_t *base, size_t msg_len, size_t frag_len, size_t n, uint32_t *out,
                          const uint32_t *img, int grid, hipStream_t s) {
    (void)grid;
    if (n == 0) return hipSuccess;
    // Messages of >= 256 fragments on short-lived 128-thread workgroups, one fragment each (sum_copy_wg_kernel,
    // the read-only SUM descriptors' shape: VERDICT r4 item 4), whatever the fragment length.  Same box,
    // interleaved rounds (profiles/r05/sum_msg_ab.txt), against the regular kernel / piece streams: config B
    // (4 KiB) 80.2-80.4 -> 87.1-87.3% (two fragments per workgroup 83.7%, four 82.1%); 16 KiB 78-79 -> 86.3%,
    // config D's shard 0 (64 GiB of 16 KiB) 79.8-79.9 -> 86.6-87.2%; 32 KiB 77 -> 86%; GM's 65,456 B 76.6 ->
    // 84.6%; 1 MiB 77.2 -> 88.4%.  A/B knobs LAMPI_SUM_MSG_WG = fragments per workgroup (0: off),
    // LAMPI_SUM_MSG_MAX = the longest fragment taken (bytes).
    static const uint32_t msg_wg = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_MSG_WG");
        return e ? (uint32_t)std::atoi(e) : 1u;
    }();
    static const size_t msg_max = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_MSG_MAX");
        return e ? (size_t)std::atoll(e) : ~(size_t)0;
    }();
    // fragments of 64 B .. 1 KiB (powers of two) in packed rows of config B's kernel (2 KiB: one per wave reads
    // faster, below); the message's last fragments through the schedules below
    static const size_t packed_max = [] {  // (A/B knob LAMPI_PACKED_SUM = the longest fragment taken, 0: off)
        const char *e = LAMPI_AB_ENV("LAMPI_PACKED_SUM");
        return e ? (size_t)std::atoll(e) : (size_t)1024;
    }();
    // fragments of 64 B .. 1 KiB (powers of two): one short-lived workgroup per 4 KiB of the message (sum_row4k_kernel),
    // the message's last fragments (past its last whole 4 KiB) through the schedules below.  Same box, interleaved
    // (profiles/r06/sum_row4k_ab.txt), against the packed rows: 1 GiB of 1 KiB (config A's shape) 74.0 -> 83.1%, 512 B
    // 70.9 -> 81.8%, 256 B 67.7 -> 82.0%, 64 B 61.9 -> 76.8%; 16 GiB of 1 KiB 77.3 -> 84.7%.  A/B knob
    // LAMPI_SUM_ROW4K=0: off (the packed rows below)
    static const bool row4k = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_ROW4K");
        return !(e && e[0] == '0');
    }();
    if (row4k && frag_len >= 64 && frag_len <= 1024 && (frag_len & (frag_len - 1)) == 0 &&
        msg_len / kRowBytes >= kSumRow4kMinRows && msg_len / kRowBytes <= 0xFFFFFFFFull) {
        const size_t nrow = msg_len / kRowBytes, done = nrow * (kRowBytes / frag_len);
        const dim3 g((unsigned)nrow);
        switch (frag_len) {
            case 64: hipLaunchKernelGGL(sum_row4k_kernel<4>, g, dim3(128), 0, s, base, out); break;
            case 128: hipLaunchKernelGGL(sum_row4k_kernel<8>, g, dim3(128), 0, s, base, out); break;
            case 256: hipLaunchKernelGGL(sum_row4k_kernel<16>, g, dim3(128), 0, s, base, out); break;
            case 512: hipLaunchKernelGGL(sum_row4k_kernel<32>, g, dim3(128), 0, s, base, out); break;
            default: hipLaunchKernelGGL(sum_row4k_kernel<64>, g, dim3(128), 0, s, base, out); break;
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess || done >= n) return e;
        return launch_sum_msg(base + done * frag_len, msg_len - done * frag_len, frag_len, n - done, out + done, img,
                              grid, s);
    }
    if (frag_len <= packed_max) {
        size_t done = 0;
        const hipError_t e = launch_packed<true>(base, msg_len, frag_len, 0u, out, nullptr, s, &done);
        if (e != hipSuccess) return e;
        if (done >= n && done) return hipSuccess;
        if (done)
            return launch_sum_msg(base + done * frag_len, msg_len - done * frag_len, frag_len, n - done, out + done, img,
                                  grid, s);
    }
    const uint32_t R = (uint32_t)std::min<size_t>((frag_len + kRowBytes - 1) / kRowBytes, 0xFFFFFFFFu);
    if (msg_wg && frag_len <= msg_max && (n >= 256 || R > 8) && R > 1 && img) {  // (few large fragments too:
        // 16 x 16 MiB on the regular kernel, one fragment per chain, read 1.9%)
        // fragments over one row: the read-only descriptors' schedule (sum_ro_groups), as one workgroup
        // per fragment in batches under 4,096 fragments ran a single round of too few workgroups (1 MiB x 1,024
        // 74.6 -> 46.7%, profiles/r05/sum_ro_sched_ab.txt)
        const uint32_t W = sum_ro_groups(n, R);
        const MsgSource src{base, msg_len, frag_len, 0u};
        if (W <= 1) {
            launch_sum_copy(src, n, out, s);
            return hipGetLastError();
        }
        if (W < 0xFFFFFFFFu) return launch_sum_copy_groups(src, n, out, s, W);
    }
    // fragments of at most 2 KiB one per wave (as launch_sum_desc: 1,976 B 51.2 -> 74.9%, 2 KiB 68 -> 84.2%)
    static const bool ro_waves = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_RO_WAVES");
        return !(e && e[0] == '0');
    }();
    // messages of fragments up to 1 KiB: the SUM piece streams with 256 fragments per workgroup (many fragments
    // share a row; profiles/r05/sum_tiny_ab.txt: 64 B 6.5 -> 19.8%, 256 B 22.8 -> 48.6%, 512 B 44.7 -> 67.6%,
    // 1 KiB 70.2 -> 72.4%).  A/B knob LAMPI_SUM_TINY = the longest fragment taken (0: off).
    static const uint32_t tiny_max = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_TINY");
        return e ? (uint32_t)std::atoi(e) : 1024u;
    }();
    if (img && frag_len <= tiny_max && n / 256 >= 256) {
        hipLaunchKernelGGL((crc_stream_kernel<MsgSource, kStreamD, kStreamK, true, kSumWv, kSumCap>),
                           frags_grid(n, 256), dim3(64 * kSumWv), 0, s, MsgSource{base, msg_len, frag_len, 0u}, n, 256u,
                           img, out, nullptr);
        return hipGetLastError();
    }
    if (ro_waves && frag_len <= kRowBytes / 2 && n >= 256) {
        launch_sum_copy(MsgSource{base, msg_len, frag_len, 0u}, n, out, s, true);
        return hipGetLastError();
    }
    if (msg_wg && frag_len <= msg_max && n >= 256 && R <= 1) {
        hipLaunchKernelGGL(sum_copy_wg_kernel<MsgSource>,
                           dim3((unsigned)std::min<size_t>((n + msg_wg - 1) / msg_wg, kMaxWgGrid)), dim3(kSumWgThreads), 0,
                           s, MsgSource{base, msg_len, frag_len, 0u}, n, out);
        return hipGetLastError();
    }
    if (msg_len != 0 && frag_len % kRowBytes == 0 && msg_len % frag_len == 0 && regular_msg_frag(frag_len, true) &&
        ((uintptr_t)base & 15u) == 0 && n <= 0xFFFFFFFFull) {
        return launch_regular<true>(base, n, frag_len, 0u, out, nullptr, s);
    }
    if (img) {
        const uint32_t fpg = sum_frags_per_wg(n, frag_len);
        hipLaunchKernelGGL((crc_stream_kernel<MsgSource, kStreamD, kStreamK, true, kSumWv, kSumCap>),
                           frags_grid(n, fpg), dim3(64 * kSumWv), 0, s, MsgSource{base, msg_len, frag_len, 0u}, n, fpg, img, out,
                           nullptr);
        return hipGetLastError();
    }
    const uint32_t fpw = pick_fpw(n, 1);
    hipLaunchKernelGGL(sum_rows_kernel<MsgSource>, grid_for(n, fpw), dim3(kBlock), 0, s,
                       MsgSource{base, msg_len, frag_len, 0u}, n, fpw, out);
    return hipGetLastError();
}

// The table-light CRC copy (crc_light_copy_kernel) takes contiguous messages whose source chunks are all
// 16-byte aligned and whose destination is dword-aligned.
static bool light_copy_ok(const uint8_t *base, size_t msg_len, size_t frag_len, const uint8_t *dst, size_t dst_stride,
                          size_t n) {
    const size_t R = (frag_len + kRowBytes - 1) / kRowBytes;
    return msg_len != 0 && frag_len >= kRowBytes && frag_len % 16 == 0 && msg_len % 16 == 0 &&
           ((uintptr_t)base & 15u) == 0 && ((uintptr_t)dst & 3u) == 0 && dst_stride % 4 == 0 &&
           frag_len <= (1u << 30) && n * R <= (1ull << 26);  // <= 2^24 workgroups of 256 threads
}

static hipError_t launch_crc_light_copy(const uint8_t *base, size_t msg_len, size_t frag_len, uint32_t partial,
                                        uint8_t *dst, size_t dst_stride, size_t n, uint32_t *out, const uint32_t *img,
                                        hipStream_t s) {
    const uint32_t R = (uint32_t)((frag_len + kRowBytes - 1) / kRowBytes);
    const size_t items = n * R;
    const int kWv = light_waves();
    auto launch = [&](uint32_t *o) {
        if (kWv == 16)
            hipLaunchKernelGGL(crc_light_copy_kernel<16>, dim3((unsigned)((items + 15) / 16)), dim3(1024), 0, s, base,
                               msg_len, (uint32_t)frag_len, R, items, partial, dst, dst_stride, img, o);
        else if (kWv == 8)
            hipLaunchKernelGGL(crc_light_copy_kernel<8>, dim3((unsigned)((items + 7) / 8)), dim3(512), 0, s, base,
                               msg_len, (uint32_t)frag_len, R, items, partial, dst, dst_stride, img, o);
        else
            hipLaunchKernelGGL(crc_light_copy_kernel<4>, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, base,
                               msg_len, (uint32_t)frag_len, R, items, partial, dst, dst_stride, img, o);
    };
    if (R == 1) {
        launch(out);
        return hipGetLastError();
    }
    uint32_t *rows = nullptr;
    bool pooled = false;
    hipError_t e = stream_scratch(s, items * sizeof(uint32_t), (void **)&rows, &pooled);
    if (e != hipSuccess) return e;
    launch(rows);
    e = hipGetLastError();
    if (e == hipSuccess) {
        const size_t per_wg = R <= kJoinThreadRows ? 256 : 4;  // fragments per workgroup
        hipLaunchKernelGGL(crc_light_join_kernel, dim3((unsigned)((n + per_wg - 1) / per_wg)), dim3(256), 0, s, rows, n,
                           R, out);
        e = hipGetLastError();
    }
    return scratch_done(s, rows, pooled, e);
}

hipError_t launch_msg_bcopy(const uint8_t *base, size_t msg_len, size_t frag_len, uint32_t partial, uint8_t *dst,
                            size_t dst_stride, size_t n, uint32_t *out, int mode, const uint32_t *img, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const bool regular = msg_len != 0 && frag_len % kRowBytes == 0 && msg_len % frag_len == 0 &&
                         ((uintptr_t)base & 15u) == 0 && ((uintptr_t)dst & 3u) == 0 && dst_stride % 4 == 0 &&
                         n <= 0xFFFFFFFFull;  // dword-aligned dwordx4 stores run at the aligned rate (GM slots)
    if (mode == LAMPI_CSUM_CRC32) {
        // fragments of 64 B .. 1 KiB (powers of two) over >= 256 whole 4 KiB rows: two passes -- the copy on
        // sum_row4k_copy_kernel (its sums land in out and are overwritten), then the read-only CRC of the source in
        // packed rows (launch_crc_msg); the fragments past the last whole 4 KiB through the schedules below.  Same box,
        // interleaved (profiles/r06/crc_copy_2pass_ab.txt), against the one-pass table-light copy, of read + write:
        // 1 KiB 33.9 -> 52.1%, 256 B 9.0 -> 49.5%, 64 B 2.3 -> 48.4%.  A/B knob LAMPI_CRC_COPY_2PASS=0: off
        static const bool two_pass = [] {
            const char *e = LAMPI_AB_ENV("LAMPI_CRC_COPY_2PASS");
            return !(e && e[0] == '0');
        }();
        if (two_pass && frag_len >= 64 && frag_len <= 1024 && (frag_len & (frag_len - 1)) == 0 &&
            msg_len / kRowBytes >= kSumRow4kMinRows && msg_len / kRowBytes <= 0xFFFFFFFFull) {
            const size_t nrow = msg_len / kRowBytes, done = nrow * (kRowBytes / frag_len);
            const dim3 g((unsigned)nrow);
            switch (frag_len) {
                case 64: hipLaunchKernelGGL(sum_row4k_copy_kernel<4>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
                case 128: hipLaunchKernelGGL(sum_row4k_copy_kernel<8>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
                case 256: hipLaunchKernelGGL(sum_row4k_copy_kernel<16>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
                case 512: hipLaunchKernelGGL(sum_row4k_copy_kernel<32>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
                default: hipLaunchKernelGGL(sum_row4k_copy_kernel<64>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
            }
            hipError_t e = hipGetLastError();
            if (e == hipSuccess) e = launch_crc_msg(base, nrow * kRowBytes, frag_len, partial, done, out, img, 0, s);
            if (e != hipSuccess || done >= n) return e;
            return launch_msg_bcopy(base + done * frag_len, msg_len - done * frag_len, frag_len, partial,
                                    dst + done * dst_stride, dst_stride, n - done, out + done, mode, img, s);
        }
        if (light_copy_ok(base, msg_len, frag_len, dst, dst_stride, n))
            return launch_crc_light_copy(base, msg_len, frag_len, partial, dst, dst_stride, n, out, img, s);
        if (regular) return launch_crc_regular_copy(base, n, frag_len, partial, dst, dst_stride, out, img, s);
        // ragged or unaligned messages: one wave per fragment on the same tables (any alignment)
        return launch_crc_light_frag_copy(MsgCopySource{base, msg_len, frag_len, partial, dst, dst_stride}, n, img,
                                          out, s);
    }
    // SUM copies of 64 B .. 1 KiB fragments (powers of two): one short-lived workgroup per 4 KiB of the message
    // (sum_row4k_copy_kernel), the fragments past the last whole 4 KiB through the schedules below.  Same box,
    // interleaved (profiles/r06/sum_row4k_copy_ab.txt), against one workgroup per fragment, of read + write: 1 KiB
    // 56.4 -> 79.3%, 256 B 17.2 -> 78.2%, 64 B 5.0 -> 79.2%.  A/B knob LAMPI_SUM_ROW4K_COPY=0: off
    static const bool row4k_copy = [] {
        const char *e = LAMPI_AB_ENV("LAMPI_SUM_ROW4K_COPY");
        return !(e && e[0] == '0');
    }();
    if (row4k_copy && mode == LAMPI_CSUM_SUM32 && frag_len >= 64 && frag_len <= 1024 && (frag_len & (frag_len - 1)) == 0 &&
        msg_len / kRowBytes >= kSumRow4kMinRows && msg_len / kRowBytes <= 0xFFFFFFFFull) {
        const size_t nrow = msg_len / kRowBytes, done = nrow * (kRowBytes / frag_len);
        const dim3 g((unsigned)nrow);
        switch (frag_len) {
            case 64: hipLaunchKernelGGL(sum_row4k_copy_kernel<4>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
            case 128: hipLaunchKernelGGL(sum_row4k_copy_kernel<8>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
            case 256: hipLaunchKernelGGL(sum_row4k_copy_kernel<16>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
            case 512: hipLaunchKernelGGL(sum_row4k_copy_kernel<32>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
            default: hipLaunchKernelGGL(sum_row4k_copy_kernel<64>, g, dim3(128), 0, s, base, dst, dst_stride, out); break;
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess || done >= n) return e;
        return launch_msg_bcopy(base + done * frag_len, msg_len - done * frag_len, frag_len, partial,
                                dst + done * dst_stride, dst_stride, n - done, out + done, mode, img, s);
    }
    const uint64_t rpf = (frag_len + kRowBytes - 1) / kRowBytes;
    const uint32_t W = msg_len != 0 && rpf < 0xFFFFFFFFull ? sum_copy_groups((uint32_t)rpf, frag_len % kRowBytes == 0)
                                                            : 1u;
    if (W > 1) return launch_sum_copy_groups(MsgCopySource{base, msg_len, frag_len, 0u, dst, dst_stride}, n, out, s, W);
    if (msg_len != 0 && frag_len >= kRowBytes && frag_len % 16 == 0 && msg_len % 16 == 0 &&
        ((uintptr_t)base & 15u) == 0 && ((uintptr_t)dst & 3u) == 0 && dst_stride % 4 == 0 &&
        n * rpf <= 0xFFFFFFFFull) {
        if (rpf > 1) {  // rows add into out
            const hipError_t e = hipMemsetAsync(out, 0, n * sizeof(uint32_t), s);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(sum_copy_row_kernel<>, dim3((unsigned)std::min<size_t>(n * rpf, kMaxWgGrid)), dim3(kSumRowThreads), 0, s,
                           base, msg_len, frag_len, (uint32_t)rpf, (uint32_t)(n * rpf), out, dst, dst_stride);
        return hipGetLastError();
    }
    // SUM: sum_copy_wg_kernel, one short-lived workgroup per 4 KiB row of any layout (textbook copy
    // shape, non-temporal stores): 4M x 4 KiB 69.8 -> 78.9% of read + write, GM 65,456-byte payloads
    // into 64 KiB slots at +72 61.6 -> 75.0% (profiles/r02_nt/)
    if (frag_len > kRowBytes && msg_len != 0) {  // fragments of several rows: row items (MsgRowCopySource)
        const hipError_t e = hipMemsetAsync(out, 0, n * sizeof(uint32_t), s);
        if (e != hipSuccess) return e;
        launch_sum_copy(MsgRowCopySource{base, msg_len, frag_len, dst, dst_stride, (uint32_t)rpf}, n * rpf, out, s);
        return hipGetLastError();
    }
    // fragments of at most one row: one workgroup each
    launch_sum_copy(MsgCopySource{base, msg_len, frag_len, 0u, dst, dst_stride}, n, out, s);
    return hipGetLastError();
}

hipError_t launch_header_csum(const uint8_t *hdrs, size_t n, size_t stride, uint32_t crclen, uint32_t word_count,
                              int mode, const uint32_t *img, uint8_t *out, size_t out_stride, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(header_csum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, hdrs, (uint32_t)n, stride,
                       crclen, word_count, mode, img, out, out_stride);
    return hipGetLastError();
}

hipError_t launch_header_check(const uint8_t *hdrs, size_t n, size_t stride, uint32_t hdr_bytes, uint32_t word_count,
                               uint32_t csum_offset, int mode, const uint32_t *img, uint32_t *mask, uint32_t *nbad,
                               hipStream_t s) {
    hipError_t e = hipMemsetAsync(nbad, 0, sizeof(uint32_t), s);
    if (e != hipSuccess || n == 0) return e;
    hipLaunchKernelGGL(header_check_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, hdrs, (uint32_t)n,
                       stride, hdr_bytes, word_count, csum_offset, mode, img, mask, nbad);
    return hipGetLastError();
}

hipError_t launch_header_compare(const uint8_t *hdrs, size_t n, size_t stride, uint32_t crclen, uint32_t csum_offset,
                                 int mode, const uint32_t *img, uint32_t *mask, uint32_t *nbad, hipStream_t s) {
    hipError_t e = hipMemsetAsync(nbad, 0, sizeof(uint32_t), s);
    if (e != hipSuccess || n == 0) return e;
    header_compare_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, s>>>(hdrs, (uint32_t)n, stride, crclen,
                                                                         csum_offset, mode, img, mask, nbad);
    return hipGetLastError();
}

hipError_t launch_check_data(const uint32_t *calc, const uint8_t *expected, size_t exp_stride, const uint8_t *lengths,
                             size_t len_stride, size_t n, uint32_t *mask, uint32_t *nbad, hipStream_t s) {
    hipError_t e = hipMemsetAsync(nbad, 0, sizeof(uint32_t), s);
    if (e != hipSuccess || n == 0) return e;
    hipLaunchKernelGGL(check_data_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, calc, expected,
                       exp_stride, lengths, len_stride, (uint32_t)n, mask, nbad);
    return hipGetLastError();
}

hipError_t launch_scatter_u32(const uint32_t *vals, size_t n, uint8_t *dst, size_t stride, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_u32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, vals, (uint32_t)n, dst,
                       stride);
    return hipGetLastError();
}

hipError_t launch_chain(const lampi_copy_desc *d, size_t npieces, const uint32_t *first, size_t nfrags, uint32_t *out,
                        int mode, const uint32_t *img, uint32_t *vals, uint32_t *phase, hipStream_t s,
                        const ChainVerdict *verdict) {
    if (nfrags == 0) return hipSuccess;
    ChainVerdict v = verdict ? *verdict : ChainVerdict{};
    if (mode == LAMPI_CSUM_NONE) {  // copies on the SUM kernels, no checksum
        v.nocheck = 1;
        mode = LAMPI_CSUM_SUM32;
    }
    if (v.copied) {
        const size_t nwords = (nfrags + 31) / 32;
        hipLaunchKernelGGL(zero_verdicts_kernel, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, s, v.mask, nwords,
                           v.nbad);
    }
    constexpr uint32_t kSmall = 256;  // pieces up to this many bytes: one thread each
    const bool sum = mode != LAMPI_CSUM_CRC32;
    if (npieces) {
        if (sum)
            hipLaunchKernelGGL(chain_phase_kernel, dim3((unsigned)((nfrags + 255) / 256)), dim3(256), 0, s, d, first,
                               (uint32_t)nfrags, phase);
        const uint32_t fpw = pick_fpw(npieces, 1);
        const PieceSource src{d, sum ? phase : nullptr, kSmall};
        if (sum)
            hipLaunchKernelGGL(sum_rows_kernel<PieceSource>, grid_for(npieces, fpw), dim3(kBlock), 0, s, src, npieces,
                               fpw, vals);
        else
            launch_crc_rows_copy(src, npieces, 1, img, vals, s);
        hipLaunchKernelGGL(chain_small_kernel, dim3((unsigned)((npieces + 255) / 256)), dim3(256), 0, s, d,
                           (uint32_t)npieces, phase, kSmall, mode, img, vals);
    }
    hipLaunchKernelGGL(chain_fold_kernel, dim3((unsigned)((nfrags + kWaves - 1) / kWaves)), dim3(kBlock), 0, s, d, first,
                       (uint32_t)nfrags, vals, mode, img, out, v);
    return hipGetLastError();
}

hipError_t launch_crc_combine(const uint32_t *vals, uint32_t n, const uint32_t *tabs, uint32_t npow,
                              uint32_t *out, hipStream_t s, uint64_t *sig, uint64_t seq) {
    hipLaunchKernelGGL(crc_combine_kernel, dim3(1), dim3(1024), 2 * npow * sizeof(uint32_t), s, vals, n, tabs, npow,
                       out, sig, seq);
    return hipGetLastError();
}

// One host-call piece by value (HostOneSource): the piece-stream kernel on a single fragment,
// its result stored to out and followed by the host signal.
hipError_t launch_host_one(const uint8_t *addr, uint32_t len, uint32_t partial, uint32_t *out, int mode,
                           const uint32_t *img, hipStream_t s, uint64_t *sig, uint64_t seq) {
    const HostOneSource src{(uint64_t)(uintptr_t)addr, len, partial, sig, seq};
    if (mode == LAMPI_CSUM_CRC32)
        hipLaunchKernelGGL((crc_stream_kernel<HostOneSource, kStreamD, kStreamK, false, kStreamWv, kStreamCap>), dim3(1),
                           dim3(64 * kStreamWv), 0, s, src, (size_t)1, 1u, img, out, nullptr);
    else
        hipLaunchKernelGGL((crc_stream_kernel<HostOneSource, kStreamD, kStreamK, true, kStreamWv, kStreamCap>), dim3(1),
                           dim3(64 * kStreamWv), 0, s, src, (size_t)1, 1u, img, out, nullptr);
    return hipGetLastError();
}

hipError_t launch_sum_finish(const uint32_t *partials, uint32_t npart, const uint8_t *src, uint64_t len,
                             uint32_t pint, uint32_t plen, uint32_t *out3, hipStream_t s, uint64_t *sig, uint64_t seq) {
    hipLaunchKernelGGL(sum_stream_finish_kernel, dim3(1), dim3(partials ? 256 : 1024), 0, s, partials, npart, src, len,
                       pint, plen, out3, sig, seq);
    return hipGetLastError();
}

hipError_t launch_fill_frags(uint64_t *dst, size_t n, uint64_t frag_words, uint64_t seed, uint64_t k0,
                             uint64_t kstep, int grid, hipStream_t s) {
    if (n == 0 || frag_words == 0) return hipSuccess;
    hipLaunchKernelGGL(fill_frags_kernel, dim3(grid * 16), dim3(256), 0, s, dst, n, frag_words, seed, k0, kstep);
    return hipGetLastError();
}

hipError_t launch_fill_stream(uint8_t *dst, size_t nbytes, uint64_t seed, uint64_t byte_off, int grid,
                              hipStream_t s) {
    if (nbytes == 0) return hipSuccess;
    size_t need = (nbytes / 16 + 255) / 256;
    size_t cap = (size_t)grid * 16;
    int g = (int)(need < 1 ? 1 : (need < cap ? need : cap));
    hipLaunchKernelGGL(fill_stream_kernel, dim3(g), dim3(256), 0, s, dst, nbytes, seed, byte_off);
    return hipGetLastError();
}

}  // namespace lampi
