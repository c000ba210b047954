// send_ring_caller.cc -- a native C++ caller of the device-resident send step written in place
// (include/lampi_csum.h: lampi_msg_bcopy_strided, lampi_chain_csum_batch_strided, lampi_frag_bcopy_batch_strided,
// lampi_header_csum_batch_strided), in the shape of LA-MPI's GM send: gmSendFragDesc::init packs each fragment
// into a 64 KiB NIC buffer -- 72-byte gmHeaderData, then the payload -- stores the payload checksum into
// dataChecksum (@64) and then the byte-swapped header CRC (or the header word sum) into checksum (@68)
// (ref src/path/gm/sendFrag.cc:143-226, src/path/gm/header.h:56-70).
//
// One ring per mode (CRC, SUM, checksumming off) is packed on one stream: a contiguous message of 65,456-byte
// fragments (odd start address, short last fragment), typemap fragments gathered from scattered pieces, and
// descriptor copies of ragged lengths; then every header is stamped in place.  The ring comes back to the host
// and every byte is checked against what the reference's send loop would have left there, computed with the
// oracle (oracle/libcsum_ref.so, the reference-pinned restatement -- test infrastructure): payload bytes,
// dataChecksum, checksum, and the receiver's header test (CRC: uicrc(header, 72) == 0; SUM: the 18 words sum to
// twice the stored word, gm/path.cc:364-393).  With checksumming off the two checksum words are left as they
// were (sendFrag.cc:153-155, :219).  Prints one line per mode and "bad N done"; exits 1 on any mismatch.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "lampi_csum.h"
#include "../../oracle/csum_ref.h"

#define HIPCHECK(x)                                                                   \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::printf("HIP error %d at %s:%d\n", (int)e_, __FILE__, __LINE__);      \
            std::exit(2);                                                             \
        }                                                                             \
    } while (0)

static constexpr size_t kBuf = 65536, kHdr = 72, kPayload = 65456, kWords = 18, kDcsum = 64, kHcsum = 68;

static void wr32(uint8_t *p, uint32_t v) { std::memcpy(p, &v, 4); }
static uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}

struct Piece {
    size_t src, dst, len;
};

static int run_mode(int mode, hipStream_t s) {
    std::mt19937_64 rng(900 + mode);
    const size_t n_msg = 21, n_tm = 16, n_desc = 27, nbuf = n_msg + n_tm + n_desc;
    const size_t msg_len = (n_msg - 1) * kPayload + 4099;
    const size_t src_len = 4u << 20;

    // host images: the ring (random header fields, checksum word 0), the message, the piece source
    std::vector<uint8_t> ring(nbuf * kBuf), msg(msg_len + 1), src(src_len);
    oracle_fill_stream(ring.data(), 31 + mode, 0, ring.size());
    for (size_t b = 0; b < nbuf; ++b) wr32(&ring[b * kBuf + kHcsum], 0u);
    oracle_fill_stream(msg.data(), 32, 0, msg.size());
    oracle_fill_stream(src.data(), 33, 0, src.size());

    uint8_t *d_ring = nullptr, *d_msg = nullptr, *d_src = nullptr;
    HIPCHECK(hipMalloc((void **)&d_ring, ring.size()));
    HIPCHECK(hipMalloc((void **)&d_msg, msg.size()));
    HIPCHECK(hipMalloc((void **)&d_src, src.size()));
    HIPCHECK(hipMemcpy(d_ring, ring.data(), ring.size(), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_msg, msg.data(), msg.size(), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_src, src.data(), src.size(), hipMemcpyHostToDevice));

    // typemap fragments: pieces of 1 B .. 20 KB gathered into payloads of random length
    std::vector<Piece> pieces;
    std::vector<uint32_t> first{0};
    const size_t sizes[] = {1, 3, 64, 777, 4096, 20000};
    for (size_t f = 0; f < n_tm; ++f) {
        size_t pos = (n_msg + f) * kBuf + kHdr;
        const size_t end = pos + rng() % (kPayload + 1);
        while (pos < end) {
            const size_t k = std::min(end - pos, sizes[rng() % 6]);
            pieces.push_back({(size_t)(rng() % (src_len - k)), pos, k});
            pos += k;
        }
        first.push_back((uint32_t)pieces.size());
    }
    std::vector<lampi_copy_desc> pd(pieces.size());
    for (size_t i = 0; i < pieces.size(); ++i)
        pd[i] = {(uint64_t)(uintptr_t)(d_src + pieces[i].src), (uint64_t)(uintptr_t)(d_ring + pieces[i].dst),
                 (uint32_t)pieces[i].len, (uint32_t)pieces[i].len, LAMPI_CRC_INITIAL_REGISTER, 0u};
    // descriptor copies: ragged lengths (0, 1, 3, a full payload, random)
    std::vector<lampi_copy_desc> cd(n_desc);
    std::vector<size_t> c_src(n_desc), c_len(n_desc);
    for (size_t i = 0; i < n_desc; ++i) {
        c_len[i] = i == 0 ? 0 : i == 1 ? 1 : i == 2 ? 3 : i == 3 ? kPayload : rng() % (kPayload + 1);
        c_src[i] = rng() % (src_len - kPayload);
        cd[i] = {(uint64_t)(uintptr_t)(d_src + c_src[i]),
                 (uint64_t)(uintptr_t)(d_ring + (n_msg + n_tm + i) * kBuf + kHdr), (uint32_t)c_len[i],
                 (uint32_t)c_len[i], LAMPI_CRC_INITIAL_REGISTER, 0u};
    }
    lampi_copy_desc *d_pieces = nullptr, *d_cd = nullptr;
    uint32_t *d_first = nullptr;
    HIPCHECK(hipMalloc((void **)&d_pieces, std::max<size_t>(1, pd.size()) * sizeof(lampi_copy_desc)));
    HIPCHECK(hipMalloc((void **)&d_cd, cd.size() * sizeof(lampi_copy_desc)));
    HIPCHECK(hipMalloc((void **)&d_first, first.size() * sizeof(uint32_t)));
    HIPCHECK(hipMemcpy(d_pieces, pd.data(), pd.size() * sizeof(lampi_copy_desc), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_cd, cd.data(), cd.size() * sizeof(lampi_copy_desc), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_first, first.data(), first.size() * sizeof(uint32_t), hipMemcpyHostToDevice));

    const bool none = mode == LAMPI_CSUM_NONE;
    int rc = 0;
    // the message: payload k at buffer k + 72, dataChecksum at buffer k + 64 (out_stride = the buffer size)
    rc |= lampi_msg_bcopy_strided(d_msg + 1, msg_len, kPayload, d_ring + kHdr, kBuf, LAMPI_CRC_INITIAL_REGISTER,
                                  none ? nullptr : d_ring + kDcsum, kBuf, mode, s);
    rc |= lampi_chain_csum_batch_strided(d_pieces, pd.size(), d_first, n_tm,
                                         none ? nullptr : d_ring + n_msg * kBuf + kDcsum, kBuf, mode, s);
    rc |= lampi_frag_bcopy_batch_strided(d_cd, n_desc, none ? nullptr : d_ring + (n_msg + n_tm) * kBuf + kDcsum,
                                         kBuf, mode, s);
    // then every header's checksum in place: headerChecksum(headerp, sizeof(gmHeader) - 4, GM_HDR_WORDS)
    rc |= lampi_header_csum_batch_strided(d_ring, nbuf, kBuf, (uint32_t)(kHdr - 4), (uint32_t)kWords,
                                          none ? nullptr : d_ring + kHcsum, kBuf, mode, s);
    HIPCHECK(hipStreamSynchronize(s));
    std::vector<uint8_t> got(ring.size());
    HIPCHECK(hipMemcpy(got.data(), d_ring, got.size(), hipMemcpyDeviceToHost));

    // what the reference's send loop leaves in the ring
    std::vector<uint8_t> want = ring;
    auto stamp = [&](size_t b, const std::vector<std::pair<const uint8_t *, size_t>> &parts) {
        uint8_t *p = &want[b * kBuf + kHdr];
        uint32_t crc = LAMPI_CRC_INITIAL_REGISTER, sum = 0, pint = 0, plen = 0;
        for (auto &pt : parts) {
            std::memcpy(p, pt.first, pt.second);
            p += pt.second;
            crc = oracle_uicrc(pt.first, pt.second, crc);
            sum += oracle_uicsum(pt.first, pt.second, &pint, &plen);
        }
        if (none) return;
        wr32(&want[b * kBuf + kDcsum], mode == LAMPI_CSUM_CRC32 ? crc : sum);
        wr32(&want[b * kBuf + kHcsum],
             oracle_header_checksum(&want[b * kBuf], kHdr - 4, (int)kWords, mode == LAMPI_CSUM_CRC32));
    };
    for (size_t k = 0; k < n_msg; ++k)
        stamp(k, {{&msg[1 + k * kPayload], std::min(kPayload, msg_len - k * kPayload)}});
    for (size_t f = 0; f < n_tm; ++f) {
        std::vector<std::pair<const uint8_t *, size_t>> parts;
        for (uint32_t j = first[f]; j < first[f + 1]; ++j) parts.push_back({&src[pieces[j].src], pieces[j].len});
        stamp(n_msg + f, parts);
    }
    for (size_t i = 0; i < n_desc; ++i) stamp(n_msg + n_tm + i, {{&src[c_src[i]], c_len[i]}});

    size_t bad_bytes = 0, bad_hdr = 0;
    for (size_t i = 0; i < got.size(); ++i) bad_bytes += got[i] != want[i];
    if (!none)
        for (size_t b = 0; b < nbuf; ++b) {
            const uint8_t *h = &got[b * kBuf];
            if (mode == LAMPI_CSUM_CRC32) {
                bad_hdr += oracle_uicrc(h, kHdr, LAMPI_CRC_INITIAL_REGISTER) != 0u;
            } else {
                uint32_t w = 0;
                for (size_t j = 0; j < kWords; ++j) w += rd32(h + 4 * j);
                bad_hdr += w != 2u * rd32(h + kHcsum);
            }
        }
    const bool ok = rc == 0 && bad_bytes == 0 && bad_hdr == 0;
    std::printf("send_ring mode %d buffers %zu pieces %zu rc %d bad_bytes %zu bad_headers %zu %s\n", mode, nbuf,
                pieces.size(), rc, bad_bytes, bad_hdr, ok ? "ok" : "BAD");
    for (void *p : {(void *)d_ring, (void *)d_msg, (void *)d_src, (void *)d_pieces, (void *)d_cd, (void *)d_first})
        HIPCHECK(hipFree(p));
    return ok ? 0 : 1;
}

int main() {
    hipStream_t s = nullptr;
    HIPCHECK(hipStreamCreate(&s));
    int bad = 0;
    for (int mode : {LAMPI_CSUM_CRC32, LAMPI_CSUM_SUM32, LAMPI_CSUM_NONE}) bad += run_mode(mode, s);
    HIPCHECK(hipStreamDestroy(s));
    std::printf("bad %d done\n", bad);
    return bad ? 1 : 0;
}
