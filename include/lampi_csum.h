/*
 * lampi_csum.h -- C ABI of the MI355X fragment-checksum engine (liblampi_csum.so).
 *
 * Drop-in for LA-MPI's per-fragment data-integrity checksums:
 *   CRC mode  = uicrc / bcopy_uicrc   (CRC-32/MPEG-2: poly 0x04C11DB7, MSB-first,
 *               init 0xFFFFFFFF, no reflection, no final XOR)
 *   SUM mode  = uicsum / bcopy_uicsum (sum mod 2^32 of little-endian 32-bit words,
 *               trailing partial word zero-padded in its high bytes)
 * as declared in the reference at src/util/MemFunctions.h:43-65 and applied per
 * fragment on the send/receive datapath in src/path/{gm,ib,quadrics}.
 *
 * All computation runs in hand-written HIP kernels for gfx950.  There is no CPU
 * fallback: if no GPU is usable the host entry points abort with a message and the
 * device entry points return a nonzero error code.
 *
 * Conventions (mirroring the reference):
 *   - the caller owns every buffer; nothing is retained after a call returns
 *     (device entry points: after the stream work completes);
 *   - checksums are never overloaded as error codes: the scalar host entry points
 *     return the checksum (as the reference does); the device entry points return
 *     0 on success or a hipError_t value and write checksums to an output array;
 *   - chaining state lives with the caller (CRC `partial`, SUM (pint, plen));
 *   - `stream` is a hipStream_t passed as void* (NULL = the default stream);
 *     device entry points are stream-ordered, asynchronous, and thread-safe;
 *   - no global mutable state is visible: the lookup tables are built once per
 *     device on first use and are read-only afterwards.
 */
#ifndef LAMPI_CSUM_H
#define LAMPI_CSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LAMPI_CRC_POLYNOMIAL      0x04C11DB7u   /* ref src/util/MemFunctions.h:36 */
#define LAMPI_CRC_INITIAL_REGISTER 0xFFFFFFFFu  /* ref src/util/MemFunctions.h:37 */

/* Checksum mode; the reference selects it at run time with usecrc()
 * (src/include/internal/state.h:129-132, mpirun -crc). */
enum lampi_csum_mode {
    LAMPI_CSUM_CRC32 = 0,   /* uicrc  */
    LAMPI_CSUM_SUM32 = 1,   /* uicsum */
    /* Checksumming off: a network whose doChecksum flag is false (mpirun -mf/-if/-qf nochecksum,
     * src/run/Input.cc:1986-2067; gmState.doChecksum src/path/gm/state.h:140).  Accepted by the copying
     * batches only.  Receive side (lampi_copy_to_app_batch, lampi_chain_copy_to_app_batch and their host
     * forms): the bytes are copied, the checksum output is 0 and every fragment is DataOK, as CopyFunction /
     * nonContigCopyFunction and CheckData behave with checksumming off (src/path/gm/recvFrag.h:178-181,
     * :198-199, :231-232).  Send side (lampi_frag_bcopy_batch[_strided], lampi_msg_bcopy[_strided],
     * lampi_chain_csum_batch[_strided], lampi_host_msg_bcopy): the bytes are copied (copylen of each
     * descriptor) and the checksum output is NOT written -- it may be NULL --, as the sender's MEMCOPY_FUNC
     * leaves dataChecksum unset (src/path/gm/sendFrag.cc:153-155, :185-187, :206-208);
     * lampi_header_csum_batch_strided writes nothing either (no header checksum, :219-225). */
    LAMPI_CSUM_NONE = 2
};

/* Flag OR'ed into `mode` of lampi_frag_csum_batch[_strided] for batches of up to 32,768 descriptors:
 * split the work by bytes instead of by fragment count.  A plan kernel cuts fragments longer than the
 * plan's window into segments checksummed by different workgroups (their parts are joined exactly:
 * crc(s, A||B) = shift_|B|(crc(s, A)) ^ crc(0, B); sums add) and groups segments into workgroups of
 * about equal bytes.  It pays where a batch holds few or large fragments (1 GiB of 4 MiB descriptors:
 * 34% -> 64% of the HBM roofline; one 16 MiB fragment: 1.5 ms -> 51 us) and costs a second launch
 * (~10 us) on every call, so small batches should not set it.  Results are identical. */
#define LAMPI_CSUM_BY_BYTES 0x100

/* Hint OR'ed into `mode` of the copy batches (lampi_frag_bcopy_batch, lampi_copy_to_app_batch):
 * fragments span about r 4 KiB rows (1..4095; GM's 65,456-byte payloads: 16).  Each fragment then runs
 * as r row groups in parallel, joined exactly afterwards (a second, small launch) -- the one-row-per-wave
 * shape of the message copy instead of one wave (SUM: one workgroup) walking every row.  Results are
 * identical for any lengths (a longer fragment gets longer groups); r = 0 or 1 is the default walk.
 * Both modes: GM payloads CRC 60 -> 71%, SUM 57 -> 72%; the receive step CRC 59 -> 69%, SUM 56 -> 72%.
 * Also accepted by lampi_frag_csum_batch[_strided] (read-only; LAMPI_CSUM_BY_BYTES first): CRC with
 * r >= 8 walks each fragment's rows in one wave of the table-light kernel (above 16 rows, one wave per
 * 8 rows, joined exactly) -- 1 GiB of GM payloads CRC 56 -> 80%, of 1 MiB / 4 MiB descriptors 57 / 34
 * -> 80%; smaller r and SUM size workgroups by the hinted length and cut fragments of more than 16
 * rows into 16-row segments on the device (out zeroed, parts joined exactly): SUM 61 -> 74%.
 * Without the hint the library learns it: batches of >= 256 descriptors are sampled on the device every
 * 16th call per stream and entry point, and later batches whose sampled fragments all span 8+ rows
 * (within a factor of two) run as if the hint had been given; CRC copies / receives of fragments all
 * <= 2 KiB (IB) run two to a wave.  The hint, when given, wins; LAMPI_CSUM_NO_SHAPES=1 in the environment
 * turns the learning off.  Results never depend on either. */
#define LAMPI_CSUM_ROWS_HINT(r) ((int)(((unsigned)(r) & 0xFFFu) << 16))
#define LAMPI_CSUM_ROWS_HINT_MASK LAMPI_CSUM_ROWS_HINT(0xFFFu)
#define LAMPI_CSUM_ROWS_HINT_OF(mode) ((((unsigned)(mode)) >> 16) & 0xFFFu)

/* ------------------------------------------------------------------------------------
 * Host-memory, synchronous entry points (same meaning as the reference overloads).
 * The bytes are moved to the GPU, checksummed (and copied) there, and moved back.
 * ---------------------------------------------------------------------------------- */

/* replaces unsigned int uicrc(const void*, unsigned long, unsigned int)
 *   ref src/util/MemFunctions.cc:1331-1367 (mangled _Z5uicrcPKvmj) */
unsigned int lampi_uicrc(const void *src, unsigned long crclen, unsigned int partial_crc);

/* replaces unsigned int bcopy_uicrc(const void*, void*, unsigned long, unsigned long, unsigned int)
 *   ref src/util/MemFunctions.cc:1263-1321 (_Z11bcopy_uicrcPKvPvmmj).
 *   Copies copylen bytes; the CRC covers max(copylen, crclen) bytes of src. */
unsigned int lampi_bcopy_uicrc(const void *src, void *dst, unsigned long copylen,
                               unsigned long crclen, unsigned int partial_crc);

/* replaces unsigned int uicsum(const void*, unsigned long, unsigned int*, unsigned int*)
 *   ref src/util/MemFunctions.cc:1073-1222 (_Z6uicsumPKvmPjS1_).
 *   Returns the increment to the running sum; (*pint, *plen) is the partial-word state
 *   (*plen in 0..3; 4 or more is treated as 0, where the reference is undefined). */
unsigned int lampi_uicsum(const void *src, unsigned long csumlen, unsigned int *pint,
                          unsigned int *plen);

/* replaces unsigned int bcopy_uicsum(const void*, void*, unsigned long, unsigned long,
 *                                    unsigned int*, unsigned int*)
 *   ref src/util/MemFunctions.cc:518-875 (_Z12bcopy_uicsumPKvPvmmPjS2_).
 *   Copies copylen bytes; the sum covers max(copylen, csumlen) bytes of src. */
unsigned int lampi_bcopy_uicsum(const void *src, void *dst, unsigned long copylen,
                                unsigned long csumlen, unsigned int *pint, unsigned int *plen);

/* replaces unsigned long csum(const void*, unsigned long, unsigned long*, unsigned long*)
 *   ref src/util/MemFunctions.cc:913-1071 (_Z4csumPKvmPmS1_): sum mod 2^64 of little-endian
 *   64-bit words with the trailing partial word zero-padded; (*plong, *plen) chain it like
 *   uicsum's state (*plen in 0..7; 8 or more is treated as 0).  No path caller in the reference. */
unsigned long lampi_csum(const void *src, unsigned long csumlen, unsigned long *plong, unsigned long *plen);

/* replaces unsigned long bcopy_csum(const void*, void*, unsigned long, unsigned long,
 *                                   unsigned long*, unsigned long*)
 *   ref src/util/MemFunctions.cc:142-516 (_Z10bcopy_csumPKvPvmmPmS2_).
 *   Copies copylen bytes; the sum covers max(copylen, csumlen) bytes of src. */
unsigned long lampi_bcopy_csum(const void *src, void *dst, unsigned long copylen, unsigned long csumlen,
                               unsigned long *plong, unsigned long *plen);

/* ------------------------------------------------------------------------------------
 * Host-memory message path: a range of a host message's fragments in one call.
 * Fragment k of the message = bytes [k*frag_len, min((k+1)*frag_len, msg_len)) -- the path
 * layer's split (src/path/gm/path.cc:98-121); a zero-length message is one empty fragment.
 * The call covers fragments k_first .. k_first+k_count-1 (a sender gated by clear-to-send /
 * maxOutstandingFrags, gm/path.cc:104-118, passes the fragments it may send now) and writes
 * their checksums to h_out[0 .. k_count).  Every fragment starts from `partial` (CRC mode,
 * CRC_INITIAL_REGISTER for the path's per-fragment value) or a fresh state (SUM mode).
 *
 * Inside, a chunked pipeline on the calling thread's own streams: H2D of chunk i+1 overlaps
 * the checksum kernels of chunk i and the D2H of chunk i-1.  The DMA engines read the
 * message and write the slots in place, page-locked or pageable (the runtime stages pageable
 * H2D at the pinned rate; pageable slots halve the D2H rate: register NIC rings with
 * lampi_host_register).  Synchronous: everything is written when the call returns.  Returns 0 or a hipError_t
 * (invalid arguments -- frag_len 0 or above 1 GiB among them -- hipErrorInvalidValue; nothing is written
 * then; after a failure nothing is left in flight).
 * ---------------------------------------------------------------------------------- */

/* Checksum-only: what the sender stores in dataChecksum for each fragment of the range --
 * the per-fragment uicrc / uicsum of gmSendFragDesc::init (src/path/gm/sendFrag.cc:147-155)
 * without the copy, and the Quadrics checksum over the DMA source
 * (src/path/quadrics/sendFrag.h:861-872). */
int lampi_host_msg_csum(const void *h_msg, size_t msg_len, size_t frag_len, size_t k_first, size_t k_count,
                        uint32_t partial, uint32_t *h_out, int mode);

/* Fused copy + checksum into NIC buffers: fragment k_first+i is copied to
 * h_ring + i*slot_stride (slot_stride >= frag_len; e.g. the payload area of a ring of
 * header + payload buffers: h_ring = first buffer + 72, slot_stride = the buffer size) and
 * h_out[i] = bcopy_uicrc / bcopy_uicsum of it (copylen = crclen = the fragment length), as the
 * send loop of gmPath::send does per fragment (src/path/gm/path.cc:98-176, sendFrag.cc:147-155).
 * The bytes written to the slots are exactly the bytes checksummed; no other byte of the ring
 * is touched.  h_ring must not overlap h_msg.  mode LAMPI_CSUM_NONE: the fragments are copied
 * (through the same DMA pipeline, no kernel) and h_out is unused (may be NULL). */
int lampi_host_msg_bcopy(const void *h_msg, size_t msg_len, size_t frag_len, size_t k_first, size_t k_count,
                         void *h_ring, size_t slot_stride, uint32_t partial, uint32_t *h_out, int mode);

/* ------------------------------------------------------------------------------------
 * Host-memory receive path: a batch of received fragments in one call.
 * The reference's receive loop drains every pending NIC event (gmPath::receive,
 * src/path/gm/path.cc:286-313; ibPath::receive, src/path/ib/path.cc:630-741), checks each
 * header (gm/path.cc:364-393, ib/path.cc:652-680), matches the fragment to a posted receive and
 * delivers it with RecvDesc_t::CopyToApp (src/path/common/BaseDesc.cc:288-342).  These entry
 * points take the drained batch at once: the fragments sit anywhere in a host NIC ring
 * [h_ring, h_ring + ring_bytes) (page-locked or pageable; every byte of it may be read by the
 * DMA engines, so it must be one readable range), the application buffers anywhere in host
 * memory (they must not overlap the ring).  Synchronous, on the calling thread's own streams (the
 * pipeline of the send path): when the call returns every result and delivered byte is in place.
 * Return 0 or a hipError_t; invalid arguments return hipErrorInvalidValue before anything is
 * written.  Masks hold one bit per fragment, bit (i % 32) of word i / 32, SET when fragment i
 * FAILS; *h_nbad receives the number of failures.
 * ---------------------------------------------------------------------------------- */

/* One received fragment to deliver (32 bytes, little-endian): offset 0 frag_off, 8 app, 16 app_len,
 * 24 length, 28 expected. */
typedef struct lampi_host_recv_frag {
    uint64_t frag_off;  /* the payload's offset in the ring (BaseRecvFragDesc_t::addr_m - h_ring) */
    void    *app;       /* host address it is delivered to: RecvDesc_t::addr_m + dataOffset() */
    int64_t  app_len;   /* room left in the posted buffer at that offset: posted_m.length_m - Offset
                           (ref BaseDesc.cc:307); may be <= 0 */
    uint32_t length;    /* bytes received, length_m (GM: event length - sizeof(gmHeader)); all of them are
                           checksummed */
    uint32_t expected;  /* the sender's checksum from the fragment's header: gmHeader_m->data.dataChecksum
                           (gm/recvFrag.h:233), msg_m->header.dataChecksum (ib/recvFrag.cc:233) */
} lampi_host_recv_frag;

/* RecvDesc_t::CopyToApp for every fragment of the batch, as lampi_copy_to_app_batch does on the device
 * (CopyFunction gm/recvFrag.h:165-182 / ib/recvFrag.cc:182-200 fused with CheckData gm/recvFrag.h:213-257
 * / ib/recvFrag.cc:229-245):
 *   lengthToCopy = app_len <= 0 ? 0 : min(length, app_len);
 *   lengthToCopy > 0:  lengthToCopy bytes ring -> app, the checksum over all `length` bytes compared with
 *                      `expected` (the bytes are delivered either way, as bcopy_uicrc does before CheckData);
 *   lengthToCopy == 0: nothing read, copied or checksummed; DataOK.
 * h_copied[i] = lengthToCopy, or -1 when the checksum differs (CopyToApp's return value); h_csum[i] = the
 * calculated checksum (CRC_INITIAL_REGISTER / 0 when nothing was checksummed); h_mask (ceil(n/32) words,
 * overwritten) and *h_nbad as above.  The fragments' ring bytes move to the GPU in as few DMA transfers as
 * their layout allows (dense runs one copy, a constant slot pitch one 2D copy), the delivered bytes come
 * back in one copy per run of fragments contiguous in the application buffer.  `mode` may carry
 * LAMPI_CSUM_ROWS_HINT(r) to override the row-group count the library derives from the fragments' mean
 * length.  Fragments up to 1 GiB.  mode LAMPI_CSUM_NONE (checksumming off): lengthToCopy bytes copied and
 * nothing more read, h_csum[i] = 0, every fragment DataOK, `expected` unused. */
int lampi_host_copy_to_app_batch(const void *h_ring, size_t ring_bytes, const lampi_host_recv_frag *h_frags,
                                 size_t n, int64_t *h_copied, uint32_t *h_csum, uint32_t *h_mask, uint32_t *h_nbad,
                                 int mode);

/* The GM receiver's header check over a batch of received headers at h_ring + h_hdr_offs[i]
 * (gmPath::receive, ref src/path/gm/path.cc:364-393), as lampi_header_check_batch does on the device:
 * header i fails unless CRC mode: uicrc(hdr_i, hdr_bytes) == 0; SUM mode: the sum of word_count words ==
 * 2 x the stored checksum at csum_offset (4-byte aligned).  Headers may sit at any byte offset; each is
 * read once (its bytes gathered into pinned staging, the checks run on the GPU). */
int lampi_host_header_check_batch(const void *h_ring, size_t ring_bytes, const uint64_t *h_hdr_offs, size_t n,
                                  uint32_t hdr_bytes, uint32_t word_count, uint32_t csum_offset, uint32_t *h_mask,
                                  uint32_t *h_nbad, int mode);

/* The IB receiver's header check over the same kind of batch (ibPath::receive, ref
 * src/path/ib/path.cc:652-680), as lampi_header_compare_batch: header i fails unless the 32-bit value at
 * csum_offset equals uicrc(hdr_i, crclen) / uicsum(hdr_i, crclen) (e.g. crclen 68, csum_offset 68 for an
 * ibDataHdr_t). */
int lampi_host_header_compare_batch(const void *h_ring, size_t ring_bytes, const uint64_t *h_hdr_offs, size_t n,
                                    uint32_t crclen, uint32_t csum_offset, uint32_t *h_mask, uint32_t *h_nbad,
                                    int mode);

/* One typemap piece in host memory (32 bytes): offset 0 src, 8 dst, 16 copylen, 20 csumlen, 24 partial,
 * 28 reserved. */
typedef struct lampi_host_piece {
    const void *src;    /* host address of the piece's bytes */
    void       *dst;    /* host address its first copylen bytes go to (NULL: checksum only) */
    uint32_t    copylen;
    uint32_t    csumlen;  /* the checksum covers max(copylen, csumlen) bytes of src */
    uint32_t    partial;  /* CRC mode, a fragment's first piece: its starting register */
    uint32_t    reserved; /* 0 */
} lampi_host_piece;

/* lampi_chain_csum_batch over pieces in host memory: fragment f is the concatenation of the checksummed
 * ranges of h_pieces[h_first[f]] .. h_pieces[h_first[f+1] - 1] (h_first: nfrags + 1 nondecreasing entries,
 * h_first[nfrags] <= npieces), each piece also copied to its dst; h_out[f] = what the reference's
 * piece-by-piece calls return (CRC: the register threaded through the pieces from the first piece's
 * partial, 0xFFFFFFFF for a fragment without pieces; SUM: the total of the increments with the
 * partial-word state threaded from a fresh state).  The send side's gather into the NIC payload
 * (src/path/gm/sendFrag.cc:157-217: bcopy_uicrc(..., csum) / csum += bcopy_uicsum(...) per typemap
 * piece; ib/sendFrag.cc:140-203) and the receive side's scatter into the application buffer
 * (non_contiguous_copy, src/path/common/BaseDesc.cc:72-163), a whole batch per call.  The DMA engines read
 * exactly the pieces' bytes and write exactly their copies: touching pieces move in one copy, equal pieces
 * at a constant stride (a strided vector) in one 2D copy.  Sources and destinations must not overlap.
 * Fragments up to 1 GiB.  Synchronous; 0 or a hipError_t (invalid arguments: hipErrorInvalidValue,
 * nothing written). */
int lampi_host_chain_csum_batch(const lampi_host_piece *h_pieces, size_t npieces, const uint32_t *h_first,
                                size_t nfrags, uint32_t *h_out, int mode);

/* RecvDesc_t::CopyToApp's non-contiguous branch for a batch of received fragments in host memory (ref
 * src/path/common/BaseDesc.cc:326-340: non_contiguous_copy :72-163, then CheckData(checkSum, len_copied),
 * gm/recvFrag.h:213-257): fragment f's pieces h_pieces[h_first[f]] .. [h_first[f+1] - 1] are the typemap
 * pieces non_contiguous_copy walks (src = the fragment's bytes in the NIC ring, dst = the application buffer,
 * copylen = csumlen = the piece's length; a fragment whose AppBufferLen <= 0 is delivered with no pieces).
 * Each piece is copied, the checksum threaded through the pieces as nonContigCopyFunction does (CRC from
 * CRC_INITIAL_REGISTER -- the pieces' partial is ignored --, SUM from a fresh state) and compared with
 * h_expected[f] (the header's dataChecksum):
 *   h_copied[f] = the bytes copied into the pieces (len_copied), or -1 when that is nonzero and the checksum
 *                 differs (CopyToApp's return value); h_csum[f] = the calculated checksum;
 *   h_mask (ceil(nfrags/32) words, bit set = corrupt, overwritten) and *h_nbad as lampi_host_copy_to_app_batch.
 * mode LAMPI_CSUM_NONE (checksumming off): copies only, h_csum 0, every fragment DataOK, h_expected unused.
 * DMA as lampi_host_chain_csum_batch.  Synchronous; 0 or a hipError_t (invalid arguments:
 * hipErrorInvalidValue, nothing written). */
int lampi_host_chain_copy_to_app_batch(const lampi_host_piece *h_pieces, size_t npieces, const uint32_t *h_first,
                                       size_t nfrags, const uint32_t *h_expected, int64_t *h_copied, uint32_t *h_csum,
                                       uint32_t *h_mask, uint32_t *h_nbad, int mode);

/* Page-lock [h_ptr, h_ptr+len) for direct DMA by the host paths (hipHostRegister) and undo it:
 * the analogue of registering NIC buffers with the network (GM gm_register_memory).  Return 0
 * or a hipError_t. */
int lampi_host_register(void *h_ptr, size_t len);
int lampi_host_unregister(void *h_ptr);

/* ------------------------------------------------------------------------------------
 * Device-resident batched entry points.
 * ---------------------------------------------------------------------------------- */

/* One fragment.  The descriptor array itself lives in device memory.
 * Layout is fixed (16 bytes, little-endian): offset 0 addr, 8 length, 12 partial. */
typedef struct lampi_frag_desc {
    uint64_t addr;      /* device address of the fragment's first byte (any alignment) */
    uint32_t length;    /* bytes (0 allowed) */
    uint32_t partial;   /* CRC mode: CRC register to start from (0xFFFFFFFF = fresh);
                           SUM mode: ignored (fresh partial-word state) */
} lampi_frag_desc;

/* out[i] = checksum of fragment d[i] (CRC register or SUM value, as uicrc/uicsum
 * would return for the same bytes).  The schedule follows the batch: a batch the
 * library has seen to be one contiguous run of equal 64 B .. 2 KiB fragments (a message handed over as
 * descriptors) runs as that message's packed rows, every descriptor still checked; otherwise, by
 * default the piece streams -- each workgroup's fragments cut into 64-byte pieces packed into full
 * 4 KiB rows, so mixed sizes keep every lane busy; with LAMPI_CSUM_ROWS_HINT (or the shape the
 * stream's earlier batches showed) long fragments one wavefront each on the table-light kernel (CRC)
 * or as row groups on short-lived workgroups (SUM); batches the library has seen to hold equal fragments
 * of 1-7 whole 4 KiB rows at 16-byte-aligned addresses on the message kernel's schedule (CRC; fragments
 * of another shape in such a batch are found and checksummed by a second launch); 1,024-65,536 fragments without a hint split by
 * size class (CRC); under 256 fragments without a hint every fragment runs as row groups sized to the
 * launch (a few large fragments no longer sit on one workgroup each; LAMPI_CSUM_ROWS_HINT(1) keeps the
 * count split for batches known to hold small fragments).  Results never depend on the schedule.
 * Replaces the per-fragment loop of gmPath::send / gmSendFragDesc::init
 * (src/path/gm/path.cc:98-176, src/path/gm/sendFrag.cc:147-155) and the Quadrics
 * checksum-only send (src/path/quadrics/sendFrag.h:861-872). */
int lampi_frag_csum_batch(const lampi_frag_desc *d_descs, size_t n, uint32_t *d_out,
                          int mode, void *stream);

/* As lampi_frag_csum_batch, with checksum i written to (char *)d_out + i*out_stride (d_out and
 * out_stride 4-byte aligned, out_stride >= 4) -- e.g. straight into the dataChecksum field of
 * an array of 72-byte gmHeaderData records: d_out = hdrs + 64, out_stride = 72
 * (src/path/gm/header.h:56-70; the send side stores it at gm/sendFrag.cc:147-155).  Other
 * bytes of the records are not touched.  Uses 4 * n bytes of stream-ordered scratch. */
int lampi_frag_csum_batch_strided(const lampi_frag_desc *d_descs, size_t n, void *d_out, size_t out_stride,
                                  int mode, void *stream);

/* out[i] = csum (64-bit words, fresh state) of fragment d[i]; d[i].partial is ignored. */
int lampi_frag_csum64_batch(const lampi_frag_desc *d_descs, size_t n, uint64_t *d_out, void *stream);

/* One fused copy + checksum (32 bytes, little-endian): offset 0 src, 8 dst, 16 copylen,
 * 20 csumlen, 24 partial, 28 reserved. */
typedef struct lampi_copy_desc {
    uint64_t src;       /* device address of the source fragment (any alignment) */
    uint64_t dst;       /* device address of the copy (any alignment; must not overlap src) */
    uint32_t copylen;   /* bytes copied src -> dst */
    uint32_t csumlen;   /* the checksum covers max(copylen, csumlen) source bytes; the residue
                           beyond copylen is checksummed but not copied (ref :1266, :1314-1317) */
    uint32_t partial;   /* CRC mode: starting register; SUM mode: ignored (fresh state) */
    uint32_t reserved;  /* 0 */
} lampi_copy_desc;

/* Fused copy + checksum per descriptor: d[i].dst gets the first copylen bytes of d[i].src
 * (no other destination byte is written) and out[i] the checksum bcopy_uicrc / bcopy_uicsum
 * would return.  Every source byte is read from HBM once; the schedule follows the batch (one
 * wavefront per fragment, row groups joined by a second launch for long fragments, two IB-sized
 * fragments per wavefront; SUM one short-lived workgroup or one wavefront per fragment).
 * Replaces the per-fragment bcopy_uicrc/bcopy_uicsum of the send side
 * (src/path/gm/sendFrag.cc:147-155, ref src/util/MemFunctions.cc:1263-1321, 518-875) and
 * the receive-side CopyFunction (src/path/gm/recvFrag.h:165-205, copylen < crclen at :174).
 * mode LAMPI_CSUM_NONE: copies only (d_out unused, may be NULL). */
int lampi_frag_bcopy_batch(const lampi_copy_desc *d_descs, size_t n, uint32_t *d_out, int mode,
                           void *stream);

/* As lampi_frag_bcopy_batch, with checksum i written to (char *)d_out + i*out_stride (d_out and out_stride
 * 4-byte aligned, out_stride >= 4): the send step in place -- d_out = the first buffer's
 * gmHeaderData.dataChecksum (@64 of the 72-byte header, src/path/gm/header.h:56-70), out_stride = the buffer
 * size, as gmSendFragDesc::init stores it (src/path/gm/sendFrag.cc:149-151); other bytes of the records are
 * not touched.  out_stride != 4 uses 4 * n bytes of stream-ordered scratch and a second, small launch. */
int lampi_frag_bcopy_batch_strided(const lampi_copy_desc *d_descs, size_t n, void *d_out, size_t out_stride,
                                   int mode, void *stream);

/* Chained checksums over typemap pieces (non-contiguous datatypes).  Fragment f is the
 * concatenation of the checksummed ranges (max(copylen, csumlen) bytes at src) of pieces
 * d_pieces[d_first[f]] .. d_pieces[d_first[f+1] - 1], in that order (d_first: nfrags + 1
 * nondecreasing entries); each piece is also copied to its dst (copylen bytes, 0 = no copy).
 * out[f] = what the reference's piece-by-piece calls return: CRC mode the register threaded
 * through every piece from d_pieces[d_first[f]].partial (0xFFFFFFFF for a fragment with no
 * pieces; other pieces' partial is ignored), SUM mode the total of the increments with the
 * partial-word state threaded from a fresh state -- i.e. the checksum of the packed bytes.
 * Send side: gather into the payload, src/path/gm/sendFrag.cc:157-217 (also ib/sendFrag.cc:140-203,
 * quadrics/sendFrag.h:988-1051); receive side: scatter to the application buffer,
 * src/path/common/BaseDesc.cc:72-163.  Fragments up to 4 GiB - 1 bytes.  Uses
 * 8 * npieces bytes of stream-ordered scratch. */
int lampi_chain_csum_batch(const lampi_copy_desc *d_pieces, size_t npieces, const uint32_t *d_first,
                           size_t nfrags, uint32_t *d_out, int mode, void *stream);

/* As lampi_chain_csum_batch, with fragment f's checksum written to (char *)d_out + f*out_stride (as
 * lampi_frag_bcopy_batch_strided: the typemap send's `headerp->dataChecksum = csum`,
 * src/path/gm/sendFrag.cc:216).  mode LAMPI_CSUM_NONE: the pieces are copied, d_out is unused (may be NULL). */
int lampi_chain_csum_batch_strided(const lampi_copy_desc *d_pieces, size_t npieces, const uint32_t *d_first,
                                   size_t nfrags, void *d_out, size_t out_stride, int mode, void *stream);

/* Fragments a contiguous device-resident message like lampi_msg_csum and copies fragment k
 * to d_dst + k*dst_stride (dst_stride >= frag_len; e.g. frag_len for a plain copy, or the
 * slot size of a staging ring) with its checksum fused: bcopy_uicrc / bcopy_uicsum of every
 * fragment (copylen = crclen = the fragment length), ref src/path/gm/sendFrag.cc:147-155.
 * Source and destination must not overlap. */
int lampi_msg_bcopy(const void *d_msg, size_t msg_len, size_t frag_len, void *d_dst, size_t dst_stride,
                    uint32_t partial, uint32_t *d_out, int mode, void *stream);

/* As lampi_msg_bcopy, with fragment k's checksum written to (char *)d_out + k*out_stride (as
 * lampi_frag_bcopy_batch_strided): a GM send of one message into a ring of header + payload buffers is
 * d_dst = first buffer + 72, dst_stride = out_stride = the buffer size, d_out = first buffer + 64.
 * mode LAMPI_CSUM_NONE: copies only, d_out unused (may be NULL). */
int lampi_msg_bcopy_strided(const void *d_msg, size_t msg_len, size_t frag_len, void *d_dst, size_t dst_stride,
                            uint32_t partial, void *d_out, size_t out_stride, int mode, void *stream);

/* Fragments a contiguous device-resident message the way the path layer does
 * (fragment k = bytes [k*frag_len, min((k+1)*frag_len, msg_len)),
 * src/path/gm/path.cc:98-121) and writes ceil(msg_len/frag_len) checksums to d_out.
 * Every fragment starts from `partial` (CRC mode) or a fresh state (SUM mode).  Fragments of 64 B .. 2 KiB
 * (powers of two) in messages of at least 1 MiB from a 16-byte-aligned base are checksummed 64 / (frag_len / 64)
 * to a 4 KiB row of the uniform-batch kernel. */
int lampi_msg_csum(const void *d_msg, size_t msg_len, size_t frag_len, uint32_t partial,
                   uint32_t *d_out, int mode, void *stream);

/* ------------------------------------------------------------------------------------
 * Headers and receive-side verification (device-resident, batched).
 * Headers are n records of `stride` bytes starting at d_hdrs (d_hdrs, stride and
 * csum_offset 4-byte aligned).  Masks hold one bit per fragment, bit (i % 32) of word
 * i / 32, SET when fragment i FAILS; *d_nbad receives the number of failures.
 * ---------------------------------------------------------------------------------- */

/* out[i] = BasePath_t::headerChecksum(hdr_i, crclen, word_count)
 * (ref src/path/common/path.h:280-314): CRC mode the byte-swapped uicrc of the first crclen
 * bytes (so CRC(header || stored) == 0), SUM mode the sum of word_count 32-bit words.
 * Senders: src/path/gm/sendFrag.cc:218-225, gm/recvFrag.cc:125-130, quadrics/sendFrag.h:876-879. */
int lampi_header_csum_batch(const void *d_hdrs, size_t n, size_t stride, uint32_t crclen,
                            uint32_t word_count, uint32_t *d_out, int mode, void *stream);

/* As lampi_header_csum_batch, with header i's value written to (char *)d_out + i*out_stride (4-byte aligned):
 * the sender's `headerp->checksum = BasePath_t::headerChecksum(headerp, sizeof(gmHeader) - 4, GM_HDR_WORDS)`
 * in place (src/path/gm/sendFrag.cc:218-225) is d_out = d_hdrs + 68, out_stride = stride, crclen 68 -- run
 * after dataChecksum was stamped (lampi_frag_bcopy_batch_strided / lampi_msg_bcopy_strided on the same
 * stream).  Each header's bytes are read before its own word is written; d_out + i*out_stride must not lie
 * inside the checksummed bytes of another header.  mode LAMPI_CSUM_NONE: nothing is written. */
int lampi_header_csum_batch_strided(const void *d_hdrs, size_t n, size_t stride, uint32_t crclen,
                                    uint32_t word_count, void *d_out, size_t out_stride, int mode, void *stream);

/* Receiver header check (ref src/path/gm/path.cc:364-393): header i fails unless
 * CRC mode: uicrc(hdr_i, hdr_bytes) == 0 (the whole header including the stored checksum);
 * SUM mode: the sum of word_count words == 2 x the stored checksum at csum_offset. */
int lampi_header_check_batch(const void *d_hdrs, size_t n, size_t stride, uint32_t hdr_bytes,
                             uint32_t word_count, uint32_t csum_offset, uint32_t *d_mask,
                             uint32_t *d_nbad, int mode, void *stream);

/* The IB receiver's header check (ref src/path/ib/path.cc:652-680): header i fails unless the
 * 32-bit value stored at csum_offset (native byte order, NOT swapped) equals
 *   CRC mode: uicrc(hdr_i, crclen)     SUM mode: uicsum(hdr_i, crclen) (fresh state)
 * -- e.g. crclen 68 / csum_offset 68 for an ibDataHdr_t, crclen = length - 4 / csum_offset =
 * length - 4 for an ACK (ib/sendFrag.cc:306-314, :327-335).  The sender's side of it is
 * lampi_frag_csum_batch_strided over descriptors {hdr_i, crclen, CRC_INITIAL_REGISTER} with
 * d_out = d_hdrs + csum_offset and out_stride = stride. */
int lampi_header_compare_batch(const void *d_hdrs, size_t n, size_t stride, uint32_t crclen, uint32_t csum_offset,
                               uint32_t *d_mask, uint32_t *d_nbad, int mode, void *stream);

/* CheckData (ref src/path/gm/recvFrag.h:213-257): fragment i fails iff its length is nonzero
 * and d_calc[i] != its expected checksum.  Expected checksums and lengths are 32-bit values
 * read at d_expected + i*expected_stride and d_lengths + i*lengths_stride -- e.g. straight
 * from an array of gmHeaderData (dataChecksum @64, dataLength @20, stride = the record size).
 * d_lengths may be NULL (every length nonzero). */
int lampi_check_data_batch(const uint32_t *d_calc, const void *d_expected, size_t expected_stride,
                           const void *d_lengths, size_t lengths_stride, size_t n, uint32_t *d_mask,
                           uint32_t *d_nbad, void *stream);

/* One received fragment to deliver (32 bytes, little-endian): offset 0 frag, 8 app,
 * 16 app_len, 24 length, 28 reserved. */
typedef struct lampi_recv_desc {
    uint64_t frag;      /* device address of the received payload (BaseRecvFragDesc_t::addr_m) */
    uint64_t app;       /* device address it is delivered to: RecvDesc_t::addr_m + dataOffset() */
    int64_t  app_len;   /* room left in the posted buffer at that offset: posted_m.length_m - Offset
                           (ref BaseDesc.cc:307); may be <= 0 */
    uint32_t length;    /* bytes received, length_m; all of them are checksummed */
    uint32_t reserved;  /* 0 */
} lampi_recv_desc;

/* RecvDesc_t::CopyToApp for a batch of contiguous fragments, fused in one pass over the payload
 * (ref src/path/common/BaseDesc.cc:288-342, locked twin :380-434; GM hooks CopyFunction
 * src/path/gm/recvFrag.h:165-182 and CheckData :213-257; IB src/path/ib/recvFrag.cc:182-245):
 *   lengthToCopy = app_len <= 0 ? 0 : min(length, app_len);
 *   lengthToCopy > 0:  copy lengthToCopy bytes frag -> app, checksum all `length` bytes
 *                      (bcopy_uicrc / bcopy_uicsum with copylen < csumlen, the bytes past the
 *                      posted buffer go to the bit bucket) and compare with the expected value;
 *   lengthToCopy == 0: nothing copied or checksummed, DataOK (CopyFunction returns the CRC
 *                      initial register or 0, CheckData passes a zero length).
 * d_copied[i] = lengthToCopy, or -1 when the checksum differs (CopyToApp's return value);
 * d_csum[i] = the calculated checksum (what the reference logs as "calculated=");
 * the expected checksum of fragment i is the 32-bit value at d_expected + i*expected_stride (read
 * for every i, whatever its descriptor says) --
 * e.g. dataChecksum (@64) of an array of 72-byte gmHeaderData records (expected_stride 72).
 * d_mask: bit (i % 32) of word i / 32 set iff fragment i is corrupt (zeroed by the call);
 * *d_nbad: number of corrupt fragments.  The schedule follows the batch's shape (the rows hint
 * above, or the shape the stream's earlier batches showed): one wavefront per fragment, row groups
 * joined by a second launch, or two IB-sized fragments per wavefront (CRC) / one workgroup or one
 * wavefront per fragment (SUM); every payload byte is read from HBM once.  mode LAMPI_CSUM_NONE
 * (checksumming off): the lengthToCopy bytes copied (the SUM copy schedules), d_csum[i] = 0, every
 * fragment DataOK, d_expected may be NULL. */
int lampi_copy_to_app_batch(const lampi_recv_desc *d_descs, size_t n, const void *d_expected,
                            size_t expected_stride, int64_t *d_copied, uint32_t *d_csum, uint32_t *d_mask,
                            uint32_t *d_nbad, int mode, void *stream);

/* RecvDesc_t::CopyToApp's non-contiguous branch on the device (ref src/path/common/BaseDesc.cc:326-340 --
 * non_contiguous_copy :72-163 and CheckData gm/recvFrag.h:213-257): lampi_chain_csum_batch's pieces and
 * fragments (the typemap pieces of each received fragment: src in the received payload, dst in the
 * application buffer, copylen = csumlen) with the checksum started from CRC_INITIAL_REGISTER (the pieces'
 * partial is ignored; SUM from a fresh state) and compared with the 32-bit value at
 * d_expected + f*expected_stride:
 *   d_copied[f] = the bytes copied (len_copied), or -1 when that is nonzero and the checksum differs;
 *   d_csum[f] = the calculated checksum; d_mask / *d_nbad as lampi_copy_to_app_batch (zeroed by the call).
 * mode LAMPI_CSUM_NONE: copies only, d_csum 0, every fragment DataOK (d_expected may be NULL).
 * Uses 8 * npieces bytes of stream-ordered scratch. */
int lampi_chain_copy_to_app_batch(const lampi_copy_desc *d_pieces, size_t npieces, const uint32_t *d_first,
                                  size_t nfrags, const void *d_expected, size_t expected_stride, int64_t *d_copied,
                                  uint32_t *d_csum, uint32_t *d_mask, uint32_t *d_nbad, int mode, void *stream);

/* ------------------------------------------------------------------------------------
 * Utilities (bench/test support, device-side).
 * ---------------------------------------------------------------------------------- */

/* Fill d_dst[0..nbytes) with bytes [byte_off, byte_off + nbytes) of the synthetic
 * stream of SURVEY.md 8(d): word64[i] = splitmix64(seed + (i+1)*0x9E3779B97F4A7C15), LE. */
int lampi_fill_stream(void *d_dst, size_t nbytes, uint64_t seed, uint64_t byte_off,
                      void *stream);

/* Fragment-strided variant: fragment i of d_dst (frag_len bytes, frag_len % 8 == 0,
 * d_dst 8-byte aligned) holds stream bytes [(k0 + i*kstep)*frag_len, +frag_len), i < n --
 * the round-robin shard (k = k0 + i*kstep) of a global batch of frag_len-byte fragments. */
int lampi_fill_stream_frags(void *d_dst, size_t n, size_t frag_len, uint64_t seed, uint64_t k0,
                            uint64_t kstep, void *stream);

/* Release the calling thread's staging resources of the host entry points (streams, device
 * buffers, pinned bounce buffer) and its device scratch of the batched entry points.  They are also released automatically when the thread exits
 * or switches to another device; the next host call on the thread allocates them again. */
void lampi_host_release(void);

/* Bytes of page-locked host memory the library's host paths hold right now, over all threads
 * (bounce buffers, result words, staging): a leak check for callers with short-lived threads. */
int64_t lampi_host_pinned_bytes(void);

/* Bytes of device scratch the library holds right now, over all threads (the per-thread, per-stream
 * buffers of the row-group joins and byte plans): freed at thread exit and by lampi_host_release(). */
int64_t lampi_device_scratch_bytes(void);

/* Version string of the engine and the gfx target it was built for. */
const char *lampi_csum_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LAMPI_CSUM_H */
