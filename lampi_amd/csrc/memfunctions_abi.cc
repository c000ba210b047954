// memfunctions_abi.cc -- the reference's C++ checksum ABI, exported by liblampi_csum.so.
//
// LA-MPI declares its checksums as overloaded C++ free functions (ref src/util/MemFunctions.h:43-65)
// and links them from MemFunctions.o.  This file defines the same twelve overloads out of line, so
// the library exports their mangled names (_Z5uicrcPKvmj, _Z11bcopy_uicrcPKvPvmm, ...): libmpi can
// drop MemFunctions.o and link -llampi_csum without recompiling a caller.  include/lampi/MemFunctions.h
// declares them with the reference's prototypes.  Each one is the C entry point with the reference's
// defaults: CRC_INITIAL_REGISTER, or a fresh (0, 0) partial-word state.  The other two functions of
// MemFunctions.o are here too, so the object can be dropped whole: ulm_initialize_crc_table and
// poisonMemory (MemFunctions.cc:1242-1261, :1380-1393).
#include <sys/types.h>

#include "../../include/lampi/MemFunctions.h"
#include "host_internal.h"

unsigned int uicrc(const void *source, unsigned long crclen, unsigned int partial_crc) {
    return lampi_uicrc(source, crclen, partial_crc);
}

unsigned int uicrc(const void *source, unsigned long crclen) {
    return lampi_uicrc(source, crclen, CRC_INITIAL_REGISTER);
}

unsigned int bcopy_uicrc(const void *source, void *destination, unsigned long copylen, unsigned long crclen,
                         unsigned int partial_crc) {
    return lampi_bcopy_uicrc(source, destination, copylen, crclen, partial_crc);
}

unsigned int bcopy_uicrc(const void *source, void *destination, unsigned long copylen, unsigned long crclen) {
    return lampi_bcopy_uicrc(source, destination, copylen, crclen, CRC_INITIAL_REGISTER);
}

unsigned int uicsum(const void *source, unsigned long csumlen, unsigned int *lastPartialInt,
                    unsigned int *lastPartialLength) {
    return lampi_uicsum(source, csumlen, lastPartialInt, lastPartialLength);
}

unsigned int uicsum(const void *source, unsigned long csumlen) {
    unsigned int pint = 0, plen = 0;
    return lampi_uicsum(source, csumlen, &pint, &plen);
}

unsigned int bcopy_uicsum(const void *source, void *destination, unsigned long copylen, unsigned long csumlen,
                          unsigned int *lastPartialInt, unsigned int *lastPartialLength) {
    return lampi_bcopy_uicsum(source, destination, copylen, csumlen, lastPartialInt, lastPartialLength);
}

unsigned int bcopy_uicsum(const void *source, void *destination, unsigned long copylen, unsigned long csumlen) {
    unsigned int pint = 0, plen = 0;
    return lampi_bcopy_uicsum(source, destination, copylen, csumlen, &pint, &plen);
}

unsigned long csum(const void *source, unsigned long csumlen, unsigned long *lastPartialLong,
                   unsigned long *lastPartialLength) {
    return lampi_csum(source, csumlen, lastPartialLong, lastPartialLength);
}

unsigned long csum(const void *source, unsigned long csumlen) {
    unsigned long plong = 0, plen = 0;
    return lampi_csum(source, csumlen, &plong, &plen);
}

unsigned long bcopy_csum(const void *source, void *destination, unsigned long copylen, unsigned long csumlen,
                         unsigned long *lastPartialLong, unsigned long *lastPartialLength) {
    return lampi_bcopy_csum(source, destination, copylen, csumlen, lastPartialLong, lastPartialLength);
}

unsigned long bcopy_csum(const void *source, void *destination, unsigned long copylen, unsigned long csumlen) {
    unsigned long plong = 0, plen = 0;
    return lampi_bcopy_csum(source, destination, copylen, csumlen, &plong, &plen);
}

// ref MemFunctions.cc:1242-1261 fills a process-global table on first use (racy, :1271-1273).  Here
// the table image is per device and built on first use anyway; calling this builds it for the
// calling thread's current device up front.  No GPU: abort, as every host entry point does.
void ulm_initialize_crc_table() {
    int dev = 0;
    hipError_t e = lampi::current_device(&dev);
    const uint32_t *img = nullptr;
    if (e == hipSuccess) e = lampi::device_tables(dev, &img);
    if (e != hipSuccess) lampi::die("ulm_initialize_crc_table", e);
}

// ref MemFunctions.cc:1380-1393 (declared in src/util/Utility.h:45): a debugging fill of
// lenInBytes / sizeof(int) ints with `pattern`.  Not a checksum; a plain host loop, like the reference's.
void poisonMemory(void *ptr, ssize_t lenInBytes, int pattern) {
    int *p = static_cast<int *>(ptr);
    for (ssize_t i = 0, n = lenInBytes / (ssize_t)sizeof(int); i < n; ++i) p[i] = pattern;
}
