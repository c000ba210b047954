/*
 * lampi/MemFunctions.h -- drop-in replacement for LA-MPI's src/util/MemFunctions.h
 * (ref src/util/MemFunctions.h:31-65).  Restores the reference's C++ overload names and
 * signatures on top of the C ABI of liblampi_csum.so, so src/path compiles unchanged:
 *
 *     #include "util/MemFunctions.h"   ->   #include "lampi/MemFunctions.h"
 *     link:  -L<repo>/lampi_amd -llampi_csum
 *
 * All twelve overloads are provided: the 32-bit uicrc/bcopy_uicrc/uicsum/bcopy_uicsum (the
 * only ones with callers in src/) and the 64-bit csum/bcopy_csum
 * (MemFunctions.h:43-50, no path caller).
 */
#ifndef LAMPI_DROPIN_MEMFUNCTIONS_H
#define LAMPI_DROPIN_MEMFUNCTIONS_H

#include "../lampi_csum.h"

#ifndef CRC_POLYNOMIAL
#define CRC_POLYNOMIAL ((unsigned int)LAMPI_CRC_POLYNOMIAL)             /* MemFunctions.h:36 */
#endif
#ifndef CRC_INITIAL_REGISTER
#define CRC_INITIAL_REGISTER ((unsigned int)LAMPI_CRC_INITIAL_REGISTER) /* MemFunctions.h:37 */
#endif

#ifdef __cplusplus

inline unsigned int uicrc(const void *source, unsigned long crclen, unsigned int partial_crc) {
    return lampi_uicrc(source, crclen, partial_crc);
}
inline unsigned int uicrc(const void *source, unsigned long crclen) {
    return lampi_uicrc(source, crclen, CRC_INITIAL_REGISTER);
}
inline unsigned int bcopy_uicrc(const void *source, void *destination, unsigned long copylen,
                                unsigned long crclen, unsigned int partial_crc) {
    return lampi_bcopy_uicrc(source, destination, copylen, crclen, partial_crc);
}
inline unsigned int bcopy_uicrc(const void *source, void *destination, unsigned long copylen,
                                unsigned long crclen) {
    return lampi_bcopy_uicrc(source, destination, copylen, crclen, CRC_INITIAL_REGISTER);
}
inline unsigned int uicsum(const void *source, unsigned long csumlen, unsigned int *lastPartialInt,
                           unsigned int *lastPartialLength) {
    return lampi_uicsum(source, csumlen, lastPartialInt, lastPartialLength);
}
inline unsigned int uicsum(const void *source, unsigned long csumlen) {
    unsigned int pint = 0, plen = 0;
    return lampi_uicsum(source, csumlen, &pint, &plen);
}
inline unsigned int bcopy_uicsum(const void *source, void *destination, unsigned long copylen,
                                 unsigned long csumlen, unsigned int *lastPartialInt,
                                 unsigned int *lastPartialLength) {
    return lampi_bcopy_uicsum(source, destination, copylen, csumlen, lastPartialInt, lastPartialLength);
}
inline unsigned int bcopy_uicsum(const void *source, void *destination, unsigned long copylen,
                                 unsigned long csumlen) {
    unsigned int pint = 0, plen = 0;
    return lampi_bcopy_uicsum(source, destination, copylen, csumlen, &pint, &plen);
}
// 64-bit additive checksums (MemFunctions.h:43-50; no path caller in the reference)
inline unsigned long csum(const void *source, unsigned long csumlen, unsigned long *lastPartialLong,
                          unsigned long *lastPartialLength) {
    return lampi_csum(source, csumlen, lastPartialLong, lastPartialLength);
}
inline unsigned long csum(const void *source, unsigned long csumlen) {
    unsigned long plong = 0, plen = 0;
    return lampi_csum(source, csumlen, &plong, &plen);
}
inline unsigned long bcopy_csum(const void *source, void *destination, unsigned long copylen, unsigned long csumlen,
                                unsigned long *lastPartialLong, unsigned long *lastPartialLength) {
    return lampi_bcopy_csum(source, destination, copylen, csumlen, lastPartialLong, lastPartialLength);
}
inline unsigned long bcopy_csum(const void *source, void *destination, unsigned long copylen,
                                unsigned long csumlen) {
    unsigned long plong = 0, plen = 0;
    return lampi_bcopy_csum(source, destination, copylen, csumlen, &plong, &plen);
}

#endif /* __cplusplus */
#endif /* LAMPI_DROPIN_MEMFUNCTIONS_H */
