/*
 * lampi/MemFunctions.h -- drop-in replacement for LA-MPI's src/util/MemFunctions.h
 * (ref src/util/MemFunctions.h:31-65).  Declares the reference's twelve C++ overloads with its
 * own prototypes; liblampi_csum.so defines them (lampi_amd/csrc/memfunctions_abi.cc) and
 * exports their mangled names, so either
 *
 *     #include "util/MemFunctions.h"   ->   #include "lampi/MemFunctions.h"     (recompile), or
 *     keep the reference header and replace MemFunctions.o with -llampi_csum    (relink only)
 *
 *     link:  -L<repo>/lampi_amd -llampi_csum
 *
 * All twelve overloads are provided: the 32-bit uicrc/bcopy_uicrc/uicsum/bcopy_uicsum (the
 * only ones with callers in src/) and the 64-bit csum/bcopy_csum
 * (MemFunctions.h:43-50, no path caller).  C callers use the
 * lampi_* entry points of lampi_csum.h directly.
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

/* 64-bit additive checksums (MemFunctions.h:43-50; no path caller in the reference) */
unsigned long bcopy_csum(const void *source, void *destination, unsigned long copylen, unsigned long csumlen);
unsigned long bcopy_csum(const void *source, void *destination, unsigned long copylen, unsigned long csumlen,
                         unsigned long *lastPartialLong, unsigned long *lastPartialLength);
unsigned long csum(const void *source, unsigned long csumlen);
unsigned long csum(const void *source, unsigned long csumlen, unsigned long *lastPartialLong,
                   unsigned long *lastPartialLength);

/* 32-bit additive checksums (MemFunctions.h:52-59) */
unsigned int bcopy_uicsum(const void *source, void *destination, unsigned long copylen, unsigned long csumlen);
unsigned int bcopy_uicsum(const void *source, void *destination, unsigned long copylen, unsigned long csumlen,
                          unsigned int *lastPartialInt, unsigned int *lastPartialLength);
unsigned int uicsum(const void *source, unsigned long csumlen);
unsigned int uicsum(const void *source, unsigned long csumlen, unsigned int *lastPartialInt,
                    unsigned int *lastPartialLength);

/* CRC-32 (MemFunctions.h:60-65) */
unsigned int bcopy_uicrc(const void *source, void *destination, unsigned long copylen, unsigned long crclen);
unsigned int bcopy_uicrc(const void *source, void *destination, unsigned long copylen, unsigned long crclen,
                         unsigned int partial_crc);
unsigned int uicrc(const void *source, unsigned long crclen, unsigned int partial_crc);
unsigned int uicrc(const void *source, unsigned long crclen);

/* The rest of the reference's MemFunctions.o, so the object can be replaced whole at link time:
 * ulm_initialize_crc_table (MemFunctions.cc:1242-1261; here: build the current device's tables now)
 * and poisonMemory (MemFunctions.cc:1380-1393, declared in src/util/Utility.h:45). */
void ulm_initialize_crc_table();
void poisonMemory(void *ptr, long lenInBytes, int pattern);

#endif /* __cplusplus */
#endif /* LAMPI_DROPIN_MEMFUNCTIONS_H */
