// host_internal.h -- helpers shared by the C-ABI translation units of liblampi_csum.so (internal).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace lampi {

// The calling thread's current device, range-checked against the per-device table slots.
hipError_t current_device(int *dev);
// The per-device table image (built once per process, uploaded once per device).
hipError_t device_tables(int dev, const uint32_t **out);

// Checksums of the fragments of a contiguous device-resident message (lampi_msg_csum's kernel
// choice: the regular kernel for whole-4-KiB-row fragments at a 16-byte-aligned base, the piece
// streams otherwise).  n = number of fragments, >= 1.
hipError_t launch_msg_csum(const uint8_t *base, size_t msg_len, size_t frag_len, uint32_t partial, uint32_t *out,
                           int mode, int dev, const uint32_t *img, hipStream_t s);

// Pinned host memory held by the library's own staging (all threads), for leak checks
// (lampi_host_pinned_bytes).  Every hipHostMalloc of the host paths goes through these two.
hipError_t pinned_alloc(void **p, size_t bytes, unsigned flags);
void pinned_free(void *p, size_t bytes);

// The host-message pipeline's per-thread state (host_msg.cc), released with the rest of the
// thread's staging by lampi_host_release() and at thread exit.
void release_pipeline();

[[noreturn]] void die(const char *what, hipError_t e);

}  // namespace lampi
