"""Synthetic workloads of SURVEY.md 8(d) on the host side (bench support, not the checksum path).

The payload bytes themselves are generated on the device (`device.fill_stream`); this module
holds the one host-side generator the configs need: the config C fragment lengths.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def mix64(z: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    z = z ^ (z >> np.uint64(30))
    z = z * np.uint64(0xBF58476D1CE4E5B9)
    z = z ^ (z >> np.uint64(27))
    z = z * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _zipf_cdf() -> np.ndarray:
    """cdf[r], r = 0..1024, of Zipf(s = 1.1) over ranks 1..1024, summed in rank order."""
    p = np.power(np.arange(1, 1025, dtype=np.float64), -1.1)
    z = 0.0
    for v in p:  # sequential double sum, as specified
        z += float(v)
    cdf = np.empty(1025, dtype=np.float64)
    cdf[0] = 0.0
    acc = 0.0
    for r in range(1, 1025):
        acc += float(p[r - 1]) / z
        cdf[r] = acc
    cdf[1024] = 1.0
    return cdf


def zipf_lengths(min_total: int) -> np.ndarray:
    """Config C fragment lengths: L_k = 64 * r_k, r_k the smallest rank with cdf[r] > u_k,
    u_k = (mix64(0x5A1F + k) >> 11) / 2^53; fragments are taken until the total reaches
    min_total bytes."""
    cdf = _zipf_cdf()
    out = []
    total = 0
    k0 = 0
    chunk = 1 << 18
    while total < min_total:
        k = np.arange(k0, k0 + chunk, dtype=np.uint64)
        u = (mix64(np.uint64(0x5A1F) + k) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
        r = np.searchsorted(cdf[1:], u, side="right") + 1  # smallest r with cdf[r] > u
        lens = (64 * np.minimum(r, 1024)).astype(np.uint32)
        csum = total + np.cumsum(lens, dtype=np.uint64)
        stop = int(np.searchsorted(csum, np.uint64(min_total), side="left"))
        if stop < chunk:
            out.append(lens[:stop + 1])
            total = int(csum[stop])
            break
        out.append(lens)
        total = int(csum[-1])
        k0 += chunk
    return np.concatenate(out) if out else np.empty(0, np.uint32)
