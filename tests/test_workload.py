"""Host-side workload generators and the committed bench digests (CPU)."""
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(__file__), "golden")


def test_zipf_lengths_match_oracle_and_fixture(oracle):
    from lampi_amd.workload import zipf_lengths

    with open(os.path.join(GOLDEN_DIR, "fixtures.json")) as f:
        gold = json.load(f)["digests"]["C"]
    lens = zipf_lengths(4 << 30)
    assert lens.size == gold["n"] and int(lens.sum(dtype=np.uint64)) == gold["total_bytes"]
    assert np.array_equal(lens, oracle.zipf_lengths(4 << 30))
    for m in (0, 1, 64, 65, 99999, 1 << 24):
        assert np.array_equal(zipf_lengths(m), oracle.zipf_lengths(m)), m


def test_bench_digests_consistent_with_baseline(oracle):
    """bench.py's committed digests: config B, and a small entry recomputed."""
    with open(os.path.join(GOLDEN_DIR, "bench_digests.json")) as f:
        entries = {(e["seed"], e["n_total"], e["frag_bytes"], e["mode"]): (e["xor"], e["wsum"])
                   for e in json.load(f)["entries"]}
    assert entries[(2, 4194304, 4096, "crc")] == (0x959621BB, 0xC38D8899)
    assert entries[(2, 4194304, 4096, "sum")][1] == 0x88569035  # BASELINE.md SUM WSUM
    assert entries[(1, 1048576, 1024, "crc")] == (0xFEB61101, 0x41FADF13)
    assert entries[(1, 1048576, 1024, "crc")] == oracle.uniform_digest(1, 1048576, 1024, 0)
    for n in (8388608, 16777216, 33554432):
        assert (2, n, 4096, "crc") in entries


def test_bench_golden_lookup():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(GOLDEN_DIR), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.golden_digest(2, 4194304, 4096, True) == (0x959621BB, 0xC38D8899)
    assert bench.golden_digest(2, 33554432, 4096, True) is not None
    assert bench.golden_digest(2, 4194304, 4096, False) is not None
    assert bench.golden_digest(9, 17, 4096, True) is None
