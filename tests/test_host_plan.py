"""CPU: the host paths' DMA planner (lampi_amd/csrc/host_plan.h), executed on the CPU.

tests/native/plan_check.cc plans random batches -- NIC-ring fragments under the ring rules (GM's
65,456-byte payloads, 4 KiB payloads in 64 KiB slots, ragged IB payloads with truncated and skipped
deliveries, shuffled fragments) and typemap pieces under the strict rules (strided vectors gathered and
scattered, random misaligned pieces with fragment boundaries) -- and runs every planned transfer as a
memcpy: sources must arrive at their chunk offsets, destinations must receive exactly their bytes, no
transfer may read outside what the rules allow, chunks must respect their capacity and boundaries, and
the layouts that coalesce must come out as one transfer per direction.  No GPU and no library involved.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_planner_executes_exactly():
    exe = os.path.join(HERE, "native", "plan_check")
    assert os.path.exists(exe), "run __graft_entry__.build() (make -C tests/native)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert lines[-1] == "bad 0 done"
    assert all(ln.endswith(" ok") for ln in lines[:-1]) and len(lines) > 60
    # coalescing: a dense GM ring and strided vectors move in one transfer per direction
    one = [ln for ln in lines if ln.startswith(("ring_gm_dense ", "ring_4k_pitch", "vector_gather_E", "vector_scatter_E"))]
    assert one and all(" h2d 1 d2h 1 " in ln + " " for ln in one), one
