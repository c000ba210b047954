#!/usr/bin/env bash
# Round 6 final session on the product library (liblampi_csum.so, no A/B knobs): the GPU suite, smoke, the bench lines
# the round's records quote, and kernel traces of config B, config C and config A's shape.  Outputs under
# gpurun_out/final6/ (copied to profiles/r06/final/).  Any failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/final6
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit=$rc"; tail -n 3 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || { echo "!!! $name failed: stopping"; exit $rc; }
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_B 600 python bench.py
step bench_B_sum 300 python bench.py --mode sum --no-cpu-baseline
step bench_C 300 python bench.py --config C --steps 50
step bench_C_sum 300 python bench.py --config C --mode sum --steps 50
step bench_A_msg 300 python bench.py --frags 1048576 --frag-bytes 1024 --seed 1 --no-cpu-baseline
step bench_A_msg_sum 300 python bench.py --frags 1048576 --frag-bytes 1024 --seed 1 --mode sum --no-cpu-baseline
step bench_A_desc 300 python bench.py --desc --frags 1048576 --frag-bytes 1024 --seed 1 --warmup 30 --no-cpu-baseline
step bench_64_msg 300 python bench.py --frags 16777216 --frag-bytes 64 --no-cpu-baseline
step bench_64_msg_sum 300 python bench.py --frags 16777216 --frag-bytes 64 --mode sum --no-cpu-baseline
step bench_64_desc 300 python bench.py --desc --frags 16777216 --frag-bytes 64 --warmup 30 --no-cpu-baseline
step bench_64_desc_sum 300 python bench.py --desc --frags 16777216 --frag-bytes 64 --mode sum --warmup 30 --no-cpu-baseline
step bench_desc4k 300 python bench.py --desc --warmup 30 --no-cpu-baseline
step bench_recv_gm 300 python bench.py --recv --frags 16384 --frag-bytes 65456
step bench_recv_gm_sum 300 python bench.py --recv --frags 16384 --frag-bytes 65456 --mode sum
step bench_recv_ib 300 python bench.py --recv --frags 262144 --frag-bytes 1976 --warmup 30
step bench_recv_ib_sum 300 python bench.py --recv --frags 262144 --frag-bytes 1976 --mode sum --warmup 30
step bench_B_1g 300 python bench.py --frags 262144 --no-cpu-baseline
step bench_bcopy 300 python bench.py --bcopy --steps 10
step bench_bcopy_sum 300 python bench.py --bcopy --mode sum --steps 10
step bench_e2e 300 python bench.py --e2e
step prof_B 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_B -o run -- python3 bench.py --steps 20 --no-cpu-baseline
step prof_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_C -o run -- python3 bench.py --config C --steps 20
step prof_A 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_A -o run -- python3 bench.py --frags 1048576 --frag-bytes 1024 --seed 1 --steps 20 --no-cpu-baseline
echo "final session done"
