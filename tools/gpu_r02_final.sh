#!/usr/bin/env bash
# Round-2 final session on the final tree: GPU tests, smoke, every bench line DESIGN.md quotes,
# the rocprof kernel trace/stats of the default bench, and the PMC passes (one counter per run,
# no trace domains) for profiles/traffic.json.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!!! $name rc=$rc"; tail -20 "$O/$name.log"; exit $rc; fi
  grep -E '^\{|passed|failed|smoke' "$O/$name.log" | tail -1 | cut -c1-200
}
pass() {  # name counter bench-args...
  local name=$1 ctr=$2; shift 2
  echo "=== pmc $name $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_$name -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/pmc_$name.log 2>&1 || { echo "!!! pmc $name"; tail $O/pmc_$name.log; exit 1; }
}
step gputest 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step bench_sum 300 python bench.py --mode sum --no-cpu-baseline
step bench_16k 300 python bench.py --frags 1048576 --frag-bytes 16384 --no-cpu-baseline
step bench_desc 300 python bench.py --desc --no-cpu-baseline
step bench_C 300 python bench.py --config C --steps 50
step bench_C_sum 300 python bench.py --config C --mode sum --steps 50
step bench_D_shard0 300 python bench.py --config D --shard 0 --steps 10
step bench_D_shard7 300 python bench.py --config D --shard 7 --steps 10 --mode sum
step bcopy_crc 300 python bench.py --bcopy --steps 10
step bcopy_sum 300 python bench.py --bcopy --mode sum --steps 10
step recv_crc 300 python bench.py --recv --steps 10
step recv_sum 300 python bench.py --recv --mode sum --steps 10
step e2e 300 python bench.py --e2e
step slots 200 python tools/microbench/msg_bcopy_slots.py
step latency 300 python bench.py --latency
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --no-cpu-baseline
pass bench_fetch FETCH_SIZE
pass bcs_fetch FETCH_SIZE --bcopy --mode sum
pass bcs_write WRITE_SIZE --bcopy --mode sum
pass bcc_fetch FETCH_SIZE --bcopy
pass bcc_write WRITE_SIZE --bcopy
pass rvs_fetch FETCH_SIZE --recv --mode sum
pass rvs_write WRITE_SIZE --recv --mode sum
echo "=== done $(date +%T)"
