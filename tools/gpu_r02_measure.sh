#!/usr/bin/env bash
# Round-2 measurement session: every bench line DESIGN.md quotes, on one box, plus the rocprof
# kernel trace/stats and the FETCH_SIZE pass of the default bench.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02
mkdir -p $O
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!!! $name rc=$rc"; tail -20 "$O/$name.log"; exit $rc; fi
  grep '^{' "$O/$name.log" | tail -1 | cut -c1-400
}
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
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --no-cpu-baseline
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
step pmc_fetch_C 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_C -o run -- python3 bench.py --config C --steps 5 --warmup 1
echo "=== done $(date +%T)"
