#!/usr/bin/env bash
# Round 6, final library: FETCH_SIZE / WRITE_SIZE and SQ instruction counts of config B's kernel (crc_regular_kernel,
# messages) and of config B as descriptors (crc_regular_kernel<kDesc>), own passes (MI355X_MICROARCH.md HBM section);
# outputs gpurun_out/pmc6b/ -> profiles/r06/pmc/B6_*.csv, desc6_*.csv (tools/ab/r6_traffic.py reads them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc6b
pass() {
  local tag=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  local name="${tag}_${ctr[0]}"
  timeout -s KILL 150 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d "gpurun_out/pmc6b/$name" -o run -- "$@" \
    > "gpurun_out/pmc6b/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  cp "gpurun_out/pmc6b/$name/run_counter_collection.csv" "gpurun_out/pmc6b/$name.csv"
}
B="--steps 5 --warmup 3 --no-cpu-baseline"
pass B6 FETCH_SIZE -- python3 bench.py $B
pass B6 WRITE_SIZE -- python3 bench.py $B
pass B6 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -- python3 bench.py $B
pass desc6 FETCH_SIZE -- python3 bench.py --desc $B --warmup 20
echo done
