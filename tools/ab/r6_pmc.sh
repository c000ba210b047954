#!/usr/bin/env bash
# Round 6 PMC passes (rocprofv3 --pmc, one counter group per pass, own runs; MI355X_MICROARCH.md HBM section):
# FETCH_SIZE / WRITE_SIZE of the fused copies (bench.py --bcopy, both modes: replaces traffic.json's r02/r03 lines),
# the packed-row messages (1 KiB x 1M, 64 B x 16M), config C (CRC: FETCH_SIZE, SQ VALU / LDS instructions) and the
# receive-shape copy microbenchmark (tools/microbench/recv_ceiling).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc6
pass() {  # tag counters... -- command
  local tag=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  local name="${tag}_${ctr[0]}"
  timeout -s KILL 150 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d "gpurun_out/pmc6/$name" -o run -- "$@" \
    > "gpurun_out/pmc6/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
B="--steps 5 --warmup 3 --no-cpu-baseline"
pass bcopy_crc FETCH_SIZE -- python3 bench.py --bcopy $B
pass bcopy_crc WRITE_SIZE -- python3 bench.py --bcopy $B
pass bcopy_sum FETCH_SIZE -- python3 bench.py --bcopy --mode sum $B
pass bcopy_sum WRITE_SIZE -- python3 bench.py --bcopy --mode sum $B
pass packedA_crc FETCH_SIZE -- python3 bench.py --frags 1048576 --frag-bytes 1024 --seed 1 $B
pass packed64_crc FETCH_SIZE -- python3 bench.py --frags 16777216 --frag-bytes 64 $B
pass packed64_crc WRITE_SIZE -- python3 bench.py --frags 16777216 --frag-bytes 64 $B
pass configC FETCH_SIZE -- python3 bench.py --config C --steps 5 --warmup 3
pass configC SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES -- python3 bench.py --config C --steps 5 --warmup 3
pass recvceil FETCH_SIZE -- tools/microbench/recv_ceiling
pass recvceil WRITE_SIZE -- tools/microbench/recv_ceiling
echo done
