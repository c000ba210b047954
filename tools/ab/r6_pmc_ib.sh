#!/usr/bin/env bash
# Round 6: instruction counts of IB's receive step (262,144 x 1,976 B, crc_light_pair_copy_kernel<RecvSource>, two
# fragments per wave) and of config B's kernel for comparison -- SQ counters in their own passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_ib
pass() {
  local tag=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  timeout -s KILL 150 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d "gpurun_out/pmc_ib/$tag" -o run -- "$@" \
    > "gpurun_out/pmc_ib/$tag.log" 2>&1
  local rc=$?
  echo "$tag rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
R="--recv --frags 262144 --frag-bytes 1976 --steps 5 --warmup 10"
pass ib_sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH -- python3 bench.py $R
pass ib_sq2 SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -- python3 bench.py $R
pass B_sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline
echo done
