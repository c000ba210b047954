#!/usr/bin/env bash
# SQ counters of crc_list_kernel against the piece streams and the regular kernel (4 KiB descriptors,
# config B through descriptors, and config C).  Usage: tools/gpu_r03_pmc_list.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_list
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"
P2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
run() {  # name, kernel choice, bench args
  local name=$1 k=$2
  shift 2
  export LAMPI_DESC_KERNEL=$k
  timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/pmc_list/$name.1 -o pmc -- python3 bench.py "$@" --steps 5 --warmup 3 --no-cpu-baseline > /dev/null 2>&1 || return 1
  timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/pmc_list/$name.2 -o pmc -- python3 bench.py "$@" --steps 5 --warmup 3 --no-cpu-baseline > /dev/null 2>&1 || return 1
}
run desc_list list --desc && run desc_stream stream --desc && run B_regular stream && run C_list list --config C && run C_stream stream --config C
