# Round-5 PMC passes (one counter group per run, rocprofv3 --pmc alone): current receive / copy / SUM kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmc5
export TMPDIR=/tmp
pass() {  # name counter args...
  local name=$1 ctr=$2; shift 2
  echo "== $name $ctr"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc5/${name}_$ctr -o run -- python3 bench.py "$@" > gpurun_out/pmc5/${name}_$ctr.log 2>&1 || { echo "FAIL $name $ctr"; tail -5 gpurun_out/pmc5/${name}_$ctr.log; exit 1; }
}
pass recvB_crc FETCH_SIZE --recv --steps 5 --warmup 3 &&
pass recvB_crc WRITE_SIZE --recv --steps 5 --warmup 3 &&
pass recvB_sum FETCH_SIZE --recv --mode sum --steps 5 --warmup 3 &&
pass recvB_sum WRITE_SIZE --recv --mode sum --steps 5 --warmup 3 &&
pass recvGM_crc FETCH_SIZE --recv --frags 16384 --frag-bytes 65456 --steps 5 --warmup 40 &&
pass recvGM_crc WRITE_SIZE --recv --frags 16384 --frag-bytes 65456 --steps 5 --warmup 40 &&
pass recvGM_sum FETCH_SIZE --recv --mode sum --frags 16384 --frag-bytes 65456 --steps 5 --warmup 40 &&
pass recvGM_sum WRITE_SIZE --recv --mode sum --frags 16384 --frag-bytes 65456 --steps 5 --warmup 40 &&
pass descB_crc FETCH_SIZE --desc --no-cpu-baseline --steps 5 --warmup 3 &&
pass msgB_sum FETCH_SIZE --mode sum --no-cpu-baseline --steps 5 --warmup 3 &&
pass bcopyB FETCH_SIZE --bcopy --steps 3 --warmup 3 &&
pass bcopyB WRITE_SIZE --bcopy --steps 3 --warmup 3 &&
echo "== pmc5 done"
