#!/usr/bin/env bash
# Final SUM copy check: the full GPU suite, then the SUM copy bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sumwg3
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!!! $name rc=$rc"; tail -30 "$O/$name.log"; exit $rc; fi
  grep -E '^L=|passed|failed' "$O/$name.log" | cut -c1-300
}
step tests 700 python -u -m pytest tests/test_gpu_bcopy.py tests/test_gpu_recv.py tests/test_gpu_native.py tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread
step sizes 300 python tools/microbench/sum_copy_sizes.py
step bcopy_sum 200 python bench.py --bcopy --mode sum --steps 10 --no-cpu-baseline
step bcopy_crc 200 python bench.py --bcopy --mode crc --steps 10 --no-cpu-baseline
step recv_sum 200 python bench.py --recv --mode sum --steps 10 --no-cpu-baseline
step recv_crc 200 python bench.py --recv --mode crc --steps 10 --no-cpu-baseline
step slots 200 python tools/microbench/msg_bcopy_slots.py
echo "=== done $(date +%T)"
