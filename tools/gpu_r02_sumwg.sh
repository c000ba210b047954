#!/usr/bin/env bash
# SUM fused copies on sum_copy_wg_kernel: parity (bcopy/recv/chain tests), then A/B against the
# previous commit's library (ab/prev.so): descriptors, receive step, message slots.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sumwg
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!!! $name rc=$rc"; tail -30 "$O/$name.log"; exit $rc; fi
  grep -E '^L=|passed|failed' "$O/$name.log" | cut -c1-300
}
step tests 400 python -u -m pytest tests/test_gpu_bcopy.py tests/test_gpu_recv.py tests/test_gpu_chain.py tests/test_gpu_native.py -x -q --timeout 200 --timeout-method thread
for r in 1 2; do
  for v in prev prod; do
    if [ $v = prod ]; then L=lampi_amd/liblampi_csum.so; else L=ab/$v.so; fi
    LAMPI_CSUM_LIB=$L step bcopy_sum_${v}_$r 200 python bench.py --bcopy --mode sum --steps 10 --no-cpu-baseline
    LAMPI_CSUM_LIB=$L step recv_sum_${v}_$r 200 python bench.py --recv --mode sum --steps 10 --no-cpu-baseline
    LAMPI_CSUM_LIB=$L step slots_${v}_$r 200 python tools/microbench/msg_bcopy_slots.py
  done
done
echo "=== done $(date +%T)"
