#!/usr/bin/env bash
# sum_copy_wg_kernel for every SUM fused copy (unaligned destinations included): parity, then
# A/B against ab/prev.so (the one-fragment-per-wave sum_rows_kernel) by fragment size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sumwg2
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
for v in prod; do
  if [ $v = prod ]; then L=lampi_amd/liblampi_csum.so; else L=ab/$v.so; fi
  LAMPI_CSUM_LIB=$L step sizes_${v} 300 python tools/microbench/sum_copy_sizes.py
done
step bcopy_sum_prod 200 python bench.py --bcopy --mode sum --steps 10 --no-cpu-baseline
step recv_sum_prod 200 python bench.py --recv --mode sum --steps 10 --no-cpu-baseline
echo "=== done $(date +%T)"
