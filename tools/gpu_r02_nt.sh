#!/usr/bin/env bash
# A/B of the copy kernels: head.so (before: one fragment per wave SUM copy, cached stores),
# nont.so (row-per-workgroup SUM copy, cached stores), product (row-per-workgroup + nt stores).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/nt
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "!!! $name rc=$rc"; tail -20 "$O/$name.log"; exit $rc; fi
  grep -E '^\{|^L=' "$O/$name.log" | cut -c1-300
}
step tests 400 python -u -m pytest tests/test_gpu_bcopy.py tests/test_gpu_recv.py -x -q --timeout 200 --timeout-method thread
for r in 1 2; do
  for v in head nont prod; do
    if [ $v = prod ]; then L=lampi_amd/liblampi_csum.so; else L=ab/$v.so; fi
    for m in crc sum; do
      LAMPI_CSUM_LIB=$L step bcopy_${m}_${v}_$r 200 python bench.py --bcopy --mode $m --steps 10 --no-cpu-baseline
    done
    LAMPI_CSUM_LIB=$L step slots_${v}_$r 200 python tools/microbench/msg_bcopy_slots.py
  done
done
echo "=== done $(date +%T)"
