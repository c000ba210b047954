#!/usr/bin/env bash
# Round 6: SUM fused copies of descriptor batches of equal 64 B .. 1 KiB fragments on sum_row4k_copy_desc_kernel
# (LAMPI_SUM_ROW4K_COPY_DESC=1, A/B build) against the current schedules (=0) -- the copy-descriptor tests with it on
# first, then bench.py --bcopy --mode sum (its descriptor_batch lines), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"
LAMPI_SUM_ROW4K_COPY_DESC=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_bcopy.py tests/test_gpu_send.py \
  -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r6_row4k_cd_tests.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/r6_row4k_cd_tests.log; grep -E "FAILED|ERROR" gpurun_out/r6_row4k_cd_tests.log | head; tail -2 gpurun_out/r6_row4k_cd_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for spec in "1048576 1024" "16777216 64" "4194304 256"; do
    set -- $spec
    for v in 1 0; do
      out=$(timeout -k 10 200 env LAMPI_SUM_ROW4K_COPY_DESC=$v python bench.py --bcopy --mode sum --steps 10 --frags $1 --frag-bytes $2 2>/dev/null | tail -1) || { echo FAIL; exit 1; }
      python - "r$r SUMcd $2B x$1 row4k=$v" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2])
print(f"{sys.argv[1]:34s} descriptor_batch frac {d['descriptor_batch'].get('frac')} dst8 {d['descriptor_batch_dst8'].get('frac')} src8 {d['descriptor_batch_src8'].get('frac')} dst1 {d['descriptor_batch_dst1'].get('frac')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
    done
  done
done
