#!/usr/bin/env bash
# Round 6: SUM messages of 64 B .. 1 KiB fragments on short-lived 128-thread workgroups, one per 4 KiB of the message
# (sum_row4k_kernel, A/B build, LAMPI_SUM_ROW4K=1) against the packed rows (=0) -- the GPU tests that cover these
# messages first with the switch on, then interleaved bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so" LAMPI_SUM_ROW4K=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -m gpu -v --timeout 120 \
  --timeout-method thread -k "packed_row_messages or config_a_shape or small_fragment or uniform" > gpurun_out/r6_row4k_tests.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/r6_row4k_tests.log; grep -E "FAILED|ERROR" gpurun_out/r6_row4k_tests.log | head; tail -2 gpurun_out/r6_row4k_tests.log; [ $rc -eq 0 ] || exit $rc
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"
line() {
  local tag=$1; shift
  local out
  out=$(timeout -k 10 200 env "$@" 2>/dev/null | tail -1) || { echo "FAIL $tag"; exit 1; }
  python - "$tag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:30s} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
}
S="--mode sum --no-cpu-baseline --steps 20"
for r in 1 2; do
  for spec in "1048576 1024 1" "16777216 64 2" "4194304 256 2" "2097152 512 2" "16777216 1024 2"; do
    set -- $spec
    line "r$r SUM $2B x$1 row4k" LAMPI_SUM_ROW4K=1 python bench.py $S --frags $1 --frag-bytes $2 --seed $3
    line "r$r SUM $2B x$1 packed" LAMPI_SUM_ROW4K=0 python bench.py $S --frags $1 --frag-bytes $2 --seed $3
  done
done
