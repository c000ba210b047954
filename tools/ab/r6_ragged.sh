#!/usr/bin/env bash
# Round 6: ragged whole-row descriptor batches (crc_ragged_kernel) -- the new parity tests and the
# shape/parity suites first, then config C with the ragged rows against the piece streams (A/B build, LAMPI_RAGGED=0)
# and fragments per wave, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shapes.py -m gpu -v --timeout 120 --timeout-method thread \
  -k "ragged" > gpurun_out/r6_ragged_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|assert" gpurun_out/r6_ragged_tests.log | head -20; tail -2 gpurun_out/r6_ragged_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py -m gpu -q --timeout 120 \
  --timeout-method thread -x > gpurun_out/r6_ragged_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r6_ragged_suite.log; [ $rc -eq 0 ] || exit $rc
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"
line() {
  local tag=$1; shift
  local out
  out=$(timeout -k 10 200 env "$@" 2>/dev/null | tail -1) || { echo "FAIL $tag"; exit 1; }
  python - "$tag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:28s} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')} {r.get('kernel', '')[:60]}", flush=True)
PY
}
for r in 1 2; do
  line "r$r C ragged fpw16" LAMPI_RAGGED=1 python bench.py --config C --no-cpu-baseline --steps 10 --warmup 20
  line "r$r C streams" LAMPI_RAGGED=0 python bench.py --config C --no-cpu-baseline --steps 10 --warmup 20
  line "r$r C ragged fpw8" LAMPI_RAGGED=1 LAMPI_RAGGED_FPW=8 python bench.py --config C --no-cpu-baseline --steps 10 --warmup 20
  line "r$r C ragged fpw32" LAMPI_RAGGED=1 LAMPI_RAGGED_FPW=32 python bench.py --config C --no-cpu-baseline --steps 10 --warmup 20
done
