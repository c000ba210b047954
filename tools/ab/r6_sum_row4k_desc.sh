#!/usr/bin/env bash
# Round 6: SUM descriptor batches of equal 64 B .. 1 KiB fragments (learned contiguous run) on sum_row4k_desc_kernel
# (LAMPI_SUM_ROW4K_DESC=1, A/B build) against the packed rows (=0) -- the descriptor-shape tests with the switch on
# first, then interleaved bench.py --desc --mode sum lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"
LAMPI_SUM_ROW4K_DESC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py -m gpu -v \
  --timeout 120 --timeout-method thread -k "contiguous_descriptors or config_a_shape or descriptor or learned" \
  > gpurun_out/r6_row4k_desc_tests.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/r6_row4k_desc_tests.log; grep -E "FAILED|ERROR" gpurun_out/r6_row4k_desc_tests.log | head; tail -2 gpurun_out/r6_row4k_desc_tests.log; [ $rc -eq 0 ] || exit $rc
line() {
  local tag=$1; shift
  local out
  out=$(timeout -k 10 200 env "$@" 2>/dev/null | tail -1) || { echo "FAIL $tag"; exit 1; }
  python - "$tag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:34s} frac {r.get('frac')} meta {r.get('incl_metadata', {}).get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
}
S="--desc --mode sum --no-cpu-baseline --steps 20 --warmup 30"
for r in 1 2; do
  for spec in "1048576 1024 1" "16777216 64 2" "4194304 256 2"; do
    set -- $spec
    line "r$r SUMd $2B x$1 row4k" LAMPI_SUM_ROW4K_DESC=1 python bench.py $S --frags $1 --frag-bytes $2 --seed $3
    line "r$r SUMd $2B x$1 packed" LAMPI_SUM_ROW4K_DESC=0 python bench.py $S --frags $1 --frag-bytes $2 --seed $3
  done
done
