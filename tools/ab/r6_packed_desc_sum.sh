#!/usr/bin/env bash
# Round 6: SUM packed rows for contiguous descriptor batches (LAMPI_PACKED_DESC=0: the round-5 schedules).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"  # the A/B build: knobs read from the environment
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py -m gpu -q --timeout 120 \
  --timeout-method thread -k "contiguous_descriptors or config_a_shape or descriptor_batch or learned" > gpurun_out/r6_pdesc_sum_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6_pdesc_sum_tests.log; [ $rc -eq 0 ] || exit $rc
line() {
  local tag=$1; shift
  local out
  out=$(timeout -k 10 120 env "$@" 2>/dev/null | tail -1) || { echo "FAIL $tag"; exit 1; }
  echo "$out" >> gpurun_out/r6_packed_desc_sum.jsonl
  python - "$tag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:40s} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
}
A="--desc --mode sum --no-cpu-baseline --steps 10 --warmup 30"
for r in 1 2; do
  for spec in "1048576 1024 1" "16777216 64 2" "4194304 256 2" "2097152 512 2"; do
    set -- $spec
    line "r$r desc sum $2B packed" LAMPI_PACKED_DESC=1 python bench.py $A --frags $1 --frag-bytes $2 --seed $3
    line "r$r desc sum $2B old" LAMPI_PACKED_DESC=0 python bench.py $A --frags $1 --frag-bytes $2 --seed $3
  done
done
