#!/usr/bin/env bash
# Round 6: packed-row messages (64 B .. 2 KiB fragments on config B's kernel) -- parity, then bench lines
# with the packed launch and without it (LAMPI_PACKED=0 / LAMPI_PACKED_SUM=0, the round-5 schedules).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"  # the A/B build: knobs read from the environment
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread \
  -k "packed_row or config_a_shape or uniform_batches or config_b_full" > gpurun_out/r6_packed_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6_packed_tests.log; [ $rc -eq 0 ] || exit $rc
line() {  # label env... -- bench args
  local tag=$1; shift
  local out
  out=$(timeout -k 10 120 env "$@" 2>/dev/null | tail -1) || { echo "FAIL $tag"; exit 1; }
  echo "$out" >> gpurun_out/r6_packed.jsonl
  python - "$tag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:40s} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
}
for r in 1 2; do
  for spec in "16777216 64 2" "4194304 256 2" "2097152 512 2" "1048576 1024 1" "524288 2048 2"; do
    set -- $spec
    for m in crc sum; do
      line "r$r $2B $m packed" LAMPI_PACKED=1 python bench.py --frags $1 --frag-bytes $2 --seed $3 --mode $m --no-cpu-baseline
      line "r$r $2B $m old" LAMPI_PACKED=0 LAMPI_PACKED_SUM=0 python bench.py --frags $1 --frag-bytes $2 --seed $3 --mode $m --no-cpu-baseline
    done
  done
done
line "configB crc" LAMPI_PACKED=1 python bench.py --no-cpu-baseline
