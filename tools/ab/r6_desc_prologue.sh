#!/usr/bin/env bash
# Round 6: descriptor whole-row batches (crc_regular_kernel<kDesc>) with the descriptor check moved after the
# slicing-table build (desc_check inside stage_tables<kLatePre>) against the previous library (ab_libs/, built from
# the commit before) -- parity first, then interleaved bench.py --desc lines of config B and 8 / 16 KiB fragments.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py -m gpu -v --timeout 120 \
  --timeout-method thread -k "desc or learned" > gpurun_out/r6_dprol_tests.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/r6_dprol_tests.log; grep -E "FAIL|ERROR" gpurun_out/r6_dprol_tests.log | head; tail -2 gpurun_out/r6_dprol_tests.log; [ $rc -eq 0 ] || exit $rc
line() {
  local tag=$1; shift
  local out
  out=$(timeout -k 10 150 env "$@" 2>/dev/null | tail -1) || { echo "FAIL $tag"; exit 1; }
  python - "$tag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:32s} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
}
OLD="LAMPI_CSUM_LIB=$PWD/ab_libs/liblampi_csum_before.so"
NEW="LAMPI_CSUM_LIB=$PWD/lampi_amd/liblampi_csum.so"
A="--desc --no-cpu-baseline --steps 10 --warmup 30"
for r in 1 2 3; do
  for spec in "4194304 4096" "2097152 8192" "1048576 16384" "262144 4096"; do
    set -- $spec
    line "r$r desc $2B x$1 new" $NEW python bench.py $A --frags $1 --frag-bytes $2
    line "r$r desc $2B x$1 old" $OLD python bench.py $A --frags $1 --frag-bytes $2
  done
done
