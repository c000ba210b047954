#!/usr/bin/env bash
# Round 6: crc_regular_kernel's first generation of workgroups staggered (fpw -3a / -a / +a / +3a items per wave by
# groups of eight) -- "new" (product library) against the library before (ab_libs/), interleaved: the GPU parity, shape
# and send suites first, then 1 GiB and 16 GiB launches of config B and of config A's packed rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_gpu_send.py -m gpu -q \
  --timeout 120 --timeout-method thread -x > gpurun_out/r6_stagger_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6_stagger_tests.log; [ $rc -eq 0 ] || exit $rc
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
OLD="LAMPI_CSUM_LIB=$PWD/ab_libs/liblampi_csum_before.so"
NEW="LAMPI_CSUM_LIB=$PWD/lampi_amd/liblampi_csum.so"
for r in 1 2 3; do
  for v in new old; do
    if [ $v = new ]; then L=$NEW; else L=$OLD; fi
    line "r$r B 16G $v" $L python bench.py --no-cpu-baseline --steps 20
    line "r$r B 1G $v" $L python bench.py --frags 262144 --no-cpu-baseline --steps 20
    line "r$r A 1G msg $v" $L python bench.py --frags 1048576 --frag-bytes 1024 --seed 1 --no-cpu-baseline --steps 20
    line "r$r A 1G desc $v" $L python bench.py --desc --frags 1048576 --frag-bytes 1024 --seed 1 --no-cpu-baseline --steps 20 --warmup 30
    line "r$r B desc 16G $v" $L python bench.py --desc --no-cpu-baseline --steps 10 --warmup 30
  done
done
