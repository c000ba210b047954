#!/usr/bin/env bash
# Round 6: SUM fused copies of messages of 64 B .. 1 KiB fragments on sum_row4k_copy_kernel (LAMPI_SUM_ROW4K_COPY=1,
# A/B build) against one workgroup per fragment (=0) -- the message-copy tests with the switch on first, then
# interleaved bench.py --bcopy --mode sum lines (read + write bytes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"
LAMPI_SUM_ROW4K_COPY=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_bcopy.py tests/test_gpu_send.py -m gpu -v \
  --timeout 120 --timeout-method thread -k "msg_bcopy or send" > gpurun_out/r6_row4k_copy_tests.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/r6_row4k_copy_tests.log; grep -E "FAILED|ERROR" gpurun_out/r6_row4k_copy_tests.log | head; tail -2 gpurun_out/r6_row4k_copy_tests.log; [ $rc -eq 0 ] || exit $rc
line() {
  local tag=$1; shift
  local out
  out=$(timeout -k 10 200 env "$@" 2>/dev/null | tail -1) || { echo "FAIL $tag"; exit 1; }
  python - "$tag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:34s} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
}
S="--bcopy --mode sum --steps 10"
for r in 1 2; do
  for spec in "1048576 1024" "16777216 64" "4194304 256"; do
    set -- $spec
    line "r$r SUMcp $2B x$1 row4k" LAMPI_SUM_ROW4K_COPY=1 python bench.py $S --frags $1 --frag-bytes $2
    line "r$r SUMcp $2B x$1 wg" LAMPI_SUM_ROW4K_COPY=0 python bench.py $S --frags $1 --frag-bytes $2
  done
done
