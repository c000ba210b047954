#!/usr/bin/env bash
# Round 6: CRC fused copies of messages of 64 B .. 1 KiB fragments in two passes (the copy on sum_row4k_copy_kernel, then
# the read-only CRC of the source in packed rows; LAMPI_CRC_COPY_2PASS=1, A/B build) against the one-pass table-light
# copy (=0) -- the message-copy and send tests with it on first, then interleaved bench.py --bcopy lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"
LAMPI_CRC_COPY_2PASS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_bcopy.py tests/test_gpu_send.py -m gpu -v \
  --timeout 120 --timeout-method thread > gpurun_out/r6_2pass_tests.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/r6_2pass_tests.log; grep -E "FAILED|ERROR" gpurun_out/r6_2pass_tests.log | head; tail -2 gpurun_out/r6_2pass_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for spec in "1048576 1024" "16777216 64" "4194304 256"; do
    set -- $spec
    for v in 1 0; do
      out=$(timeout -k 10 200 env LAMPI_CRC_COPY_2PASS=$v python bench.py --bcopy --steps 10 --frags $1 --frag-bytes $2 2>/dev/null | tail -1) || { echo FAIL; exit 1; }
      python - "r$r CRCcp $2B x$1 2pass=$v" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:34s} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
    done
  done
done
