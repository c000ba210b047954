#!/usr/bin/env bash
# Round 3: piece-stream per-lane Horner carry.  Parity (descriptor / message / config C tests), then
# same-box interleaved A/B of config C, 4 KiB descriptors and the large-descriptor scan against ab/old.so.
# Usage: tools/gpu_r03_stream_ab.sh [ROUNDS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${1:-2}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_native.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/stream_parity.log 2>&1 || { tail -30 gpurun_out/stream_parity.log; exit 1; }
tail -2 gpurun_out/stream_parity.log
for r in $(seq 1 "$R"); do
  for v in old new; do
    if [ $v = new ]; then L=lampi_amd/liblampi_csum.so; else L=ab/$v.so; fi
    echo "== round $r $v"
    LAMPI_CSUM_LIB=$L timeout -k 10 300 python bench.py --config C --steps 20 --no-cpu-baseline 2>&1 | grep '^{' | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('configC', d['roofline']['frac'], 'parity', d['parity']['ok'])" || exit 1
    LAMPI_CSUM_LIB=$L timeout -k 10 300 python bench.py --desc --steps 20 --no-cpu-baseline 2>&1 | grep '^{' | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('desc4k', d['roofline']['frac'], 'parity', d['parity']['ok'])" || exit 1
  done
done
for v in old new; do
  if [ $v = new ]; then L=lampi_amd/liblampi_csum.so; else L=ab/$v.so; fi
  echo "== bigdesc $v"
  LAMPI_CSUM_LIB=$L timeout -k 10 300 python tools/microbench/bigdesc_scan.py crc 2>&1 | grep -v amdgpu.ids | grep count || exit 1
done
