#!/usr/bin/env bash
# Round 3: crc_list_kernel (descriptor batches on the regular kernel's shape) against the piece streams.
# Parity of the descriptor tests with the list kernel selected, then same-box interleaved A/B of
# config C, 4 KiB descriptors and the large-descriptor scan.  Usage: tools/gpu_r03_list.sh [ROUNDS] [VARIANTS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${1:-2}
VARIANTS=${2:-"stream list"}
LAMPI_DESC_KERNEL=list timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "descriptor or config_c or kat" > gpurun_out/list_parity.log 2>&1 || { tail -30 gpurun_out/list_parity.log; exit 1; }
tail -3 gpurun_out/list_parity.log
for r in $(seq 1 "$R"); do
  for v in $VARIANTS; do
    echo "== round $r $v"
    LAMPI_DESC_KERNEL=$v timeout -k 10 300 python bench.py --config C --steps 20 --no-cpu-baseline 2>&1 | grep '^{' | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('configC', d['roofline']['frac'], d['roofline'].get('kernel'), 'parity', d['parity'])" || exit 1
    LAMPI_DESC_KERNEL=$v timeout -k 10 300 python bench.py --desc --steps 20 --no-cpu-baseline 2>&1 | grep '^{' | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('desc4k', d['roofline']['frac'], 'parity', d['parity'])" || exit 1
  done
done
for v in $VARIANTS; do
  echo "== bigdesc $v"
  LAMPI_DESC_KERNEL=$v timeout -k 10 300 python tools/microbench/bigdesc_scan.py crc 2>&1 | grep -v amdgpu.ids || exit 1
done
