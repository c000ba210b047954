#!/usr/bin/env bash
# Round-3 same-box A/B of the CRC descriptor copies and the receive step: ab/NAME.so against the
# current library, interleaved.  Usage: tools/gpu_r03_desc_ab.sh ROUNDS [NAME ...] (default NAME: head)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-2}
shift
VARIANTS="${*:-head} new"
for r in $(seq 1 "$R"); do
  for v in $VARIANTS; do
    if [ $v = new ]; then L=lampi_amd/liblampi_csum.so; else L=ab/$v.so; fi
    echo "== round $r $v"
    LAMPI_CSUM_LIB=$L timeout -k 10 300 python bench.py --bcopy --steps 10 --no-cpu-baseline 2>&1 | grep '^{' | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bcopy crc msg', d['roofline']['frac'], 'desc', d['descriptor_batch']['frac'], 'src8', d['descriptor_batch_src8']['frac'], 'dst8', d['descriptor_batch_dst8']['frac'], 'dst1', d['descriptor_batch_dst1']['frac'], 'gm', d['gm_send_slots']['frac'], 'parity', d['parity']['ok_all'])" || exit 1
    LAMPI_CSUM_LIB=$L timeout -k 10 300 python bench.py --recv --steps 10 2>&1 | grep '^{' | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('recv crc', d['roofline']['frac'], 'parity', d['parity']['ok'])" || exit 1
  done
done
