#!/usr/bin/env bash
# Same-box A/B: tools/gpu_ab.sh OUT ROUNDS "lib1 lib2 ..." "bench args 1" "bench args 2" ...
# (lib "prod" = lampi_amd/liblampi_csum.so, anything else = ab/<name>.so); rounds interleave the libs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; R=$2; LIBS=$3; shift 3
mkdir -p $O
for r in $(seq 1 $R); do
  for v in $LIBS; do
    if [ $v = prod ]; then L=lampi_amd/liblampi_csum.so; else L=ab/$v.so; fi
    i=0
    for a in "$@"; do
      i=$((i+1))
      LAMPI_CSUM_LIB=$L timeout -k 10 200 python bench.py $a --no-cpu-baseline > $O/${v}_${i}_$r.log 2>&1 || { echo "!!! $v $a rc=$?"; tail -20 $O/${v}_${i}_$r.log; exit 1; }
      python - "$O/${v}_${i}_$r.log" "$v" "$a" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
fr = {k: round(v['frac'], 4) for k, v in d.items() if isinstance(v, dict) and 'frac' in v}
print(sys.argv[2], sys.argv[3], fr, 'parity', d.get('parity', {}).get('ok'), flush=True)
PY
    done
  done
done
