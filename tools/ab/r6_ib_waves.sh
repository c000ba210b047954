#!/usr/bin/env bash
# Round 6: IB's receive step and fused copies (262,144 x 1,976 B) on crc_light_pair_copy_kernel with 4 / 8 / 16 waves per
# workgroup (A/B build, LAMPI_PAIR_WAVES), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"
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
for r in 1 2; do
  for w in 4 8 16; do
    line "r$r IB recv waves=$w" LAMPI_PAIR_WAVES=$w python bench.py --recv --frags 262144 --frag-bytes 1976 --warmup 30 --steps 20
  done
done
