#!/usr/bin/env bash
# Round 6: the fixed cost of a launch -- config B's kernel (4 KiB) and the packed rows (1 KiB, 64 B) at 1, 4 and 16 GiB
# per launch (bench.py, product library), to separate the small-launch cost from the packed rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
line() {
  local tag=$1; shift
  local out
  out=$(timeout -k 10 180 "$@" 2>/dev/null | tail -1) || { echo "FAIL $tag"; exit 1; }
  python - "$tag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:28s} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
}
for r in 1 2; do
  for gib in 1 4 16; do
    line "r$r 4KiB ${gib}GiB" python bench.py --frags $((262144 * gib)) --frag-bytes 4096 --no-cpu-baseline --steps 10
    line "r$r 1KiB ${gib}GiB" python bench.py --frags $((1048576 * gib)) --frag-bytes 1024 --seed 1 --no-cpu-baseline --steps 10
    line "r$r 64B ${gib}GiB" python bench.py --frags $((16777216 * gib)) --frag-bytes 64 --no-cpu-baseline --steps 10
  done
done
