#!/usr/bin/env bash
# Round 6: config B's rows loaded coalesced (1 KiB per load instruction) with the non-temporal bit (1) or without (2),
# turned into lane-contiguous pieces through a 2 KiB LDS buffer per wave, against the product (0) -- A/B build,
# LAMPI_REG_XPOSE, interleaved; bench.py checks config B's digest.  Plain reads: coalesced + nt 86.9% in 128-thread
# workgroups against ~82% without (tools/microbench/launch_size.hip).
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
for r in 1 2 3; do
  for x in 0 1 2; do
    line "r$r B 16G xpose=$x" LAMPI_REG_XPOSE=$x python bench.py --no-cpu-baseline --steps 20
  done
  for x in 0 1; do
    line "r$r B 1G xpose=$x" LAMPI_REG_XPOSE=$x python bench.py --frags 262144 --no-cpu-baseline --steps 20
  done
done
