#!/usr/bin/env bash
# Round 6: config B with four lookup chains per wave (crc_regular_kernel<4>: 32 KiB in flight per wave instead of 16;
# the occupancy stays two workgroups per CU, set by the LDS) against the product's two -- A/B build, LAMPI_REG_CHAINS,
# interleaved; bench.py checks config B's digest.
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
  line "r$r B 16G chains=2" LAMPI_REG_CHAINS=2 python bench.py --no-cpu-baseline --steps 20
  line "r$r B 16G chains=4" LAMPI_REG_CHAINS=4 python bench.py --no-cpu-baseline --steps 20
  line "r$r B 1G chains=2" LAMPI_REG_CHAINS=2 python bench.py --frags 262144 --no-cpu-baseline --steps 20
  line "r$r B 1G chains=4" LAMPI_REG_CHAINS=4 python bench.py --frags 262144 --no-cpu-baseline --steps 20
done
