#!/usr/bin/env bash
# Round 6: packed-row messages, items per wave (LAMPI_PACKED_FPW) at 1 GiB and 16 GiB of 1 KiB / 64 B fragments.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"  # the A/B build: knobs read from the environment
mkdir -p gpurun_out
line() {
  local tag=$1; shift
  local out
  out=$(timeout -k 10 120 env "$@" 2>/dev/null | tail -1) || { echo "FAIL $tag"; exit 1; }
  echo "$out" >> gpurun_out/r6_packed_fpw.jsonl
  python - "$tag" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2]); r = d.get("roofline", {})
print(f"{sys.argv[1]:40s} frac {r.get('frac')} kernel_ms {r.get('kernel_avg_ms')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
}
for r in 1 2; do
  for f in 12 8 6 4 16; do
    line "r$r 1KiB x1M fpw$f crc" LAMPI_PACKED_FPW=$f python bench.py --frags 1048576 --frag-bytes 1024 --seed 1 --no-cpu-baseline
  done
  for f in 12 6; do
    line "r$r 1KiB x16M fpw$f crc" LAMPI_PACKED_FPW=$f python bench.py --frags 16777216 --frag-bytes 1024 --seed 1 --no-cpu-baseline --steps 10
    line "r$r 64B x16M fpw$f crc" LAMPI_PACKED_FPW=$f python bench.py --frags 16777216 --frag-bytes 64 --no-cpu-baseline
  done
done
