#!/usr/bin/env bash
# tools/ab/env_ab.sh VAR ROUNDS "BENCH ARGS" VALUE...   -- same-box A/B of an env knob, interleaved rounds.
# Each run: bench.py with VAR=VALUE ("-" = unset); prints value, roofline frac, kernel ms and parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"  # the A/B build: knobs read from the environment
mkdir -p gpurun_out
var=$1; rounds=$2; args=$3; shift 3
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    if [ "$v" = "-" ]; then
      out=$(timeout -k 10 120 env -u "$var" python bench.py $args 2>/dev/null) || { echo "FAIL $var=$v rc=$?"; exit 1; }
    else
      out=$(timeout -k 10 120 env "$var=$v" python bench.py $args 2>/dev/null) || { echo "FAIL $var=$v rc=$?"; exit 1; }
    fi
    echo "$out" >> gpurun_out/env_ab.jsonl
    python - "$r" "$var=$v" "$out" <<'PY'
import json, sys
r, tag, line = sys.argv[1], sys.argv[2], sys.argv[3].strip().splitlines()[-1]
d = json.loads(line)
rf = d.get("roofline", {})
print(f"round {r} {tag:32s} frac {rf.get('frac')} kernel_ms {rf.get('kernel_avg_ms')} ms_per_step {d.get('ms_per_step')} parity {d.get('parity', {}).get('ok')}", flush=True)
PY
  done
done
