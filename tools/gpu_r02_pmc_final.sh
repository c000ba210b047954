#!/usr/bin/env bash
# Round-2 closing PMC passes (one counter group per run, no trace domains): FETCH_SIZE and
# WRITE_SIZE of the fused-copy and receive benches, for profiles/traffic.json (tools/pmc_traffic.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmcf
mkdir -p $O
pass() {  # name counter bench-args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/$name -o run -- python3 bench.py "$@" --steps 3 --warmup 1 \
    > $O/$name.log 2>&1 || { echo "!!! $name"; tail $O/$name.log; exit 1; }
  echo "ok $name"
}
pass bc_fetch FETCH_SIZE --bcopy
pass bc_write WRITE_SIZE --bcopy
pass rv_fetch FETCH_SIZE --recv
pass rv_write WRITE_SIZE --recv
echo PMC_DONE
