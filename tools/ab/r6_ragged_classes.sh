#!/usr/bin/env bash
# Round 6: config C's size classes alone (tools/microbench/configc_classes.py, CRC and SUM) with the ragged rows
# (LAMPI_RAGGED=1, 16 / 64 fragments per wave) and without (the piece streams) -- VERDICT r5 item 1's "class B alone" test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export LAMPI_CSUM_LIB="$PWD/lampi_amd/liblampi_csum_ab.so"
for v in "LAMPI_RAGGED=0" "LAMPI_RAGGED=1" "LAMPI_RAGGED=1 LAMPI_RAGGED_FPW=64"; do
  echo "== $v"
  timeout -k 10 300 env $v python tools/microbench/configc_classes.py 2>&1 | grep "^crc" || exit 1
done
