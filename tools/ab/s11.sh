set -o pipefail
A="--desc --no-cpu-baseline --steps 20 --warmup 30"
tools/ab/env_ab.sh LAMPI_DESC_FPW 2 "$A" - 8 16 24 32 | sed "s/^/4k /"
tools/ab/env_ab.sh LAMPI_DESC_FPW 1 "$A --frags 262144 --frag-bytes 16384" - 6 12 24 | sed "s/^/16k /"
