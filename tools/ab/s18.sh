set -o pipefail
tools/ab/env_ab.sh LAMPI_LEFTOVER_WGS 2 "--recv --no-cpu-baseline --steps 20 --warmup 60 --frags 262144 --frag-bytes 1976" 256 32 | sed "s/^/IBrecv /"
tools/ab/env_ab.sh LAMPI_LEFTOVER_WGS 2 "--desc --no-cpu-baseline --steps 20 --warmup 30" 256 32 | sed "s/^/desc4k /"
