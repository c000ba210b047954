set -o pipefail
A="--desc --mode sum --no-cpu-baseline --steps 10 --warmup 30"
tools/ab/env_ab.sh LAMPI_SUM_RO_WGS 1 "$A --frags 256 --frag-bytes 16777216" 32768 65536
tools/ab/env_ab.sh LAMPI_SUM_RO_WGS 1 "$A --frags 1024 --frag-bytes 1048576" 32768 65536
tools/ab/env_ab.sh LAMPI_SUM_RO_WGS 1 "$A --frags 2048 --frag-bytes 4194304" 32768 65536
M="--mode sum --no-cpu-baseline --steps 10 --warmup 30"
tools/ab/env_ab.sh LAMPI_SUM_MSG_WG 1 "$M --frags 256 --frag-bytes 16777216" 0 1
tools/ab/env_ab.sh LAMPI_SUM_MSG_WG 1 "$M --frags 1024 --frag-bytes 1048576" 0 1
tools/ab/env_ab.sh LAMPI_SUM_MSG_WG 1 "$M --frags 2048 --frag-bytes 4194304" 0 1
tools/ab/env_ab.sh LAMPI_SUM_MSG_WG 1 "$M --frags 1024 --frag-bytes 4194304" 0 1
tools/ab/env_ab.sh LAMPI_SUM_MSG_WG 1 "$M --frags 16384 --frag-bytes 262144" 0 1
