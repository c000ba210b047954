set -o pipefail
tools/ab/env_ab.sh LAMPI_SUM_MSG_MAX 2 "--mode sum --no-cpu-baseline --steps 20 --frags 1048576 --frag-bytes 16384" 4096 16384
tools/ab/env_ab.sh LAMPI_SUM_MSG_MAX 2 "--mode sum --no-cpu-baseline --steps 5 --config D --shard 0" 4096 16384
