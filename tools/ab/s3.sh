set -o pipefail
tools/ab/env_ab.sh LAMPI_SUM_MSG_MAX 2 "--mode sum --no-cpu-baseline --steps 10 --frags 65536 --frag-bytes 65456" 16384 1073741824
tools/ab/env_ab.sh LAMPI_SUM_MSG_MAX 2 "--mode sum --no-cpu-baseline --steps 10 --frags 4096 --frag-bytes 1048576" 16384 1073741824
tools/ab/env_ab.sh LAMPI_SUM_MSG_MAX 2 "--mode sum --no-cpu-baseline --steps 10 --frags 524288 --frag-bytes 32768" 16384 1073741824
