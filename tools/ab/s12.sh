set -o pipefail
R="--mode sum --no-cpu-baseline --steps 20 --warmup 60"
tools/ab/env_ab.sh LAMPI_SUM_GRP_WAVES 2 "--recv $R --frags 16384 --frag-bytes 65456" 0 1 | sed "s/^/recvGM /"
tools/ab/env_ab.sh LAMPI_SUM_GRP_WAVES 1 "--recv $R --frags 262144 --frag-bytes 16384" 0 1 | sed "s/^/recv16k /"
tools/ab/env_ab.sh LAMPI_SUM_GRP_WAVES 1 "--desc $R --frags 65536 --frag-bytes 65456" 0 1 | sed "s/^/descGM /"
tools/ab/env_ab.sh LAMPI_SUM_GRP_WAVES 1 "--bcopy $R --frags 131072 --frag-bytes 32768" 0 1 | sed "s/^/bcopy32k /"
