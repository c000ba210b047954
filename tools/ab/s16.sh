set -o pipefail
R="--mode sum --no-cpu-baseline --steps 20 --warmup 60"
tools/ab/env_ab.sh LAMPI_SUM_GRP_PER_WG 2 "--recv $R --frags 16384 --frag-bytes 65456" 1 2 4 | sed "s/^/recvGM /"
tools/ab/env_ab.sh LAMPI_SUM_GRP_PER_WG 1 "--recv $R --frags 262144 --frag-bytes 16384" 1 2 | sed "s/^/recv16k /"
tools/ab/env_ab.sh LAMPI_SUM_GRP_PER_WG 1 "--desc $R --frags 65536 --frag-bytes 65456" 1 2 | sed "s/^/descGM /"
tools/ab/env_ab.sh LAMPI_SUM_GRP_PER_WG 1 "--bcopy $R --frags 131072 --frag-bytes 32768" 1 2 | sed "s/^/bcopy32k /"
