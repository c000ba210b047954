set -o pipefail
for fb in "543392 1976" "524288 2048" "699050 1536"; do set -- $fb
  tools/ab/env_ab.sh LAMPI_CRC_RO_PAIRS 2 "--desc --no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2" 0 1 | sed "s/^/desc$2 /"
done
tools/ab/env_ab.sh LAMPI_CRC_RO_PAIRS 2 "--no-cpu-baseline --steps 10 --warmup 30 --frags 543392 --frag-bytes 1976" 0 1 | sed "s/^/msg1976 /"
tools/ab/env_ab.sh LAMPI_CRC_RO_PAIRS 1 "--config C --no-cpu-baseline --steps 20" 0 1 | sed "s/^/configC /"
