set -o pipefail
for fb in "543392 1976" "1048576 1024" "4194304 256" "16777216 64" "524288 2048"; do set -- $fb
  tools/ab/env_ab.sh LAMPI_SUM_RO_WAVES 1 "--desc --mode sum --no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2" 0 1 | sed "s/^/desc$2 /"
  tools/ab/env_ab.sh LAMPI_SUM_RO_WAVES 1 "--mode sum --no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2" 0 1 | sed "s/^/msg$2 /"
done
