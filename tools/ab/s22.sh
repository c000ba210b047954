set -o pipefail
for fb in "16777216 64" "4194304 256" "1048576 1024" "543392 1976"; do set -- $fb
  tools/ab/env_ab.sh LAMPI_SUM_TINY 1 "--desc --mode sum --no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2" 0 1024 | sed "s/^/desc$2 /"
done
