set -o pipefail
for fb in "16777216 64" "4194304 256" "2097152 512" "1048576 1024"; do set -- $fb
  tools/ab/env_ab.sh LAMPI_SUM_TINY 1 "--mode sum --no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2" 0 4096 | sed "s/^/msg$2 /"
done
