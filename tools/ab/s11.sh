set -o pipefail
A="--desc --no-cpu-baseline --steps 10 --warmup 30"
for fb in "524288 8192" "262144 16384" "149796 28672" "131072 32768" "65536 65536"; do
  set -- $fb
  tools/ab/env_ab.sh LAMPI_CRC_DESC_REGULAR 2 "$A --frags $1 --frag-bytes $2" 1 16 | sed "s/^/$2x$1 /"
done
