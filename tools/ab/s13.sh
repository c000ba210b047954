set -o pipefail
R="--recv --no-cpu-baseline --steps 20 --warmup 60"
tools/ab/env_ab.sh LAMPI_PAIR_WAVES 2 "$R --frags 262144 --frag-bytes 1976" 4 8 16 | sed "s/^/IBcrc /"
tools/ab/env_ab.sh LAMPI_LIGHT_WAVES 2 "$R --frags 16384 --frag-bytes 65456" 4 8 | sed "s/^/GMcrc /"
tools/ab/env_ab.sh LAMPI_PAIR_WAVES 1 "$R --mode sum --frags 262144 --frag-bytes 1976" 8 | sed "s/^/IBsum /"
