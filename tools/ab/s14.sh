set -o pipefail
export TMPDIR=/tmp
LAMPI_CRC_PARTITION=12 tools/ab/env_ab.sh LAMPI_CRC_PARTITION_FORK 2 "--config C --no-cpu-baseline --steps 20" 0 1
mkdir -p gpurun_out/s14
LAMPI_CRC_PARTITION=12 LAMPI_CRC_PARTITION_FORK=1 timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s14/fork -o run -- python3 bench.py --config C --no-cpu-baseline --steps 20 > gpurun_out/s14/fork.log 2>&1
