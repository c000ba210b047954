set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s14
LAMPI_CRC_PARTITION=12 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s14/prof -o run -- python3 bench.py --config C --no-cpu-baseline --steps 20 > gpurun_out/s14/prof.log 2>&1
