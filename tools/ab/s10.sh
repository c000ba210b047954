set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/s10_pytest.log 2>&1 || { tail -30 gpurun_out/s10_pytest.log; exit 1; }
tail -2 gpurun_out/s10_pytest.log
A="--desc --no-cpu-baseline --steps 20 --warmup 30"
tools/ab/env_ab.sh LAMPI_CRC_DESC_REGULAR 3 "$A" 0 1
tools/ab/env_ab.sh LAMPI_CRC_DESC_REGULAR 1 "$A --frags 262144" 0 1
