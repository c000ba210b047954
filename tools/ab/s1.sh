set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 600 python -u -m pytest tests/test_gpu_native.py -m gpu -x -v --timeout 300 --timeout-method thread -k "receive_path or typemap" > gpurun_out/s1/pytest.log 2>&1 || { tail -30 gpurun_out/s1/pytest.log; exit 1; }
tail -3 gpurun_out/s1/pytest.log
tools/ab/env_ab.sh LAMPI_SUM_MSG_WG 3 "--mode sum --no-cpu-baseline --steps 20" 0 2 1 4
