set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_bcopy.py tests/test_gpu_recv.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/s8_pytest.log 2>&1 || { tail -30 gpurun_out/s8_pytest.log; exit 1; }
tail -3 gpurun_out/s8_pytest.log
