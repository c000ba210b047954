set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "multirow or short_lived or short_last" > gpurun_out/s7_pytest.log 2>&1 || { tail -30 gpurun_out/s7_pytest.log; exit 1; }
tail -3 gpurun_out/s7_pytest.log
