set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_d.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests_d.log; exit 1; }
tail -3 gpurun_out/tests_d.log
grep -E "native|leak" gpurun_out/tests_d.log
timeout -k 10 120 tests/native/host_leak 1000 && timeout -k 10 120 python bench.py --latency > gpurun_out/latency.log 2>&1 && tail -1 gpurun_out/latency.log
