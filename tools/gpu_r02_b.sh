set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/tests_b.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests_b.log; exit 1; }
tail -3 gpurun_out/tests_b.log
timeout -k 10 300 python bench.py --recv --steps 10 --warmup 3 > gpurun_out/recv_crc.log 2>&1 || { echo RECV_FAIL; tail -20 gpurun_out/recv_crc.log; exit 1; }
tail -1 gpurun_out/recv_crc.log
timeout -k 10 300 python bench.py --recv --mode sum --steps 10 --warmup 3 > gpurun_out/recv_sum.log 2>&1 || { echo RECV_FAIL; tail -20 gpurun_out/recv_sum.log; exit 1; }
tail -1 gpurun_out/recv_sum.log
