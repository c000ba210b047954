set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "full_shard" -x -v --timeout 240 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 || { echo SHARD_FAIL; tail -30 gpurun_out/shard_tests.log; exit 1; }
tail -6 gpurun_out/shard_tests.log
timeout -k 10 120 python bench.py --gpus 2 --steps 3 > gpurun_out/gpus2.log 2>&1; echo "gpus2 rc=$?"; tail -3 gpurun_out/gpus2.log
timeout -k 10 300 python bench.py --config D --shard 0 --steps 10 > gpurun_out/shard0.log 2>&1 || { echo D_FAIL; tail -20 gpurun_out/shard0.log; exit 1; }
tail -1 gpurun_out/shard0.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
