set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_h.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests_h.log; exit 1; }
tail -1 gpurun_out/tests_h.log
timeout -k 10 200 python bench.py --latency > gpurun_out/latency_h.log 2>&1 && tail -1 gpurun_out/latency_h.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['results'][-1])"
