set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_i.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests_i.log; exit 1; }
tail -1 gpurun_out/tests_i.log
for m in crc sum; do
timeout -k 10 300 python bench.py --config C --mode $m --steps 50 > gpurun_out/benchC_$m.log 2>&1 && tail -1 gpurun_out/benchC_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C $m', d['roofline']['frac'], d['one_wavefront_per_fragment'], d['parity']['ok'])"
done
