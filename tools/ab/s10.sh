set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/s10_pytest.log 2>&1 || { tail -30 gpurun_out/s10_pytest.log; exit 1; }
tail -2 gpurun_out/s10_pytest.log
for fb in "4194304 4096" "262144 16384"; do set -- $fb
  timeout -k 10 120 python bench.py --desc --no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['roofline']['frac'], d.get('parity',{}).get('ok'))"
done
