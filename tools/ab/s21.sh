set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/s21_pytest.log 2>&1 || { tail -30 gpurun_out/s21_pytest.log; exit 1; }
tail -2 gpurun_out/s21_pytest.log
one() { out=$(timeout -k 10 120 python bench.py $1 2>/dev/null) || { echo "FAIL $1"; return 0; }
  python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-75s %.4f %s' % (sys.argv[2], d['roofline']['frac'], (d.get('parity') or {}).get('ok')))" "$out" "$1"; }
for fb in "16777216 64" "4194304 256" "1048576 1024" "699050 1536" "524288 2048" "543392 1976" "4194304 4096"; do set -- $fb
  one "--desc --no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2"
  one "--no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2"
done
one "--config C --no-cpu-baseline --steps 20"
