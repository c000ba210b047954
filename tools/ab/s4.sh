set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 600 python -u -m pytest tests/test_gpu_recv.py tests/test_gpu_shapes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s4/pytest.log 2>&1 || { tail -30 gpurun_out/s4/pytest.log; exit 1; }
tail -2 gpurun_out/s4/pytest.log
for m in crc sum; do
  for v in 0 1; do
    echo "== mode $m LAMPI_SHAPES_UNKEYED=$v"
    LAMPI_SHAPES_UNKEYED=$v timeout -k 10 300 python bench.py --recv --alternate --mode $m --steps 10 --warmup 40 2>/dev/null | tee -a gpurun_out/s4/alt.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('gm', d['gm'], 'ib', d['ib'], 'ok', d['parity']['ok'])"
  done
done
