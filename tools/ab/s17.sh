set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_gpu_native.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/s17_pytest.log 2>&1 || { tail -30 gpurun_out/s17_pytest.log; exit 1; }
tail -2 gpurun_out/s17_pytest.log
for v in 0 4096; do
LAMPI_SMALL_BATCH=$v timeout -k 10 300 python bench.py --latency 2>/dev/null | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read())
for r in d['results']:
    if 'fragments' in r: print('latency SMALL_BATCH=$v', r['fragments'], r['stream_us_per_call'], r['sync_round_trip_us'], r['graph_us_per_call'])
"
done
