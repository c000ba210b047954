set -o pipefail
for v in 0 4096; do
  LAMPI_SMALL_BATCH=$v timeout -k 10 300 python bench.py --latency 2>/dev/null | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read())
for r in d['results']:
    if 'fragments' in r: print('SMALL_BATCH=$v', r['fragments'], r['stream_us_per_call'], r['sync_round_trip_us'], r['graph_us_per_call'])
"
done
