# Round-5 final survey: read-only CRC / SUM, messages and descriptors, across fragment sizes (4-8 GiB each
# except the small-count rows), one line per (mode, entry point, shape): roofline fraction and parity.
set -o pipefail
one() { out=$(timeout -k 10 120 python bench.py $1 2>/dev/null) || { echo "FAIL $1"; return 0; }
  python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-80s %.4f %s' % (sys.argv[2], d['roofline']['frac'], (d.get('parity') or {}).get('ok')))" "$out" "$1"; }
for mode in crc sum; do
for fb in "1048576 1024" "543392 1976" "4194304 4096" "524288 8192" "262144 16384" "131072 32768" "65536 65456" "16384 262144" "4096 1048576" "1024 4194304" "256 16777216" "200 1048576" "16 16777216"; do
  set -- $fb
  one "--desc --mode $mode --no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2"
  one "--mode $mode --no-cpu-baseline --steps 10 --warmup 30 --frags $1 --frag-bytes $2"
done; done
