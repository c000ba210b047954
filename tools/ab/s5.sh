set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s5
for m in crc sum; do
  timeout -k 10 120 python bench.py --recv --mode $m --frags 16384 --frag-bytes 65456 --steps 20 --warmup 60 > gpurun_out/s5/recv_$m.json 2>/dev/null || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s5/prof_$m -o run -- python3 bench.py --recv --mode $m --frags 16384 --frag-bytes 65456 --steps 20 --warmup 60 > gpurun_out/s5/prof_$m.log 2>&1 || exit 1
done
echo done
