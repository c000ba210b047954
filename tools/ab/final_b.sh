# Round-5 final (b): bench lines, the rocprof kernel trace of the default bench, PMC traffic passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
b() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { echo "FAIL bench $name"; tail -5 $O/bench_$name.err; exit 1; }; tail -1 $O/bench_$name.json | cut -c1-400; }
b B &&
b B_sum --mode sum &&
b C --config C &&
b C_sum --config C --mode sum &&
b D0 --config D --shard 0 &&
b recv_gm --recv --frags 16384 --frag-bytes 65456 &&
b recv_gm_sum --recv --mode sum --frags 16384 --frag-bytes 65456 &&
b bcopy --bcopy &&
b desc --desc &&
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_B -o run -- python3 bench.py --steps 20 > $O/prof_B.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_B_fetch -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/pmc_B_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_Bsum_fetch -o run -- python3 bench.py --mode sum --steps 5 --warmup 3 --no-cpu-baseline > $O/pmc_Bsum_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_desc_fetch -o run -- python3 bench.py --desc --steps 5 --warmup 40 --no-cpu-baseline > $O/pmc_desc_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_desc -o run -- python3 bench.py --desc --steps 20 --warmup 40 --no-cpu-baseline > $O/prof_desc.log 2>&1 &&
echo "final_b done"
