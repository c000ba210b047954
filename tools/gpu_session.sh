#!/usr/bin/env bash
# tools/gpu_session.sh -- run GPU steps on the gpurun box with a time limit each.
# Usage: tools/gpu_session.sh STEP [STEP ...]   where STEP is one of:
#   smoke | tests | tests_native | tests_bcopy | bench | bench16k | benchsum | benchC | benchCsum | benchD | bcopy |
#   prof | profC | pmc | pmcC | pmcCsum | pmcDshard | pmcbcopy | pmcsq | pmcdesc | e2e | latency | copysizes | recv | gm | bigdesc
# Any failure (a test failure, fault, abort, segfault, timeout or kill) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp

run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then  # a failed test may have left a faulting kernel: stop
    echo "!!! $name ended with $rc: stopping the session"
    exit $rc
  fi
  return 0
}

for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    bench) run bench 600 python bench.py ;;
    bench16k) run bench16k 600 python bench.py --frags 1048576 --frag-bytes 16384 --no-cpu-baseline ;;
    benchsum) run benchsum 600 python bench.py --mode sum --no-cpu-baseline ;;
    benchC) run benchC 600 python bench.py --config C --steps 50 ;;
    benchCsum) run benchCsum 600 python bench.py --config C --mode sum --steps 50 ;;
    benchD) run benchD 600 python bench.py --desc --no-cpu-baseline ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
            -- python3 bench.py --steps 20 --no-cpu-baseline ;;
    pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run \
            -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline &&
         run pmc_ea 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv \
            -d gpurun_out/pmc_ea -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    profC) run profC 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profC -o run \
            -- python3 bench.py --config C --steps 20 ;;
    pmcC) run pmcC_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcC_fetch -o run \
            -- python3 bench.py --config C --steps 5 --warmup 1 ;;
    pmcCsum) run pmcCsum_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcCsum_fetch -o run \
            -- python3 bench.py --config C --mode sum --steps 5 --warmup 1 ;;
    pmcDshard) run pmcD0_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcD0_fetch -o run \
            -- python3 bench.py --config D --shard 0 --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmcbcopy) run pmcbcopy_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcbcopy_fetch \
            -o run -- python3 bench.py --bcopy --steps 5 --warmup 3 &&
         run pmcbcopy_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcbcopy_write \
            -o run -- python3 bench.py --bcopy --steps 5 --warmup 3 ;;
    pmclds) for cfg in B C R; do  # LDS array cycles and bank conflicts, stall split (R: GM receive, learned row groups)
             args="--no-cpu-baseline"; [ $cfg = C ] && args="--config C"
             [ $cfg = R ] && args="--recv --frags 16384 --frag-bytes 65456 --warmup 40"
             run pmc_lds$cfg 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY \
                 SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv \
                 -d gpurun_out/pmc_lds$cfg -o run -- python3 bench.py --steps 3 $args
           done ;;
    pmcsq) for cfg in B C D; do
             extra="--no-cpu-baseline"; [ $cfg = C ] && extra="--config C"; [ $cfg = D ] && extra="--desc --no-cpu-baseline"
             run pmc_sq$cfg 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
                 SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv \
                 -d gpurun_out/pmc_sq$cfg -o run -- python3 bench.py --steps 3 --warmup 1 $extra
           done ;;
    pmcdesc) for spec in crc:1024:1048576:256 crc:256:4194304:1024 sum:4194304:4096:0 sum:16404:65456:0; do  # FETCH_SIZE per line
               IFS=: read -r m nf fb h <<< "$spec"
               run pmcdesc_${m}_${fb}_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
                 -d gpurun_out/pmcdesc_${m}_${fb}_fetch -o run -- python3 bench.py --desc --mode $m --frags $nf \
                 --frag-bytes $fb --rows-hint $h --steps 5 --warmup 1 --no-cpu-baseline || exit 1
             done ;;
    e2e) run e2e 600 python bench.py --e2e ;;
    latency) run latency 300 python bench.py --latency ;;
    copysizes) run copysizes_crc 400 python tools/microbench/desc_copy_sizes.py crc &&
               run copysizes_sum 400 python tools/microbench/desc_copy_sizes.py sum ;;
    recv) run recv 600 python bench.py --recv --steps 10 &&
          run recvsum 600 python bench.py --recv --mode sum --steps 10 ;;
    bcopy) run bcopy 600 python bench.py --bcopy --steps 10 &&
           run bcopysum 600 python bench.py --bcopy --mode sum --steps 10 ;;
    gm) for m in crc sum; do  # GM's 65,456-byte payloads, with and without LAMPI_CSUM_ROWS_HINT(16)
          for h in 0 16; do
            run gm_recv_${m}_h$h 600 python bench.py --recv --mode $m --frags 16384 --frag-bytes 65456 --rows-hint $h --steps 20 --warmup 60 &&
            run gm_desc_${m}_h$h 600 python bench.py --desc --mode $m --frags 16404 --frag-bytes 65456 --rows-hint $h --steps 20 --warmup 60 --no-cpu-baseline
          done
        done ;;
    bigdesc) for spec in 16404:65456:16 1024:1048576:256 256:4194304:1024; do  # read-only, LAMPI_CSUM_ROWS_HINT
               IFS=: read -r nf fb h <<< "$spec"
               run desc_${fb}_h$h 600 python bench.py --desc --frags $nf --frag-bytes $fb --rows-hint $h --steps 20 --warmup 60 --no-cpu-baseline
             done &&
             run prof_desc_gm 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_desc_gm -o run \
               -- python3 bench.py --desc --frags 16404 --frag-bytes 65456 --rows-hint 16 --steps 20 --warmup 60 --no-cpu-baseline &&
             run pmc_desc_gm_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_desc_gm_fetch -o run \
               -- python3 bench.py --desc --frags 16404 --frag-bytes 65456 --rows-hint 16 --steps 5 --warmup 1 --no-cpu-baseline ;;
    tests_bcopy) run pytest_bcopy 600 python -m pytest tests/test_gpu_bcopy.py -m gpu -x -q ;;
    tests_chain) run pytest_chain 600 python -m pytest tests/test_gpu_chain.py -m gpu -x -q ;;
    tests_csum64) run pytest_csum64 600 python -m pytest tests/test_gpu_csum64.py -m gpu -x -q ;;
    tests_verify) run pytest_verify 600 python -m pytest tests/test_gpu_verify.py -m gpu -x -q ;;
    tests_native) run pytest_native 600 python -u -m pytest tests/test_gpu_native.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    sweep) run sweep 500 tools/microbench/frags_sweep ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== session done"
