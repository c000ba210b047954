set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 tools/microbench/copy2 > gpurun_out/copy2.txt 2>&1 || { echo COPY2_FAIL; tail gpurun_out/copy2.txt; exit 1; }
cat gpurun_out/copy2.txt
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_bc_fetch -o run -- python3 bench.py --bcopy --steps 3 --warmup 1 > gpurun_out/pmc_bc_fetch.log 2>&1 || { echo PMC1_FAIL; tail gpurun_out/pmc_bc_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_bc_write -o run -- python3 bench.py --bcopy --steps 3 --warmup 1 > gpurun_out/pmc_bc_write.log 2>&1 || { echo PMC2_FAIL; tail gpurun_out/pmc_bc_write.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_rv_fetch -o run -- python3 bench.py --recv --steps 3 --warmup 1 > gpurun_out/pmc_rv_fetch.log 2>&1 || { echo PMC3_FAIL; tail gpurun_out/pmc_rv_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_rv_write -o run -- python3 bench.py --recv --steps 3 --warmup 1 > gpurun_out/pmc_rv_write.log 2>&1 || { echo PMC4_FAIL; tail gpurun_out/pmc_rv_write.log; exit 1; }
echo PMC_DONE
