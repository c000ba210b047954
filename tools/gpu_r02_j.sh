set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bcopy.py tests/test_gpu_recv.py tests/test_gpu_chain.py tests/test_gpu_csum64.py tests/test_gpu_parity.py tests/test_gpu_native.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_j.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests_j.log; exit 1; }
tail -1 gpurun_out/tests_j.log
for e in 1 2; do
LAMPI_EXP_SUMROWS=$e timeout -k 10 600 python -u -m pytest tests/test_gpu_bcopy.py tests/test_gpu_recv.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_j$e.log 2>&1 || { echo TESTS_FAIL_$e; tail -40 gpurun_out/tests_j$e.log; exit 1; }
tail -1 gpurun_out/tests_j$e.log
done
for e in 0 1 2 0 1 2; do
if [ $e != 0 ]; then export LAMPI_EXP_SUMROWS=$e; else unset LAMPI_EXP_SUMROWS; fi
timeout -k 10 300 python bench.py --recv --mode sum --steps 10 --warmup 3 > gpurun_out/recv_sum_j.log 2>&1 && tail -1 gpurun_out/recv_sum_j.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp=$e recv sum', d['roofline']['frac'], d['parity']['ok'])"
timeout -k 10 300 python bench.py --bcopy --mode sum --steps 10 > gpurun_out/bcopysum_j.log 2>&1 && tail -1 gpurun_out/bcopysum_j.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('exp=$e bcopy sum msg', d['roofline']['frac'], 'desc', d['descriptor_batch']['frac'], 'src8', d['descriptor_batch_src8']['frac'], 'dst8', d['descriptor_batch_dst8']['frac'], 'dst1', d['descriptor_batch_dst1']['frac'], d['parity']['ok_all'])"
done
