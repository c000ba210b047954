set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bcopy.py tests/test_gpu_recv.py tests/test_gpu_chain.py tests/test_gpu_csum64.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_l.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests_l.log; exit 1; }
tail -1 gpurun_out/tests_l.log
timeout -k 10 300 python tools/microbench/msg_bcopy_slots.py > gpurun_out/slots_l.txt 2>&1; cat gpurun_out/slots_l.txt | grep L=
timeout -k 10 300 python bench.py --recv --steps 10 > gpurun_out/recv_l.log 2>&1 && tail -1 gpurun_out/recv_l.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('recv crc', d['roofline']['frac'], d['parity']['ok'])"
timeout -k 10 300 python bench.py --recv --mode sum --steps 10 > gpurun_out/recvs_l.log 2>&1 && tail -1 gpurun_out/recvs_l.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('recv sum', d['roofline']['frac'], d['parity']['ok'])"
timeout -k 10 300 python bench.py --bcopy --steps 10 > gpurun_out/bcopy_l.log 2>&1 && tail -1 gpurun_out/bcopy_l.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('bcopy crc msg', d['roofline']['frac'], 'desc', d['descriptor_batch']['frac'], 'src8', d['descriptor_batch_src8']['frac'], 'dst8', d['descriptor_batch_dst8']['frac'], 'dst1', d['descriptor_batch_dst1']['frac'], d['parity']['ok_all'])"
timeout -k 10 300 python bench.py --bcopy --mode sum --steps 10 > gpurun_out/bcopys_l.log 2>&1 && tail -1 gpurun_out/bcopys_l.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('bcopy sum msg', d['roofline']['frac'], 'desc', d['descriptor_batch']['frac'], 'src8', d['descriptor_batch_src8']['frac'], 'dst8', d['descriptor_batch_dst8']['frac'], 'dst1', d['descriptor_batch_dst1']['frac'], d['parity']['ok_all'])"
