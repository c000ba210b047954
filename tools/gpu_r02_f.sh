set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export LAMPI_BENCH_BACKEND=gloo LAMPI_BENCH_SHARE_GPU=1
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/rehearse_g2.log 2>&1 || { echo G2_FAIL; tail -20 gpurun_out/rehearse_g2.log; exit 1; }
grep '^{' gpurun_out/rehearse_g2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('g2', d['n_gpus'], d['value'], d['parity'], [ (p['rank'], p['roofline_frac']) for p in d['per_gpu']], d['aggregate'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 4 --steps 5 --warmup 2 > gpurun_out/rehearse_g4.log 2>&1 || { echo G4_FAIL; tail -20 gpurun_out/rehearse_g4.log; exit 1; }
grep '^{' gpurun_out/rehearse_g4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('g4', d['n_gpus'], d['value'], d['parity'], [ (p['rank'], p['roofline_frac']) for p in d['per_gpu']])"
unset LAMPI_BENCH_BACKEND LAMPI_BENCH_SHARE_GPU
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/torchrun_g2_fail.log 2>&1; echo "torchrun nccl g2 on 1 GPU rc=$? (expected nonzero)"; grep -m2 "need" gpurun_out/torchrun_g2_fail.log
timeout -k 10 200 python bench.py --latency > gpurun_out/latency_f.log 2>&1 && tail -1 gpurun_out/latency_f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['results'][-1])"
