set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "small_batch or byte_balanced or across_chains or edges_and_alignment or descriptor_batch_random or two_buffers or maximum_length" > gpurun_out/s9_pytest.log 2>&1 || { tail -30 gpurun_out/s9_pytest.log; exit 1; }
tail -3 gpurun_out/s9_pytest.log
LAMPI_SMALL_BATCH=4096 timeout -k 10 300 python tools/microbench/small_batch.py 2>&1 | grep -v amdgpu.ids
