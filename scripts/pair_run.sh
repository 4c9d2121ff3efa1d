set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_batch.py -k "paired or queue_admission or shared_mode or c3 or c5 or shard" > gpurun_out/pair_tests.log 2>&1 && \
timeout -k 10 200 python -u scripts/admit_order.py 256 > gpurun_out/pair_time.log 2>&1 && \
MD_PAIR=0 timeout -k 10 200 python -u scripts/admit_order.py 256 > gpurun_out/pair_time0.log 2>&1
