set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/park.log
for k in 0 4 8 16; do
  MD_QPARK=$k timeout -k 10 100 python -u scripts/batch_time.py 256 7 MD_QPARK=$k >> gpurun_out/park.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_batch.py -k "paired or queue_admission or c3 or c5 or shard" > gpurun_out/pair_tests.log 2>&1
