set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/xcd.log
for k in 0 1 0 1; do
  timeout -k 10 100 python -u scripts/batch_time.py 256 7 MD_QXCD=$k >> gpurun_out/xcd.log 2>&1 || exit 1
done
MD_QXCD=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_parity.py -k "batch or paired or queue_admission or shared" > gpurun_out/xcd_tests.log 2>&1
