set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/park.log
for v in 0 1536 0 1536; do
  timeout -k 10 100 python -u scripts/batch_time.py 256 7 MD_VARIANT=$v >> gpurun_out/park.log 2>&1 || exit 1
done
