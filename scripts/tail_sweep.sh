# Queue tail threshold (one tile per item once at most 16 k graphs run; MD_VARIANT bits 13-15)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/tail_sweep.log
for k in 0 1 3 7 0 1 3 7; do
  timeout -k 10 100 python -u scripts/batch_time.py 256 7 MD_VARIANT=$((k << 13)) >> gpurun_out/tail_sweep.log 2>&1 || exit 1
done
