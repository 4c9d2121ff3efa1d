# Admission sweep of the batch kernels (MD_VARIANT bits 16+ = graphs running at once):
#   bash scripts/wq_sweep.sh "96 160 256" 256 [reps]   -> gpurun_out/wq_sweep.log
set -e
mkdir -p gpurun_out
for K in $1; do
  timeout -k 10 120 python scripts/batch_time.py $2 ${3:-3} MD_VARIANT=$((K * 65536)) >> gpurun_out/wq_sweep.log 2>&1
done
