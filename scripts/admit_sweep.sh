# Admission-limit sweep of queue mode (MD_VARIANT bits 16+ = graphs running at once; 0 = the
# default rule): scripts/admit_sweep.sh "48 64 96" "256 512"
set -e
for K in ${1:-0 64 96 128 160 192}; do
  for NB in ${2:-256 512}; do
    echo "K=$K NB=$NB" >> gpurun_out/admit_sweep.log
    MD_VARIANT=$((K * 65536)) timeout -k 10 60 python scripts/batch_prof.py $NB 2>&1 | grep -E "^batch|idle" >> gpurun_out/admit_sweep.log
  done
done
