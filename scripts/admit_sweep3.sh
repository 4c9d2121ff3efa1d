# Admission limit sweep on the C3 batch (kernel and wall ms), current kernels
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/admit_sweep3.log
for a in 64 80 96 112 128 96 80 112; do
  timeout -k 10 100 python -u scripts/batch_time.py 256 7 MD_VARIANT=$((a << 16)) >> gpurun_out/admit_sweep3.log 2>&1 || exit 1
done
