# Admission limit x admission order (seed order / edge count descending) on the C3 batch
set -o pipefail
mkdir -p gpurun_out
for a in 32 48 64 96 128; do
  echo "== admit $a" >> gpurun_out/admit_sweep2.log
  MD_VARIANT=$((a << 16)) timeout -k 10 150 python -u scripts/admit_order.py 256 >> gpurun_out/admit_sweep2.log 2>&1 || exit 1
done
