# A/B of two library builds on the batch timer, alternating: bash scripts/ab_lib.sh A.so B.so [graphs]
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for lib in "$1" "$2"; do
    echo "== $lib" >> gpurun_out/ab_lib.log
    MD_LIB=$PWD/$lib timeout -k 10 100 python -u scripts/batch_time.py ${3:-256} 7 >> gpurun_out/ab_lib.log 2>&1 || exit 1
  done
done
