# A/B timings of the batch launches: bash scripts/wq_ab.sh "<env settings ...>" graphs reps
#   each setting is a comma list for batch_time.py, e.g. "MD_WQPARK=96 MD_WQPARK=160,MD_LIB=..."
set -e
mkdir -p gpurun_out
for S in $1; do
  timeout -k 10 150 python scripts/batch_time.py $2 ${3:-3} $S >> gpurun_out/wq_ab.log 2>&1
done
