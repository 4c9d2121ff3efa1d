# single-graph rollout time (gmm1000_s0, first line of scripts/gpu_prof.py) for MD_VARIANT values, alternating
set -e
VS=${1:-"0 2048"}
mkdir -p gpurun_out
for r in 1 2; do
  for v in $VS; do
    MD_VARIANT=$v timeout -k 10 60 python scripts/gpu_prof.py 0 > gpurun_out/ab_single_run.log 2>&1
    echo -n "MD_VARIANT=$v: "; head -1 gpurun_out/ab_single_run.log
  done
done
