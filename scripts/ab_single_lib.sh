# A/B of two library builds on the single-graph rollout (spec_prof's kernel median), alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in "$1" "$2"; do
    echo "== $lib" >> gpurun_out/ab_single_lib.log
    MD_LIB=$PWD/$lib timeout -k 10 100 python -u scripts/spec_prof.py ${3:-gmm1000_s0} 2>&1 | grep -v amdgpu.ids | head -3 >> gpurun_out/ab_single_lib.log || exit 1
  done
done
