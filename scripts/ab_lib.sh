#!/bin/bash
# A/B of two library builds, alternating processes (each build run REPS times in turn):
#   bash scripts/ab_lib.sh batch  A.so B.so [graphs]        batch timer (scripts/batch_time.py)
#   bash scripts/ab_lib.sh single A.so B.so [graph]         single-graph kernel median (scripts/spec_prof.py)
#   bash scripts/ab_lib.sh df     A.so B.so GRAPHS [reps]   dataflow A/B timer (scripts/df_ab.py, AB_MODES=k)
# A build may be "" (the in-tree library).  Output: gpurun_out/ab_<mode>.log
set -o pipefail
M=$1; A=$2; B=$3
mkdir -p gpurun_out
LOG=gpurun_out/ab_$M.log
REPS=2; [ "$M" = single ] && REPS=3
for r in $(seq $REPS); do
  for lib in "$A" "$B"; do
    echo "== ${lib:-intree} pass $r" >> $LOG
    case $M in
      batch) MD_LIB=${lib:+$PWD/$lib} timeout -k 10 100 python -u scripts/batch_time.py ${4:-256} 7 >> $LOG 2>&1 || exit 1 ;;
      single) MD_LIB=${lib:+$PWD/$lib} timeout -k 10 100 python -u scripts/spec_prof.py ${4:-gmm1000_s0} 2>&1 | grep -v amdgpu.ids | head -3 >> $LOG || exit 1 ;;
      df) MD_LIB=${lib:+$PWD/$lib} timeout -k 10 300 env AB_MODES=${AB_MODES:-1} python -u scripts/df_ab.py $4 ${5:-15} >> $LOG 2>&1 || exit 1 ;;
      *) echo "mode: batch | single | df" >&2; exit 2 ;;
    esac
  done
done
