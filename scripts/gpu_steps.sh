#!/bin/bash
# Runs GPU steps one after another on the gpurun box, each under its own time limit, output in
# OUTDIR/<k>.out / .err, stopping at the first failure (no retries):
#   bash scripts/gpu_steps.sh OUTDIR SECONDS "command 1" "command 2" ...
# e.g. the round-3 A/B measurements in DESIGN.md:
#   bash scripts/gpu_steps.sh gpurun_out/ab 400 \
#     "env AB_VAR=MD_EARLY AB_MODES=0,1 python -u scripts/df_ab.py gmm1000_s0,gmm1000_s1,er1000,gmm200_s7 15" \
#     "env AB_VAR=MD_SPEC AB_MODES=16,24,32 python -u scripts/df_ab.py gmm1000_s0,er1000 11" \
#     "python -u scripts/df_prof.py gmm1000_s0"
O=$1; S=$2; shift 2
mkdir -p "$O"
k=0
for cmd in "$@"; do
  k=$((k + 1))
  timeout -k 10 "$S" bash -c "$cmd" > "$O/$k.out" 2> "$O/$k.err"
  rc=$?
  echo "step $k rc=$rc: $cmd" | tee -a "$O/steps.txt"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
