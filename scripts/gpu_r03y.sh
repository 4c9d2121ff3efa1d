#!/bin/bash
O=gpurun_out/r03y
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step ab 400 env AB_VAR=MD_SPEC AB_MODES=16,24,32 python -u scripts/df_ab.py gmm1000_s0,gmm1000_s1,er1000,gmm200_s7 11
step df_prof32 240 env MD_SPEC=32 python -u scripts/df_prof.py gmm1000_s0
