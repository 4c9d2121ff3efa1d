#!/bin/bash
# early speculative requests: parity tests, A/B against MD_EARLY=0, profile
O=gpurun_out/r03v
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step pytest 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step ab 400 env AB_VAR=MD_DF AB_MODES=0,1,2 python -u scripts/df_ab.py gmm1000_s0,gmm1000_s1,er1000,gmm200_s7 15
step df_prof2 240 env MD_DF=2 python -u scripts/df_prof.py gmm1000_s0
