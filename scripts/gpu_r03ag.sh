#!/bin/bash
# early speculative requests: parity tests, A/B against MD_EARLY=0, profile
O=gpurun_out/r03ag
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step df_prof 240 python -u scripts/df_prof.py gmm1000_s0
