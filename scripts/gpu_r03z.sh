#!/bin/bash
# synchronous-hooking union pass: full GPU suite, A/B against MD_SV=0, s0 profile, batch timing
O=gpurun_out/r03z
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step df_prof 240 python -u scripts/df_prof.py gmm1000_s0
