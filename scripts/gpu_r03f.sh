#!/bin/bash
O=gpurun_out/r03f
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step df_prof 200 python -u scripts/df_prof.py gmm1000_s0
step df_ab 200 python -u scripts/df_ab.py gmm1000_s0 21
