#!/bin/bash
O=gpurun_out/r03af
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step pytest 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dataflow or speculative or prebuild" --timeout 200 --timeout-method thread -p no:cacheprovider
step ab 500 env AB_VAR=MD_DF AB_MODES=1,2 python -u scripts/df_ab.py gmm1000_s0,gmm1000_s1,gmm1000_s2,er1000,gmm200_s7 15
