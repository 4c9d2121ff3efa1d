#!/bin/bash
# synchronous-hooking union pass: full GPU suite, A/B against MD_SV=0, s0 profile, batch timing
O=gpurun_out/r03w
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
step ab 400 env AB_VAR=MD_SV AB_MODES=0,1 python -u scripts/df_ab.py gmm1000_s0,gmm1000_s1,er1000,gmm200_s7 15
step s0 120 python -u scripts/s0_prof.py
step s0_old 120 env MD_SV=0 python -u scripts/s0_prof.py
step df_prof 240 python -u scripts/df_prof.py gmm1000_s0
step batch_new 240 python -u scripts/batch_time.py 256 5 MD_SV=1
step batch_old 240 python -u scripts/batch_time.py 256 5 MD_SV=0
