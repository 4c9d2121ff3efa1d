#!/bin/bash
O=gpurun_out/r03i
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
MD_LIB=$PWD/build/libmdroll_dbg.so MD_DF=1 step dbg_df1_g1000 120 python -u scripts/df_one.py gmm1000_s0 12
MD_DF=1 step df1_g1000 120 python -u scripts/df_one.py gmm1000_s0 20
MD_DF=1 step df1_er1000 120 python -u scripts/df_one.py er1000 10
MD_DF=1 step df1_g200 120 python -u scripts/df_one.py gmm200_s7 20
DF_MODES=0,2,1 step df_ab 400 python -u scripts/df_ab.py gmm1000_s0,gmm1000_s1,er1000,gmm200_s7 15
step df_prof 240 python -u scripts/df_prof.py gmm1000_s0
step pytest 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_degree.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
