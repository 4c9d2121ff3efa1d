#!/bin/bash
# Dataflow mode with the rank-0 prebuild: debug-bounds build first on the case that faulted,
# then the normal build's A/B, profile and GPU tests.  Stops at the first failure.
O=gpurun_out/r03h
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
MD_LIB=$PWD/build/libmdroll_dbg.so MD_DF=1 step dbg_df1_g200 60 python -u scripts/df_one.py gmm200_s7 5
MD_LIB=$PWD/build/libmdroll_dbg.so MD_DF=1 step dbg_df1_g1000 60 python -u scripts/df_one.py gmm1000_s0 5
MD_LIB=$PWD/build/libmdroll_dbg.so MD_DF=1 step dbg_df1_er100 60 python -u scripts/df_one.py er100 5
DF_MODES=0,2,1 step df_ab 400 python -u scripts/df_ab.py gmm1000_s0,gmm1000_s1,er1000,gmm200_s7 15
step df_prof 240 python -u scripts/df_prof.py gmm1000_s0
step pytest 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_degree.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
