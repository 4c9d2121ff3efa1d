#!/bin/bash
# Baseline phase profiles of the current build: single-graph per-step stamps, queue-mode pieces.
O=gpurun_out/r03c
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step single_prof 300 python -u scripts/gpu_prof.py 0
MD_LIB=$PWD/mdcommunity_amd/csrc/build/libmdroll_qprof.so MD_VARIANT=8 step batch_qprof 300 python -u scripts/batch_prof.py 256
