#!/bin/bash
# Phase profiles of the current build: single-graph device stamps (gpu_prof.py), the speculative
# timeline (spec_prof.py), the queue-mode per-piece profile (qprof build, batch_prof.py).
O=gpurun_out/r03prof
mkdir -p $O
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step gpu_prof 200 python -u scripts/gpu_prof.py 0
step spec_prof 200 python -u scripts/spec_prof.py gmm1000_s0
MD_LIB=$PWD/mdcommunity_amd/csrc/build/libmdroll_qprof.so MD_VARIANT=8 step batch_prof 300 python -u scripts/batch_prof.py 256
