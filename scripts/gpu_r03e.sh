#!/bin/bash
# Speculative-step timelines with and without the dataflow mode.
O=gpurun_out/r03e
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step spec_df1 200 python -u scripts/spec_prof.py gmm1000_s0
MD_DF=0 step spec_df0 200 python -u scripts/spec_prof.py gmm1000_s0
