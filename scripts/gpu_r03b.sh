#!/bin/bash
O=gpurun_out/r03b
mkdir -p $O
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest_batch 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -p no:cacheprovider
step sweep 400 python -u scripts/admit_sweep_c5.py 4096 0,96,256,384,640 2
step sweep512 200 python -u scripts/admit_sweep_c5.py 512 0 3
