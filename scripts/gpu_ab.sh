#!/bin/bash
# A/B of two library builds: correctness tests on the first (default build), then alternating
# batch timings (scripts/ab_lib.sh batch) and single-graph timings (scripts/ab_lib.sh single).
# Usage: bash scripts/gpu_ab.sh A.so B.so [tests]
O=gpurun_out/ab
mkdir -p $O
rm -f gpurun_out/ab_batch.log gpurun_out/ab_single.log
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest $3 -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.out 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.out
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
bash scripts/ab_lib.sh batch $1 $2 256 || exit $?
grep -h "batch\|==" gpurun_out/ab_batch.log
if [ "$4" == "single" ]; then
  bash scripts/ab_lib.sh single $1 $2 || exit $?
  cat gpurun_out/ab_single.log
fi
