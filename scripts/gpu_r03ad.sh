#!/bin/bash
# queue-mode tail: park threshold sweep (256 and 512 graphs)
O=gpurun_out/r03ad
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
for q in 8 12 16 4; do
  step b256_q$q 200 python -u scripts/batch_time.py 256 5 MD_QPARK=$q
done
for q in 8 16; do
  step b512_q$q 200 python -u scripts/batch_time.py 512 3 MD_QPARK=$q
done
