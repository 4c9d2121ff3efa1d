#!/bin/bash
# Round-3 first GPU pass: host CPU facts, GPU tests, the C4 real-scale dump, the RCCL branch at
# world size 1, the default bench line.  Each GPU step under its own time limit; stops after a
# timeout / abort / fault (exit status other than 0 or 1).
O=gpurun_out/r03a
mkdir -p $O
{ echo "nproc $(nproc)"; python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
  cat /sys/fs/cgroup/cpu.max 2>&1; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; free -g | head -2; } > $O/host.txt
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step dump_real 300 python -u scripts/dump_real_scale.py
step rccl1 300 python -u bench.py --rccl --steps 3 --warmup 1 --batch-graphs 64 --c5-graphs 128 --degree-steps 0 --real-steps 0 --no-cpu-baseline --no-per-step
step bench 900 python -u bench.py
