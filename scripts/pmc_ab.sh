#!/bin/bash
# WRITE_SIZE per md_rollout_kernel dispatch of the single-graph bench workload under several
# settings, one rocprofv3 PMC pass each, same box (run from the repo root):
#   CFGS="base:MD_EG_APPLY=1 loop:MD_EG_APPLY=0 other:MD_LIB=$PWD/other/libmdroll.so" bash scripts/pmc_ab.sh
# Each config is name:ENV=VALUE (ENV=VALUE may be empty: name: runs the defaults).  Output:
# gpurun_out/pmc_ab/<name>/run_counter_collection.csv (sum Counter_Value per Dispatch_Id of
# md_rollout_kernel for the bytes per launch).  Used for the trace-publish placement.
R=$(pwd)
OUT=$R/gpurun_out/pmc_ab
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--batch-graphs 0 --c5-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 0 --steps 2 --warmup 1"
for cfg in ${CFGS:-base: loop:MD_EG_APPLY=0}; do
  name=${cfg%%:*}
  E=${cfg#*:}
  env $E timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/$name -o run -- python $R/bench.py $ARGS > $OUT/$name.log 2>&1 || exit 1
  echo "$name done"
done
