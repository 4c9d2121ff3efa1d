#!/bin/bash
# Round profile on the GPU box (run from the repo root): the default bench line, rocprofv3
# kernel-trace stats of the single-graph and batch workloads, and PMC passes of both
# (FETCH_SIZE / WRITE_SIZE for HBM traffic; two SQ passes for MFMA busy / instruction mix / LDS;
# GRBM_GUI_ACTIVE for the clock), one counter group per run (MI355X_MICROARCH.md PMC slots).
# Then scripts/rocprof_summary.py writes summary.txt and traffic.json (tagged with the kernel
# source hash that bench.py checks).
# Usage: bash scripts/gpu_profile_round.sh r02 [--no-bench]
set -e
TAG=${1:-r02}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "--no-bench" ]; then
  timeout -k 10 500 python $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
  echo "bench done"
fi
SINGLE="--batch-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 0"
BATCH="--steps 0 --batch-graphs 256 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 0"
SQ1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
SQ2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/single -o run -- python $R/bench.py $SINGLE > $OUT/single.log 2>&1
echo "single kernel trace done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/batch -o run -- python $R/bench.py $BATCH --batch-steps 2 > $OUT/batch.log 2>&1
echo "batch kernel trace done"
for W in single batch; do
  if [ $W = single ]; then ARGS="$SINGLE --steps 2 --warmup 1"; else ARGS="$BATCH --batch-steps 1"; fi
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$W -o run -- python $R/bench.py $ARGS > $OUT/pmc_fetch_$W.log 2>&1
  echo "$W fetch pass done"
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$W -o run -- python $R/bench.py $ARGS > $OUT/pmc_write_$W.log 2>&1
  echo "$W write pass done"
  timeout -s KILL 180 rocprofv3 --pmc $SQ1 -d $OUT/pmc_sq1_$W -o run -- python $R/bench.py $ARGS > $OUT/pmc_sq1_$W.log 2>&1
  echo "$W sq1 pass done"
  timeout -s KILL 180 rocprofv3 --pmc $SQ2 -d $OUT/pmc_sq2_$W -o run -- python $R/bench.py $ARGS > $OUT/pmc_sq2_$W.log 2>&1
  echo "$W sq2 pass done"
done
cd $R
python scripts/rocprof_summary.py $OUT > /dev/null
echo "summary done"
