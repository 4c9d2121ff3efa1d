#!/bin/bash
# Round profile on the GPU box (run from the repo root), in this order so that the bench line
# carries the traffic measured from the same build in the same session:
#  1. rocprofv3 kernel-trace stats of the single-graph, batch (256), C5 (4096), degree-cost and
#     N = 18 000 testReal-sized (degree step 1, unit stepRatio 0.01) workloads;
#  2. PMC passes of every workload (HBM traffic and the SQ_1 group; SQ_2/SQ_3 for the single
#     graph and the batch), one counter group per run
#     (FETCH_SIZE / WRITE_SIZE for HBM traffic; SQ groups for MFMA busy, wave states, LDS, the
#     instruction mix; GRBM_GUI_ACTIVE for the clock; MI355X_MICROARCH.md PMC slots);
#  3. scripts/rocprof_summary.py -> summary.txt + traffic.json (tagged with the kernel source
#     hash), copied to profiles/traffic.json where bench.py reads it;
#  4. the default bench line.
# Usage: bash scripts/gpu_profile_round.sh r03 [nobench]
# (WL="single batch" limits the workloads; PART=a summarises that part on the box and deletes its
# databases, for a round split over several gpurun calls: merge with rocprof_summary.py --merge)  (then bench.py on its own, reading the
# profiles/traffic.json copied from gpurun_out/prof_<tag>/traffic.json)
TAG=${1:-r03}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SINGLE="--batch-graphs 0 --c5-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 0"
BATCH="--steps 0 --batch-graphs 256 --c5-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 0"
C5="--steps 0 --batch-graphs 0 --c5-graphs 4096 --c5-steps 1 --c5-shard-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 0"
DEGREE="--steps 0 --batch-graphs 0 --c5-graphs 0 --no-cpu-baseline --degree-steps 2 --no-per-step --real-steps 0"
REAL_DEGREE="--steps 0 --batch-graphs 0 --c5-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 1 --real-cases degree"
REAL_UNIT="--steps 0 --batch-graphs 0 --c5-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 1 --real-cases unit"
SQ1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
SQ2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES"
SQ3="SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES"
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
cd /tmp
WL=${WL:-single batch c5 degree real_degree real_unit}
for W in $WL; do
  case $W in
    single) run single_trace 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/single -o run -- python $R/bench.py $SINGLE ;;
    batch) run batch_trace 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/batch -o run -- python $R/bench.py $BATCH --batch-steps 2 ;;
    c5) run c5_trace 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/c5 -o run -- python $R/bench.py $C5 ;;
    degree) run degree_trace 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/degree -o run -- python $R/bench.py $DEGREE ;;
    real_degree) run real_degree_trace 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/real_degree -o run -- python $R/bench.py $REAL_DEGREE ;;
    real_unit) run real_unit_trace 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/real_unit -o run -- python $R/bench.py $REAL_UNIT ;;
  esac
done
for W in $WL; do
  case $W in
    single) ARGS="$SINGLE --steps 2 --warmup 1" ;;
    batch) ARGS="$BATCH --batch-steps 1" ;;
    c5) ARGS="$C5" ;;
    degree) ARGS="$DEGREE" ;;
    real_degree) ARGS="$REAL_DEGREE" ;;
    real_unit) ARGS="$REAL_UNIT" ;;
  esac
  run pmc_fetch_$W 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$W -o run -- python $R/bench.py $ARGS
  run pmc_write_$W 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$W -o run -- python $R/bench.py $ARGS
  run pmc_sq1_$W 240 rocprofv3 --pmc $SQ1 -d $OUT/pmc_sq1_$W -o run -- python $R/bench.py $ARGS
  if [ $W = single ] || [ $W = batch ]; then
    run pmc_sq2_$W 180 rocprofv3 --pmc $SQ2 -d $OUT/pmc_sq2_$W -o run -- python $R/bench.py $ARGS
    timeout -s KILL 120 rocprofv3 --pmc $SQ3 -d $OUT/pmc_sq3_$W -o run -- python $R/bench.py $ARGS > $OUT/pmc_sq3_$W.log 2>&1
    echo "pmc_sq3_$W rc=$? (optional)"
  fi
done
cd $R
if [ -n "${PART:-}" ]; then
  # one part of a round split over gpurun calls: summarise this part's databases here and drop
  # them (the merged-back gpurun_out/ is capped at 64 MiB); merge the parts' traffic_<part>.json
  # afterwards (scripts/rocprof_summary.py --merge)
  python scripts/rocprof_summary.py $OUT > /dev/null && mv $OUT/traffic.json $OUT/traffic_$PART.json && \
    mv $OUT/summary.txt $OUT/summary_$PART.txt && find $OUT -name "*.db" -delete && echo "summary $PART done"
  exit $?
fi
python scripts/rocprof_summary.py $OUT > /dev/null && cp $OUT/traffic.json profiles/traffic.json && echo "summary done"
if [ "${2:-}" != "nobench" ]; then
  timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
  echo "bench rc=$?"
fi
