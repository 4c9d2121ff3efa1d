#!/bin/bash
# Round profile on the GPU box: bench line, rocprofv3 kernel-trace stats of the bench command
# (single-graph workload and batch workload separately), PMC FETCH_SIZE / WRITE_SIZE passes of both.
# Usage (from the repo root): bash scripts/gpu_profile_round.sh r01
set -e
TAG=${1:-r01}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "bench done"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/single -o run -- python $R/bench.py --batch-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step > $OUT/single.log 2>&1
echo "single profile done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/batch -o run -- python $R/bench.py --steps 0 --batch-graphs 256 --batch-steps 2 --no-cpu-baseline --degree-steps 0 --no-per-step > $OUT/batch.log 2>&1
echo "batch profile done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python $R/bench.py --batch-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --steps 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1
echo "fetch pass done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python $R/bench.py --batch-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --steps 2 --warmup 1 > $OUT/pmc_write.log 2>&1
echo "write pass done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_batch -o run -- python $R/bench.py --steps 0 --batch-graphs 256 --batch-steps 1 --no-cpu-baseline --degree-steps 0 --no-per-step > $OUT/pmc_fetch_batch.log 2>&1
echo "batch fetch pass done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_batch -o run -- python $R/bench.py --steps 0 --batch-graphs 256 --batch-steps 1 --no-cpu-baseline --degree-steps 0 --no-per-step > $OUT/pmc_write_batch.log 2>&1
echo "batch write pass done"
cd $R
python scripts/rocprof_summary.py $OUT > /dev/null
find $OUT -name "*stats*.csv" | head -20
