set -e
R=$(pwd)
mkdir -p gpurun_out/l2
export TMPDIR=/tmp
cd /tmp
MD_QXCD=${QXCD:-0} timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/l2/pmc -o run -- python $R/bench.py --steps 0 --batch-graphs 256 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 0 --batch-steps 1 > $R/gpurun_out/l2/run.log 2>&1
echo done
