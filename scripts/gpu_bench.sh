#!/bin/bash
# the default bench line (reads profiles/traffic.json of the same build), then the RCCL world-1 line
O=gpurun_out/bench_${1:-r03}
mkdir -p $O
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --rccl --batch-graphs 0 --degree-steps 0 --real-steps 0 --no-cpu-baseline > $O/rccl.json 2> $O/rccl.err
echo "rccl rc=$?"
