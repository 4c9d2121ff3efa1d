#!/bin/bash
# Latency probe of the wave-item kernel: slot-0 timelines at two batch sizes (all steps in
# md_wq_kernel), a piece profile at 32 graphs, the per-step time of small dedicated launches,
# and the cascade's dispatches at 256.
set -e
mkdir -p gpurun_out/r05
O=gpurun_out/r05/lat.log
: > $O
for nb in 32 256; do
  MD_PROF_ALL=1 MD_VARIANT=$((256*65536+4)) MD_WQPARK=0 timeout -k 10 120 python scripts/wq_timeline.py $nb >> $O 2>&1
done
for nb in 1 8 17 32; do
  timeout -k 10 120 python scripts/batch_time.py $nb 3 >> $O 2>&1
done
timeout -k 10 120 python scripts/batch_time.py 32 3 MD_WQPARK=0 >> $O 2>&1
MD_LIB=mdcommunity_amd/csrc/build/libmdroll_qprof.so MD_WQPARK=0 MD_VARIANT=8 timeout -k 10 120 python scripts/batch_prof.py 32 >> $O 2>&1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/kt256 -o kt -- python3 scripts/batch_time.py 256 2 >> $O 2>&1
