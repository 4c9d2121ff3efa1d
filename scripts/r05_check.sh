#!/bin/bash
# Round-5 kernel iteration check: wave-item identity, the batch tests, C3/C5 timings, the slot-0
# timeline and the piece profile at 32 graphs (gpurun_out/r05/t.log, gpurun_out/wq_ab.log).
set -e
mkdir -p gpurun_out/r05
O=gpurun_out/r05/t.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k 'wave_items' --timeout 240 --timeout-method thread > $O 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread >> $O 2>&1
bash scripts/wq_ab.sh "${AB:-MD_WQPARK=96}" 256 3
bash scripts/wq_ab.sh 'MD_WQPARK=96' 4096 2
MD_PROF_ALL=1 MD_VARIANT=$((256*65536+4)) MD_WQPARK=0 timeout -k 10 120 python scripts/wq_timeline.py 32 >> $O 2>&1
MD_LIB=mdcommunity_amd/csrc/build/libmdroll_qprof.so MD_WQPARK=0 MD_VARIANT=8 timeout -k 10 120 python scripts/batch_prof.py 32 >> $O 2>&1
