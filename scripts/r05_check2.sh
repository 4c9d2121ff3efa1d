#!/bin/bash
# Round-5 check: batch-speculation identity, wave identity, batch tests, then C3/C5 timings
set -e
mkdir -p gpurun_out/r05
O=gpurun_out/r05/t2.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k 'batch_speculation or wave_items' --timeout 300 --timeout-method thread > $O 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread >> $O 2>&1
bash scripts/wq_ab.sh "${AB:-MD_BSPEC=1 MD_BSPEC=0}" 256 3
bash scripts/wq_ab.sh "${AB5:-MD_BSPEC=1 MD_BSPEC=0}" 4096 2
