#!/bin/bash
O=gpurun_out/r03ai
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dataflow or speculative or prebuild" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.out 2>&1 || { echo "pytest failed"; tail -5 $O/pytest.out; exit 1; }
tail -1 $O/pytest.out
bash scripts/lib_ab.sh $O build/ab/libmdroll_base.so gmm1000_s0,gmm1000_s2,er1000 15
