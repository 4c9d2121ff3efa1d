#!/bin/bash
# diagnosis: the dataflow identity test on the index-checked build
O=gpurun_out/r03u
mkdir -p $O
MD_LIB=$PWD/build/libmdroll_dbg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dataflow_mode and unit" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.out 2>&1
echo "rc=$?" >> $O/pytest.out
