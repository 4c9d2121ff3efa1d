#!/bin/bash
# queue-mode piece profile (qprof build)
O=gpurun_out/r03ae
mkdir -p $O
timeout -k 10 300 env MD_LIB=$PWD/mdcommunity_amd/csrc/build/libmdroll_qprof.so MD_VARIANT=8 python -u scripts/batch_prof.py 256 > $O/qprof.out 2> $O/qprof.err
echo "qprof rc=$?"
timeout -k 10 300 env MD_LIB=$PWD/mdcommunity_amd/csrc/build/libmdroll_qprof.so python -u scripts/batch_prof.py 256 > $O/qidle.out 2> $O/qidle.err
echo "qidle rc=$?"
