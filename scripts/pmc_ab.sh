#!/bin/bash
# WRITE_SIZE per md_rollout_kernel dispatch, MD_EG_APPLY=1 vs 0 vs MD_VARIANT=2048 (no end-game), same box
R=$(pwd)
OUT=$R/gpurun_out/pmc_ab
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--batch-graphs 0 --c5-graphs 0 --no-cpu-baseline --degree-steps 0 --no-per-step --real-steps 0 --steps 2 --warmup 1"
for cfg in ${CFGS:-a1 a0 v2048}; do
  case $cfg in
    a1) E="MD_EG_APPLY=1" ;;
    a0) E="MD_EG_APPLY=0" ;;
    v2048) E="MD_VARIANT=2048" ;;
    old) E="MD_LIB=$R/ab/libold.so" ;;
    new) E="MD_EG_APPLY=1" ;;
    nostc) E="MD_LIB=$R/ab/libnostc.so" ;;
    nopub) E="MD_LIB=$R/ab/libnopub.so" ;;
    nocopy) E="MD_LIB=$R/ab/libnocopy.so" ;;
  esac
  env $E timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/$cfg -o run -- python $R/bench.py $ARGS > $OUT/$cfg.log 2>&1 || exit 1
  echo "$cfg done"
done
