#!/bin/bash
# round-end check on the GPU box: the GPU test suite, then the profile round (traces, PMC
# passes, summary) of the same build; the bench line runs after profiles/traffic.json is copied
set -o pipefail
O=gpurun_out/final_${1:-r03}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.out 2>&1
rc=$?
tail -2 $O/pytest.out
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_profile_round.sh ${1:-r03} nobench
