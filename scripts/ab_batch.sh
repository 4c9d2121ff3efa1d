#!/bin/bash
# A/B of the batch workload (256 graphs, shared mode) across library builds given as arguments.
set -e
mkdir -p gpurun_out
for L in "$@"; do
  MD_LIB=$L timeout -k 10 120 python bench.py --steps 0 --batch-graphs 256 --batch-steps 3 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));b=d['batch'];print('$L',round(b['value']),round(b['ms_per_step'],2))"
done
