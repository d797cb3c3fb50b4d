#!/bin/bash
# Interleaved A/B on one box: raw graph launch (default) vs torch's replay every step.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_raw
for rep in 1 2 3; do
  for mode in 1 0; do
    timeout -k 10 120 env VMAS_GRAPH_RAW_LAUNCH=$mode python bench.py --steps 200 --warmup 20 --cpu-steps 0 > gpurun_out/ab_raw/raw${mode}_$rep.json 2> gpurun_out/ab_raw/raw${mode}_$rep.log || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,1), 'M', d['ms_per_step'])" gpurun_out/ab_raw/raw${mode}_$rep.json
  done
done
