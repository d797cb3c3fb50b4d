#!/bin/bash
# Interleaved A/B on one box: speculative replay (default) vs waiting for the action flags first.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_spec
for rep in 1 2 3; do
  for mode in 1 0; do
    timeout -k 10 120 env VMAS_GRAPH_SPECULATIVE=$mode python bench.py --steps 200 --warmup 20 --cpu-steps 0 > gpurun_out/ab_spec/spec${mode}_$rep.json 2> gpurun_out/ab_spec/spec${mode}_$rep.log || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,1), 'M', d['ms_per_step'])" gpurun_out/ab_spec/spec${mode}_$rep.json
  done
done
