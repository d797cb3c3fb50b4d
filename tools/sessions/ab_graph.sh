#!/bin/bash
# Interleaved A/B of graph-mode variants on one box (bench line per run -> gpurun_out/ab_graph.log)
set -u
mkdir -p gpurun_out
: > gpurun_out/ab_graph.log
A="${A:-VMAS_GRAPH_PAR_OBS=4}"; B="${B:-VMAS_GRAPH_PAR_OBS=0}"
for rep in 1 2 3; do
  for cfg in "$A" "$B"; do
    v=$(env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 --cpu-steps 0 2>/dev/null | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_us_per_launch'], d['config']['step_mode'])") || exit 1
    echo "$cfg $v" | tee -a gpurun_out/ab_graph.log
  done
done
