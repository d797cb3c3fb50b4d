#!/bin/bash
# Eager-step (graph_step=False, the reference's default API) bench lines for C2-C5.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/eager
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-steps 0 --graph off "$@" > $OUT/$name.json 2> $OUT/$name.log || exit 1
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value']/1e6,2), 'M', d['ms_per_step'], d['config']['step_mode'])"
}
run c2_balance_sub10
run c3_transport --scenario transport --substeps 0
run c4_discovery --scenario discovery --envs 16384 --n-agents 8 --substeps 0 --kw '{"use_agent_lidar": true}'
run c5_flocking --scenario flocking --n-agents 8 --substeps 0
