#!/bin/bash
# Second round of k_world schedule variants around the defaults (interleaved, one box).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/ab_sched2
mkdir -p $OUT
for rep in 1 2; do
  for v in "base|" "nosplit|VMAS_JIT_SPLIT=0" "fin2|VMAS_JIT_COST_FINISH=2" "fin4|VMAS_JIT_COST_FINISH=4" "ss03|VMAS_JIT_COST_SS=0.3"; do
    name=${v%%|*}; envs=${v#*|}
    timeout -k 10 120 env X=1 $envs python bench.py --steps 60 --warmup 10 --cpu-steps 0 > $OUT/balance_${name}_$rep.json 2> $OUT/balance_${name}_$rep.log || exit 1
    python -c "import json; d=json.load(open('$OUT/balance_${name}_$rep.json')); r=d['roofline']; print('balance $name', r['kernel_us_per_launch'], round(d['value']/1e6,1))"
  done
done
