#!/bin/bash
# k_world pair-schedule variants (LPT cost knobs), interleaved on one box: balance + transport.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/ab_sched
mkdir -p $OUT
for rep in 1 2; do
  for v in "base|" "ss05|VMAS_JIT_COST_SS=0.5" "fin3lpt|VMAS_JIT_FINISH_LPT=1 VMAS_JIT_COST_FINISH=3" "fin2lpt|VMAS_JIT_FINISH_LPT=1 VMAS_JIT_COST_FINISH=2" "ss05fin3|VMAS_JIT_COST_SS=0.5 VMAS_JIT_FINISH_LPT=1 VMAS_JIT_COST_FINISH=3"; do
    name=${v%%|*}; envs=${v#*|}
    for cfg in "balance|" "transport|--scenario transport --substeps 0"; do
      sc=${cfg%%|*}; args=${cfg#*|}
      timeout -k 10 120 env X=1 $envs python bench.py --steps 60 --warmup 10 --cpu-steps 0 $args > $OUT/${sc}_${name}_$rep.json 2> $OUT/${sc}_${name}_$rep.log || exit 1
      python -c "import json; d=json.load(open('$OUT/${sc}_${name}_$rep.json')); r=d['roofline']; print('$sc $name', r['kernel_us_per_launch'], round(d['value']/1e6,1))"
    done
  done
done
