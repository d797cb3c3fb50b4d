#!/bin/bash
# A/B of k_world wave issue priority (VMAS_JIT_PRIO=0|1|2|3) on C2 and C5, interleaved twice.
set -u
mkdir -p gpurun_out/abp
run() {  # tag, prio, bench args
  VMAS_JIT_PRIO=$2 timeout -k 10 200 python bench.py --steps 60 --warmup 10 --cpu-steps 0 $3 > gpurun_out/abp/$1.json 2> gpurun_out/abp/$1.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/abp/$1.json')); r=d['roofline']; print('$1', r['kernel_us_per_launch'], r.get('kernel_us_event'), round(d['value']/1e6,1))"
}
for rep in 1 2; do
  for p in 1 2 3; do
    run bal_p${p}_$rep $p ""
    run fl_p${p}_$rep $p "--scenario flocking --n-agents 8 --substeps 0"
  done
done
