#!/bin/bash
# A/B of the k_world task placement on balance C2: VMAS_JIT_SCHED=simd|wave x VMAS_JIT_COSTS=
# relaxed|exact (cost table), interleaved twice; prints in-kernel / HIP-event k_world us.
set -u
mkdir -p gpurun_out/abs
run() {  # tag, sched, costs, bench args
  VMAS_JIT_SCHED=$2 VMAS_JIT_COSTS=$3 timeout -k 10 200 python bench.py --steps 60 --warmup 10 --cpu-steps 0 $4 > gpurun_out/abs/$1.json 2> gpurun_out/abs/$1.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/abs/$1.json')); r=d['roofline']; print('$1', r['kernel_us_per_launch'], r.get('kernel_us_event'), round(d['value']/1e6,1))"
}
for rep in 1 2; do
  for m in simd wave; do
    for c in relaxed exact; do
      run bal_${m}_${c}_$rep $m $c ""
    done
  done
done
