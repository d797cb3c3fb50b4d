#!/bin/bash
# A/B of the broadphase fixed point's driver (VMAS_JIT_GRID=host|coop|plain) across configs:
# host-driven passes (one sync per pass) vs one persistent launch (device-side passes).
set -u
mkdir -p gpurun_out/abg
for mode in host coop plain; do
  for cfg in "balance|" "transport|--scenario transport --substeps 0" "flocking|--scenario flocking --n-agents 8 --substeps 0"; do
    name=${cfg%%|*}; args=${cfg#*|}
    VMAS_JIT_GRID=$mode timeout -k 10 300 python bench.py --steps 100 --warmup 20 --cpu-steps 0 $args > gpurun_out/abg/${name}_$mode.json 2> gpurun_out/abg/${name}_$mode.log || exit $?
    python -c "import json; d=json.load(open('gpurun_out/abg/${name}_$mode.json')); r=d['roofline']; print('$name', '$mode', r['kernel'], r['kernel_us_per_launch'], d['ms_per_step'], d['value'])"
  done
done
