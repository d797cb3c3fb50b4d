#!/bin/bash
# A/B of the specialised kernel's waves per workgroup (VMAS_JIT_WAVES=8|16) across configs.
set -u
mkdir -p gpurun_out/ab
for nw in 8 16; do
  for cfg in "balance|" "transport|--scenario transport --substeps 0" "flocking|--scenario flocking --n-agents 8 --substeps 0" "discovery|--scenario discovery --envs 16384 --n-agents 8 --substeps 0 --kw {\"use_agent_lidar\":true}"; do
    name=${cfg%%|*}; args=${cfg#*|}
    VMAS_JIT_WAVES=$nw timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-steps 0 $args > gpurun_out/ab/${name}_$nw.json 2> gpurun_out/ab/${name}_$nw.log || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab/${name}_$nw.json')); r=d['roofline']; print('$name', $nw, r['kernel'], r['kernel_us_per_launch'], d['ms_per_step'])"
  done
done
VMAS_JIT_WAVES=16 timeout -k 10 200 python tools/jit_phase_profile.py balance 32768 200 > gpurun_out/ab/phase16.log 2>&1 || exit $?
