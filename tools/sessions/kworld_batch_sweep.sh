#!/bin/bash
# k_world time per launch vs batch size (balance, 10 substeps, graph mode): is the kernel
# latency-bound (flat) or throughput-bound (linear in B) around the benchmark's 32 768 envs?
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for B in 4096 8192 16384 32768 65536 131072; do
  timeout -k 10 200 python bench.py --envs $B --steps 30 --warmup 10 --cpu-steps 0 > gpurun_out/sweep/b$B.json 2> gpurun_out/sweep/b$B.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sweep/b$B.json')); r=d['roofline']; print($B, r['kernel_us_per_launch'], round(d['value']/1e6,1), d['ms_per_step'], r['valu_issue']['frac'] if r.get('valu_issue') else None)"
done
