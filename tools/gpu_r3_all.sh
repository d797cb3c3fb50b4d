#!/bin/bash
# Quick discovery check (C4 bench twice), then the whole round-3 evidence session, then the clash probe.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
for i in 1 2; do
  echo "=== bench_c4_$i ($(date +%T))"
  timeout -k 10 200 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/r3d/bench_c4_$i.log 2>&1
  rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3d/bench_c4_$i.log | tail -c 400; echo
  case $rc in 0|1) ;; *) exit $rc;; esac
done
bash tools/gpu_r3_final.sh || exit $?
timeout -k 10 120 python tools/clash_probe.py flocking 4096 8 > gpurun_out/r3d/clash.log 2>&1
grep -v amdgpu.ids gpurun_out/r3d/clash.log | tail -12
