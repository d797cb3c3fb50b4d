#!/bin/bash
set -u
mkdir -p gpurun_out
for cap in 512 510 480 256; do
  echo "== cap $cap"
  VMAS_JIT_GRID_CAP=$cap timeout -k 10 120 python tools/graph_probe.py balance 2>&1 | grep -v amdgpu.ids | tail -3 || exit $?
done
