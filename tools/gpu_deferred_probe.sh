#!/bin/bash
set -u
mkdir -p gpurun_out/dp
export TMPDIR=/tmp
for v in "PROBE_CLONE=1" "PROBE_CLONE=0" "PROBE_CLONE=1 VMAS_GRAPH_DEFERRED_SPAWN=0"; do
  echo "=== $v"
  env $v timeout -k 10 120 python tools/deferred_probe.py 777 > gpurun_out/dp/probe.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/dp/probe.log | tail -16
  case $rc in 0|1) ;; *) exit $rc;; esac
done
