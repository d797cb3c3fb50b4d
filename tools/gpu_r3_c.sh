#!/bin/bash
set -u
mkdir -p gpurun_out/r3c
export TMPDIR=/tmp
for v in 1 0; do
  echo "=== probe3 PROBE_SPEC=$v"
  PROBE_SPEC=$v timeout -k 10 120 python tools/deferred_probe3.py 777 > gpurun_out/r3c/probe3_$v.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r3c/probe3_$v.log | tail -14
  case $rc in 0|1) ;; *) exit $rc;; esac
done
bash tools/gpu_r3_b.sh
