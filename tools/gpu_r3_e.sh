#!/bin/bash
set -u
mkdir -p gpurun_out/r3e
export TMPDIR=/tmp
echo "=== spawn_probe"; timeout -k 10 120 python tools/spawn_probe.py 16384 > gpurun_out/r3e/spawn_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r3e/spawn_probe.log | tail -30; case $rc in 0|1) ;; *) exit $rc;; esac
TAG=c4 ARGS="--scenario discovery" bash tools/step_trace.sh
