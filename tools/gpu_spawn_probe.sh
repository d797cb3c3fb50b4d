#!/bin/bash
set -u
mkdir -p gpurun_out/sp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sp/prof -o sp -- python tools/spawn_probe.py 16384 > gpurun_out/sp/probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/sp/probe.log | grep "T=" ; exit $rc
