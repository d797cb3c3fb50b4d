#!/bin/bash
set -u
mkdir -p gpurun_out/fp
export TMPDIR=/tmp
timeout -k 10 200 python tools/flock_probe.py > gpurun_out/fp/probe.log 2>&1; echo rc=$?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fp/prof -o p --output-format csv -- python tools/flock_probe.py > gpurun_out/fp/prof.log 2>&1; echo rc=$?
rm -f gpurun_out/fp/prof/*kernel_trace.csv
