#!/bin/bash
# Round 5: GPU-side cost of the graph -> stream transition (tools/launch_gap_probe.py, GPU-bound part)
set -u
OUT=gpurun_out/r5i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/launch_gap_probe.py balance 32768 > $OUT/probe_c2.log 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/probe_c2.log; exit 1; }
grep probe $OUT/probe_c2.log
