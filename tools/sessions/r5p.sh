#!/bin/bash
# Round 5: host issue time vs GPU time per step for C3 / C5 shard / C4 (is the step host-bound?)
set -u
OUT=gpurun_out/r5p; mkdir -p $OUT
export TMPDIR=/tmp
for sc in transport flocking discovery; do
  n=32768; [ $sc = discovery ] && n=16384
  timeout -k 10 300 python tools/launch_gap_probe.py $sc $n > $OUT/probe_$sc.log 2>&1; echo "$sc rc=$?"; grep '"step"' $OUT/probe_$sc.log
done
timeout -k 10 300 python tools/host_profile.py transport 32768 300 graph > $OUT/hostprof_c3.log 2>&1; echo "hostprof rc=$?"
