#!/bin/bash
# Round 5: the ~8 us idle gap before the post-replay launch -- graph -> stream transition cost vs
# host issue rate (tools/launch_gap_probe.py), the host timeline and cProfile of a C2 graph step.
set -u
OUT=gpurun_out/r5h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/launch_gap_probe.py balance 32768 > $OUT/probe_c2.log 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/probe_c2.log; exit 1; }
cat $OUT/probe_c2.log | grep probe
timeout -k 10 300 python tools/launch_gap_probe.py flocking 32768 > $OUT/probe_c5.log 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/probe_c5.log; exit 1; }
grep '"step"' $OUT/probe_c5.log
timeout -k 10 300 python tools/step_timeline.py balance 32768 > $OUT/timeline_c2.log 2>&1 || { echo "timeline rc=$?"; tail -5 $OUT/timeline_c2.log; exit 1; }
tail -3 $OUT/timeline_c2.log
timeout -k 10 300 python tools/host_profile.py balance 32768 300 graph > $OUT/hostprof_c2.log 2>&1 || { echo "hostprof rc=$?"; exit 1; }
head -45 $OUT/hostprof_c2.log
