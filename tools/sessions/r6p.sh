#!/bin/bash
# Round 6: host issue vs GPU time per step at C3 after the tail (transport is host-bound?), the
# host profile of the same replay path, and C2 for reference.
set -u
OUT=${OUT:-gpurun_out/r6p}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/launch_gap_probe.py transport 32768 > $OUT/gap_c3.log 2>&1 || { echo "rc=$?"; exit 1; }
tail -1 $OUT/gap_c3.log | cut -c1-300
timeout -k 10 300 python tools/launch_gap_probe.py balance 32768 > $OUT/gap_c2.log 2>&1 || { echo "rc=$?"; exit 1; }
tail -1 $OUT/gap_c2.log | cut -c1-300
timeout -k 10 300 python tools/host_profile.py transport 32768 300 graph > $OUT/hostprof_c3.log 2>&1 || { echo "rc=$?"; exit 1; }
echo "session done"
