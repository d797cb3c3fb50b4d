#!/bin/bash
# Round 6: where the host time of the host-bound configs goes (C5 shard, C4, C3): issue time vs GPU
# time per step, the host phases of a graph step, cProfile of the C5 step.
set -u
OUT=${OUT:-gpurun_out/r6e}; mkdir -p $OUT
export TMPDIR=/tmp
step() {
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-900
    case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
}
step gap_c5 300 python tools/launch_gap_probe.py flocking 32768
step gap_c4 300 python tools/launch_gap_probe.py discovery 16384
step gap_c3 300 python tools/launch_gap_probe.py transport 32768
step gap_c2 300 python tools/launch_gap_probe.py balance 32768
step timeline_c5 300 python tools/step_timeline.py flocking 32768
step timeline_c4 300 python tools/step_timeline.py discovery 16384
step hostprof_c5 300 python tools/host_profile.py flocking 32768 300 graph
step hostprof_c4 300 python tools/host_profile.py discovery 16384 300 graph
echo "session done"
