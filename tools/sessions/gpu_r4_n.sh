#!/bin/bash
# Round 4, session n: where C2's host time goes (cProfile, timeline) and k_world's per-wave phases.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 200 python tools/host_profile.py balance 32768 400 > $O/host_profile_c2.log 2>&1 || exit $?
timeout -k 10 200 python tools/step_timeline.py balance 32768 > $O/timeline_c2.log 2>&1 || exit $?
tail -1 $O/timeline_c2.log | cut -c1-400
timeout -k 10 200 python tools/jit_phase_profile.py balance 32768 200 > $O/phase_c2.log 2>&1 || exit $?
tail -25 $O/phase_c2.log
echo done
