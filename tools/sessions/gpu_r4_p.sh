#!/bin/bash
# Round 4, session p: the post-replay C++ call's phases (VMAS_HOST_TIMING) at C2 and C4.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
VMAS_HOST_TIMING=1 timeout -k 10 200 python tools/step_timeline.py balance 32768 > $O/timeline_c2.log 2>&1 || exit $?
grep -E "post_draw|wall" $O/timeline_c2.log | cut -c1-300
VMAS_HOST_TIMING=1 timeout -k 10 200 python tools/step_timeline.py discovery 16384 > $O/timeline_c4.log 2>&1 || exit $?
grep -E "post_draw|wall" $O/timeline_c4.log | cut -c1-300
echo done
