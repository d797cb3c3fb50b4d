#!/bin/bash
# Round 4, session s: dispatch traces and host timelines of the final tree (C4, C5 shard).
set -u
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
TAG=c4 ARGS="--scenario discovery" bash tools/step_trace.sh > $O/step_trace_c4.txt 2>&1 || exit $?
tail -9 $O/step_trace_c4.txt
TAG=c5 ARGS="--scenario flocking" bash tools/step_trace.sh > $O/step_trace_c5shard.txt 2>&1 || exit $?
tail -9 $O/step_trace_c5shard.txt
timeout -k 10 200 python tools/step_timeline.py flocking 32768 > $O/timeline_c5shard.log 2>&1 || exit $?
tail -1 $O/timeline_c5shard.log | cut -c1-330
timeout -k 10 200 python tools/step_timeline.py discovery 16384 > $O/timeline_c4.log 2>&1 || exit $?
tail -1 $O/timeline_c4.log | cut -c1-330
echo done
