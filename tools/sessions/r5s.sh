#!/bin/bash
# Round 5: where C3's host time goes after the signature caching -- post_draw's C++ phases,
# the per-phase host timeline and a cProfile of the graph step.
set -u
OUT=gpurun_out/r5s; mkdir -p $OUT
export TMPDIR=/tmp
VMAS_HOST_TIMING=1 timeout -k 10 300 python bench.py --scenario transport --cpu-steps 0 > $OUT/bench_c3_timing.log 2>&1; echo "bench rc=$?"; grep "post_draw\]" $OUT/bench_c3_timing.log
timeout -k 10 300 python tools/step_timeline.py transport 32768 > $OUT/timeline_c3.log 2>&1; echo "timeline rc=$?"; tail -2 $OUT/timeline_c3.log
timeout -k 10 300 python tools/host_profile.py transport 32768 300 graph > $OUT/hostprof_c3.log 2>&1; echo "hostprof rc=$?"
