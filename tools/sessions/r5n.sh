#!/bin/bash
# Round 5: where k_world's time goes after the loop-per-wave change -- per-wave phase stamps of one
# workgroup (two different workgroups) and the per-workgroup timeline of a launch (C2).
set -u
OUT=gpurun_out/r5n; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/jit_phase_profile.py balance 32768 200 > $OUT/phase_b200.log 2>&1; echo "phase rc=$?"; tail -16 $OUT/phase_b200.log
timeout -k 10 300 python tools/jit_phase_profile.py balance 32768 17 > $OUT/phase_b17.log 2>&1; echo "phase rc=$?"; tail -16 $OUT/phase_b17.log
timeout -k 10 300 python tools/kworld_wg_timeline.py balance 32768 > $OUT/wg_timeline.log 2>&1; echo "timeline rc=$?"; tail -25 $OUT/wg_timeline.log
