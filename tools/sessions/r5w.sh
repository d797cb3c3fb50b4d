#!/bin/bash
# Round 5: k_world code-generation knobs re-checked after this round's changes (loop per wave,
# epilogue): issue priority by substep, pair / entity preloads -- interleaved C2 A/B.
set -u
OUT=gpurun_out/r5w; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in "DEFAULT=1" "VMAS_JIT_PRIO=0" "VMAS_JIT_PAIR_PRELOAD=0" "VMAS_JIT_PRELOAD=0"; do
    env $v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c2_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 $v', d['value'], d['ms_per_step'], d['roofline']['kernel_us_per_launch'])"
  done
done
# the windowed respawn's phases at C4 (tools/spawn_phase_probe.py)
timeout -k 10 300 python -u tools/spawn_phase_probe.py > $OUT/spawn_phases_c4.txt 2>&1 || { echo "probe rc=$?"; tail -20 $OUT/spawn_phases_c4.txt; exit 1; }
cat $OUT/spawn_phases_c4.txt
