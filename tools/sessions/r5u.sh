#!/bin/bash
# Round 5: k_world's LPT costs, second look -- a cheaper box-line part, the finish cost (C2 A/B).
set -u
OUT=gpurun_out/r5u; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in "PART=1.8" "PART=1.2" "FINISH=2.0" "FINISH=4.5"; do
    env VMAS_JIT_COST_$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c2_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 $v', d['value'], d['ms_per_step'], d['roofline']['kernel_us_per_launch'])"
  done
done
