#!/bin/bash
# Round 5: k_world's LPT cost of a box-line part (VMAS_JIT_COST_PART) -- interleaved C2 A/B.
set -u
OUT=gpurun_out/r5t; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in 1.8 2.6 3.4; do
    VMAS_JIT_COST_PART=$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_part${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c2_part${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 part=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_us_per_launch'])"
  done
done
