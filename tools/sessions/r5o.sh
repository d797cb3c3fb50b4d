#!/bin/bash
# Round 5: the post-replay launch's span list (C2, C3, C5 shard) -- what k_copy_draw moves per step.
set -u
OUT=gpurun_out/r5o; mkdir -p $OUT
export TMPDIR=/tmp
for sc in balance transport flocking; do
  VMAS_COPY_TRACE=40 timeout -k 10 300 python bench.py --scenario $sc --steps 20 --warmup 10 --cpu-steps 0 > $OUT/trace_$sc.log 2>&1; echo "$sc rc=$?"
  grep -A40 "vmas_copy_spans_draw" $OUT/trace_$sc.log | tail -42 | head -60
done
