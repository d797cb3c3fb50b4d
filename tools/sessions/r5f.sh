#!/bin/bash
# Round 5: the expanded LIDAR angles (A/B, interleaved), step traces of C4 / C5 shard.
set -u
OUT=gpurun_out/r5f; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in 1 0; do
    for sc in flocking discovery; do
      VMAS_LIDAR_EXPAND=$v timeout -k 10 300 python bench.py --scenario $sc --steps 100 --warmup 10 --cpu-steps 0 > $OUT/bench_${sc}_exp${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
      tail -1 $OUT/bench_${sc}_exp${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc expand=$v', d['value'], d['ms_per_step'])"
    done
  done
done
TAG=r5f_c5 ARGS="--scenario flocking" bash tools/step_trace.sh > /dev/null 2>&1; cp gpurun_out/steptrace/r5f_c5/summary.txt $OUT/step_trace_c5shard.txt; tail -12 $OUT/step_trace_c5shard.txt
TAG=r5f_c4 ARGS="--scenario discovery" bash tools/step_trace.sh > /dev/null 2>&1; cp gpurun_out/steptrace/r5f_c4/summary.txt $OUT/step_trace_c4.txt; tail -14 $OUT/step_trace_c4.txt
TAG=r5f_c2 bash tools/step_trace.sh > /dev/null 2>&1; cp gpurun_out/steptrace/r5f_c2/summary.txt $OUT/step_trace_c2.txt; tail -8 $OUT/step_trace_c2.txt
