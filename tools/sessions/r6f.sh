#!/bin/bash
# Round 6: the state write-back at C5 full (262 144 envs) and C3, interleaved A/B (VMAS_GRAPH_WRITEBACK).
set -u
OUT=${OUT:-gpurun_out/r6f}; mkdir -p $OUT
export TMPDIR=/tmp
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', round(d['value']/1e6,1), d['ms_per_step'], r['kernel_us_per_launch'], r.get('kernel_us_timed_region'))"; }
for i in 1 2; do
  for v in 0 1; do
    VMAS_GRAPH_WRITEBACK=$v timeout -k 10 300 python bench.py --scenario flocking --envs 262144 --steps 30 --warmup 10 --cpu-steps 0 > $OUT/c5full_wb${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    summ $OUT/c5full_wb${v}_$i.log "c5full wb=$v"
    VMAS_GRAPH_WRITEBACK=$v timeout -k 10 300 python bench.py --scenario transport --cpu-steps 0 > $OUT/c3_wb${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    summ $OUT/c3_wb${v}_$i.log "c3 wb=$v"
    VMAS_GRAPH_WRITEBACK=$v timeout -k 10 300 python bench.py --scenario flocking --cpu-steps 0 > $OUT/c5_wb${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    summ $OUT/c5_wb${v}_$i.log "c5 wb=$v"
  done
done
echo "ab done"
OUT=gpurun_out/r6e bash tools/sessions/r6e.sh
