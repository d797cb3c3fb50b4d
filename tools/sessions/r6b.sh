#!/bin/bash
# Round 6: the state write-back (no post-replay carry; VMAS_GRAPH_WRITEBACK), the default graph step
# for user scenarios, the forced second pass: the whole -m gpu suite, then an interleaved A/B.
set -u
OUT=gpurun_out/r6b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest_gpu.log | head; exit 1; }
for i in 1 2 3; do
  for v in 1 0; do
    VMAS_GRAPH_WRITEBACK=$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_wb${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c2_wb${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2 wb=$v', d['value'], d['ms_per_step'], r['kernel_us_per_launch'], r.get('kernel_us_timed_region'))"
  done
done
for sc in transport flocking; do
  for v in 1 0; do
    VMAS_GRAPH_WRITEBACK=$v timeout -k 10 300 python bench.py --scenario $sc --cpu-steps 0 > $OUT/bench_${sc}_wb${v}.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_${sc}_wb${v}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$sc wb=$v', d['value'], d['ms_per_step'], r['kernel_us_per_launch'])"
  done
done
echo "session done"
