#!/bin/bash
# Round 6: the state write-back (no post-replay carry; VMAS_GRAPH_WRITEBACK), the speculative first
# claim (VMAS_JIT_SPEC_CLAIM), the default graph step for user scenarios, the forced second pass,
# the exact-LIDAR / fast-trig parity: the whole -m gpu suite, then an interleaved A/B.
set -u
OUT=gpurun_out/r6b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu --maxfail=4 -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest_gpu.log | head; exit 1; }
grep -E "^FASTTRIG" $OUT/pytest_gpu.log | head -2
for i in 1 2 3; do
  for v in "1 1" "0 1" "1 0"; do
    set -- $v
    VMAS_GRAPH_WRITEBACK=$1 VMAS_JIT_SPEC_CLAIM=$2 timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_wb$1_sc$2_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c2_wb$1_sc$2_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2 wb=$1 spec=$2', d['value'], d['ms_per_step'], r['kernel_us_per_launch'], (r.get('plain') or {}).get('kernel_us'), r.get('kernel_us_timed_region'))"
  done
done
for sc in transport flocking; do
  for v in 1 0; do
    VMAS_GRAPH_WRITEBACK=$v timeout -k 10 300 python bench.py --scenario $sc --cpu-steps 0 > $OUT/bench_${sc}_wb${v}.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_${sc}_wb${v}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$sc wb=$v', d['value'], d['ms_per_step'], r['kernel_us_per_launch'])"
  done
done
echo "session done"
