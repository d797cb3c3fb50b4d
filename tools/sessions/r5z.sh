#!/bin/bash
# Round 5: balance program -- the package and floor positions preloaded by wave 0 before the
# program's barrier (VMAS_BAL_PRELOAD_POS, default 1) vs loaded after it: fused-program / graph /
# scenario-oracle GPU tests, then an interleaved C2 A/B.
set -u
OUT=gpurun_out/r5z; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_fused.py tests/test_graph.py tests/test_scenario_oracle.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
for i in 1 2 3; do
  for v in 1 0; do
    VMAS_JIT_CFLAGS=-DVMAS_BAL_PRELOAD_POS=$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_pre${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c2_pre${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 preload_pos=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_us_per_launch'])"
  done
done
