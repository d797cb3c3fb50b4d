#!/bin/bash
# Round 6: balance's epilogue reading the group's state from k_world's LDS rows (VMAS_JIT_EPI_SRC):
# the fused-program / graph / JIT / scenario-oracle tests, then an interleaved C2 A/B.
set -u
OUT=gpurun_out/r6d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_fused.py tests/test_graph.py tests/test_jit.py tests/test_scenario_oracle.py -m gpu --maxfail=3 -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest.log | head; exit 1; }
for i in 1 2 3; do
  for v in 1 0; do
    VMAS_JIT_EPI_SRC=$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_src${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c2_src${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2 src=$v', d['value'], d['ms_per_step'], r['kernel_us_per_launch'], (r.get('plain') or {}).get('kernel_us'))"
  done
done
echo "session done"
