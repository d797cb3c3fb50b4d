#!/bin/bash
# Round 6: the post-replay work as the tail of balance's one fused k_world launch (csrc/vmas_tail.hpp,
# VMAS_GRAPH_TAIL): graph / fused / JIT GPU tests, an interleaved C2 A/B, a kernel trace of the tail.
set -u
OUT=${OUT:-gpurun_out/r6h}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_graph.py tests/test_fused.py tests/test_jit.py -m gpu --maxfail=3 -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest.log | head; exit 1; }
for i in 1 2 3; do
  for v in 1 0; do
    VMAS_GRAPH_TAIL=$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_tail${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c2_tail${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2 tail=$v', round(d['value']/1e6,1), d['ms_per_step'], r['kernel_us_per_launch'], (r.get('plain') or {}).get('kernel_us'))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --cpu-steps 0 --steps 40 > $OUT/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo "session done"
