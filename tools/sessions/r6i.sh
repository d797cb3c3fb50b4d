#!/bin/bash
# Round 6: the tail with one word per thread (wide virtual blocks) and transport's write-through
# outputs: graph / fused / JIT / scenario-oracle GPU tests, C2 A/B, C3, a kernel trace of C2.
set -u
OUT=${OUT:-gpurun_out/r6i}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_graph.py tests/test_fused.py tests/test_jit.py tests/test_scenario_oracle.py -m gpu --maxfail=3 -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest.log | head; exit 1; }
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', round(d['value']/1e6,1), d['ms_per_step'], r['kernel_us_per_launch'], r.get('kernel_us_timed_region'))"; }
for i in 1 2; do
  for v in 1 0; do
    VMAS_GRAPH_TAIL=$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_tail${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    summ $OUT/bench_c2_tail${v}_$i.log "c2 tail=$v"
    VMAS_GRAPH_TAIL=$v timeout -k 10 300 python bench.py --scenario transport --cpu-steps 0 > $OUT/bench_c3_tail${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    summ $OUT/bench_c3_tail${v}_$i.log "c3 tail=$v"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --cpu-steps 0 --steps 40 > $OUT/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo "session done"
