#!/bin/bash
# Round 5: holonomic agents' state.force left out of the post-replay carry
# (VMAS_GRAPH_FORCE_WRITE_ONLY, default 1) vs carried: graph / actions / fused / scenario-oracle GPU
# tests, the C5 span list, then interleaved A/Bs on C2, C5 shard and C3.
set -u
OUT=gpurun_out/r5aa; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_graph.py tests/test_actions.py tests/test_fused.py tests/test_scenario_oracle.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -B5 -A25 "Error\|FAILED" $OUT/pytest.log | head -80; exit 1; }
VMAS_COPY_TRACE=25 timeout -k 10 300 python bench.py --scenario flocking --cpu-steps 0 --steps 5 --warmup 20 > $OUT/spans_c5.log 2>&1 || { echo "span trace rc=$?"; exit 1; }
grep "spans_draw\] spans" $OUT/spans_c5.log | tail -1
b() {  # b <tag> <env assignment> <bench args...>
  local tag=$1 v=$2; shift 2
  env $v timeout -k 10 300 python bench.py --cpu-steps 0 "$@" > $OUT/bench_$tag.log 2>&1 || { echo "bench $tag rc=$?"; exit 1; }
  tail -1 $OUT/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  for v in 1 0; do
    b c2_fwo${v}_$i VMAS_GRAPH_FORCE_WRITE_ONLY=$v --scenario balance
    b c5_fwo${v}_$i VMAS_GRAPH_FORCE_WRITE_ONLY=$v --scenario flocking
    b c3_fwo${v}_$i VMAS_GRAPH_FORCE_WRITE_ONLY=$v --scenario transport
  done
done
