#!/bin/bash
# Round 5: a pre-applied replay's kernel chain launched by the post-replay C++ call
# (VMAS_GRAPH_CHAIN_IN_POST, default 1) vs its own ctypes call (0): the graph tests, then an
# interleaved A/B on the host-bound C3 and the C5 shard, C2 and C4 once each way.
set -u
OUT=gpurun_out/r5x; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_graph.py tests/test_spawn.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_graph.log 2>&1; rc=$?
tail -3 $OUT/pytest_graph.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
for i in 1 2; do
  for v in 1 0; do
    for sc in transport flocking; do
      VMAS_GRAPH_CHAIN_IN_POST=$v timeout -k 10 300 python bench.py --scenario $sc --cpu-steps 0 > $OUT/bench_${sc}_${v}_${i}.log 2>&1 || { echo "bench rc=$?"; exit 1; }
      tail -1 $OUT/bench_${sc}_${v}_${i}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc in_post=$v', d['value'], d['ms_per_step'])"
    done
  done
done
for v in 1 0; do
  for sc in balance discovery; do
    VMAS_GRAPH_CHAIN_IN_POST=$v timeout -k 10 300 python bench.py --scenario $sc --cpu-steps 0 > $OUT/bench_${sc}_${v}.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_${sc}_${v}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc in_post=$v', d['value'], d['ms_per_step'])"
  done
done
