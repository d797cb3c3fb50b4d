#!/bin/bash
# Round 5: flocking's agent.dist_rew declared write-only (not carried between replays): graph /
# scenario-oracle GPU tests, the post-replay table, C5 shard benches.
set -u
OUT=gpurun_out/r5ab; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_graph.py tests/test_scenario_oracle.py tests/test_fused.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -B5 -A25 "Error\|FAILED" $OUT/pytest.log | head -80; exit 1; }
timeout -k 10 300 python tools/post_table_probe.py flocking > $OUT/post_table_c5.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
grep "bytes:" $OUT/post_table_c5.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --scenario flocking --cpu-steps 0 > $OUT/bench_c5_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  tail -1 $OUT/bench_c5_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['ms_per_step'])"
done
