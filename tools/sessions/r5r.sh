#!/bin/bash
# Round 5: the host path's structure checks cached against core.STATIC_VERSION -- graph tests
# (recapture on parameter changes), C3 (host-bound) / C2 bench, C3 host issue vs GPU time.
set -u
OUT=gpurun_out/r5r; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -v -m gpu"
timeout -k 10 900 $T tests/test_graph.py tests/test_fused.py tests/test_actions.py > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/tests.log | tail -8
case $rc in 124|134|137|139) exit $rc;; esac
for i in 1 2; do
  for sc in transport balance flocking; do
    timeout -k 10 300 python bench.py --scenario $sc --cpu-steps 0 > $OUT/bench_${sc}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_${sc}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 python tools/launch_gap_probe.py transport 32768 > $OUT/probe_c3.log 2>&1 && grep '"step"' $OUT/probe_c3.log
