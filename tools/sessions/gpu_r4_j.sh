#!/bin/bash
# Round 4, session j: adaptive spawn window + draw-ahead with discovery's in-graph respawn -- graph
# tests, spawn tests, C4 A/B (window knob), probe.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_graph.py tests/test_spawn.py tests/test_copy_spans.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest.log | tail -6
case $rc in 0|1) ;; *) exit $rc;; esac
for i in 1 2; do
  timeout -k 10 200 python bench.py --scenario discovery --cpu-steps 0 --steps 200 > $O/c4_$i.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('$O/c4_$i.log').read().strip().splitlines()[-1]); print('C4 run $i', round(d['value']/1e6,1), d['ms_per_step'], d['config'].get('respawn_handovers'))"
done
TAG=c4 ARGS="--scenario discovery" bash tools/step_trace.sh > $O/step_trace_c4.txt 2>&1 || exit $?
tail -11 $O/step_trace_c4.txt
echo done
