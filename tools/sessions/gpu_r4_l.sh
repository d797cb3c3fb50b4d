#!/bin/bash
# Round 4, session l: write-only attributes not carried between replays (A/B), packed copy grid --
# graph / fused / sensor GPU tests, C2 / C3 / C4 / C5-shard A/B, the C4 span list and step trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_graph.py tests/test_fused.py tests/test_spawn.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest.log | tail -8
case $rc in 0|1) ;; *) exit $rc;; esac
for wo in 0 1 0 1; do
  for sc in discovery transport; do
    VMAS_GRAPH_WRITE_ONLY=$wo timeout -k 10 200 python bench.py --scenario $sc --cpu-steps 0 --steps 200 > $O/ab_wo_${sc}_$wo.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('$O/ab_wo_${sc}_$wo.log').read().strip().splitlines()[-1]); print('$sc wo=$wo', round(d['value']/1e6,1), d['ms_per_step'])"
  done
done
VMAS_COPY_TRACE=1 timeout -k 10 150 python bench.py --scenario discovery --cpu-steps 0 --steps 20 > $O/copytrace_discovery.out 2> $O/copytrace_discovery.log || exit $?
head -3 $O/copytrace_discovery.log
TAG=c4 ARGS="--scenario discovery" bash tools/step_trace.sh > $O/step_trace_c4.txt 2>&1 || exit $?
tail -9 $O/step_trace_c4.txt
timeout -k 10 200 python tools/step_timeline.py discovery 16384 > $O/timeline_c4.log 2>&1 || exit $?
tail -1 $O/timeline_c4.log
echo done
