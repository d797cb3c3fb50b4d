#!/bin/bash
# Round 5: balance box queries split over four waves in the program / k_world epilogue; same
# parity set and interleaved A/B as r5k.sh
set -u
OUT=gpurun_out/r5l; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -v -m gpu"
timeout -k 10 900 $T tests/test_fused.py tests/test_graph.py "tests/test_scenario_oracle.py::test_scenario_programs_match_oracle_full_size_gpu" "tests/test_scenario_oracle.py::test_scenario_programs_match_oracle_eager_gpu" > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/tests.log | tail -14
case $rc in 124|134|137|139) exit $rc;; esac
for i in 1 2; do
  for v in 1 0; do
    VMAS_GRAPH_FUSE=$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_fuse${v}_$i.log 2>&1 || { echo "bench rc=$?"; tail -3 $OUT/bench_c2_fuse${v}_$i.log; exit 1; }
    tail -1 $OUT/bench_c2_fuse${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 fuse=$v', d['value'], d['ms_per_step'], d['config'].get('step_mode'))"
  done
done
for v in 1 0; do
  VMAS_GRAPH_FUSE=$v timeout -k 10 300 python bench.py --scenario transport --cpu-steps 0 > $OUT/bench_c3_fuse$v.log 2>&1 || { echo "bench rc=$?"; tail -3 $OUT/bench_c3_fuse$v.log; exit 1; }
  tail -1 $OUT/bench_c3_fuse$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 fuse=$v', d['value'], d['ms_per_step'], d['config'].get('step_mode'))"
done
timeout -k 10 300 python tools/launch_gap_probe.py balance 32768 > $OUT/probe_c2.log 2>&1 && grep '"step"' $OUT/probe_c2.log
TAG=r5l_c2 bash tools/step_trace.sh > /dev/null 2>&1; cp gpurun_out/steptrace/r5l_c2/summary.txt $OUT/step_trace_c2.txt; tail -8 $OUT/step_trace_c2.txt
