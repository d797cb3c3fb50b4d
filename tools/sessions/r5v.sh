#!/bin/bash
# Round 5: balance's reward inputs preloaded before the program's barrier -- fused-program parity,
# scenario oracle at full size, C2 bench x3.
set -u
OUT=gpurun_out/r5v; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -v -m gpu"
timeout -k 10 900 $T tests/test_fused.py tests/test_graph.py "tests/test_scenario_oracle.py::test_scenario_programs_match_oracle_full_size_gpu" "tests/test_scenario_oracle.py::test_scenario_programs_match_oracle_eager_gpu" > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/tests.log | tail -8
case $rc in 124|134|137|139) exit $rc;; esac
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  tail -1 $OUT/bench_c2_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'])"
done
