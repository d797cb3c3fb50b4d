#!/bin/bash
# Round 5: the features world's relaxed-math parity with the branch-free trig reduction and with
# round 4's guard (VMAS_JIT_TRIG=guard), plus the tests fixed after the auto graph step.
set -u
OUT=gpurun_out/r5d; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -v -m gpu"
timeout -k 10 600 $T "tests/test_features.py::test_features_full_size_gpu" > $OUT/features_reduce.log 2>&1; echo "reduce rc=$?"
VMAS_JIT_TRIG=guard timeout -k 10 600 $T "tests/test_features.py::test_features_full_size_gpu" > $OUT/features_guard.log 2>&1; echo "guard rc=$?"
timeout -k 10 900 $T tests/test_scenario_oracle.py tests/test_actions.py "tests/test_graph.py::test_graph_kernel_timing_gpu" "tests/test_graph.py::test_draw_ahead_dropped_by_caller_actions_gpu" "tests/test_graph.py::test_preapplied_random_actions_match_eager_gpu" > $OUT/tests.log 2>&1; echo "tests rc=$?"
grep -h "PARITY" $OUT/*.log | cut -c1-400
timeout -k 10 300 python tools/kworld_wg_timeline.py balance 32768 > $OUT/wg_timeline_c2.log 2>&1; echo "timeline rc=$?"
cat $OUT/wg_timeline_c2.log | tail -20
timeout -k 10 600 python bench.py --scenario discovery --steps 50 --warmup 10 --cpu-steps 0 > $OUT/bench_c4.log 2>&1; echo "c4 rc=$?"
tail -1 $OUT/bench_c4.log | cut -c1-300
