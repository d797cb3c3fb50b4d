#!/bin/bash
# Round 5: the band retry (features relaxed), LIDAR conditioning certification (C4), the spawn
# hand-over through the per-target kernels, the k_world workgroup timeline with its claim stamps.
set -u
OUT=gpurun_out/r5e; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -v -m gpu"
timeout -k 10 900 $T "tests/test_features.py::test_features_full_size_gpu" "tests/test_scenario_oracle.py::test_scenario_programs_match_oracle_full_size_gpu" tests/test_spawn.py > $OUT/tests.log 2>&1; echo "tests rc=$?"
grep -E "passed|failed" $OUT/tests.log | tail -2
timeout -k 10 300 python tools/kworld_wg_timeline.py balance 32768 > $OUT/wg_timeline_c2.log 2>&1; echo "timeline rc=$?"
tail -16 $OUT/wg_timeline_c2.log
timeout -k 10 600 python bench.py --scenario discovery --steps 50 --warmup 10 --cpu-steps 0 > $OUT/bench_c4.log 2>&1; echo "c4 rc=$?"
tail -1 $OUT/bench_c4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('respawn_handovers'))"
