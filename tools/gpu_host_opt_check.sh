#!/bin/bash
# Graph-mode host path check: graph / rng GPU tests, step timeline, bench (balance, flocking).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/hostopt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph.py tests/test_rng.py -m gpu -p no:cacheprovider > gpurun_out/hostopt/pytest.log 2>&1; rc=$?; tail -16 gpurun_out/hostopt/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/step_timeline.py balance > gpurun_out/hostopt/tl_balance.json && cat gpurun_out/hostopt/tl_balance.json || exit 1
timeout -k 10 120 python tools/step_timeline.py flocking > gpurun_out/hostopt/tl_flocking.json && cat gpurun_out/hostopt/tl_flocking.json || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/hostopt/bench.json 2> gpurun_out/hostopt/bench.log && cat gpurun_out/hostopt/bench.json || exit 1
timeout -k 10 300 python bench.py --scenario flocking --n-agents 8 --substeps 0 --steps 50 --warmup 10 --cpu-steps 0 > gpurun_out/hostopt/c5.json 2>> gpurun_out/hostopt/bench.log && cat gpurun_out/hostopt/c5.json
