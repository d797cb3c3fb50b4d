#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/rng
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rng.py tests/test_graph.py -m gpu -p no:cacheprovider > gpurun_out/rng/pytest.log 2>&1; rc=$?; tail -22 gpurun_out/rng/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/step_timeline.py balance > gpurun_out/rng/tl_balance.json && cat gpurun_out/rng/tl_balance.json || exit 1
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-steps 0 > gpurun_out/rng/bench_$rep.json 2> gpurun_out/rng/bench.log && python -c "import json; d=json.load(open('gpurun_out/rng/bench_$rep.json')); print('balance', round(d['value']/1e6,1), d['ms_per_step'])" || exit 1
done
timeout -k 10 300 python bench.py --scenario flocking --n-agents 8 --substeps 0 --steps 50 --warmup 10 --cpu-steps 0 > gpurun_out/rng/c5.json 2>> gpurun_out/rng/bench.log && python -c "import json; d=json.load(open('gpurun_out/rng/c5.json')); print('flocking', round(d['value']/1e6,1), d['ms_per_step'])"
