#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/disc
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_spawn.py tests/test_rng.py tests/test_graph.py tests/test_scenarios_behaviour.py tests/test_gpu_parity.py -m gpu -p no:cacheprovider > gpurun_out/disc/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/disc/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --scenario discovery --envs 16384 --n-agents 8 --substeps 0 --kw '{"use_agent_lidar": true}' --steps 50 --warmup 10 --cpu-steps 0 > gpurun_out/disc/c4.json 2> gpurun_out/disc/c4.log && python -c "import json; d=json.load(open('gpurun_out/disc/c4.json')); print('discovery', round(d['value']/1e6,2), d['ms_per_step'], d['config']['step_mode'])" || exit 1
timeout -k 10 300 python tools/step_breakdown.py discovery 16384 8 > gpurun_out/disc/breakdown.log 2>&1; head -2 gpurun_out/disc/breakdown.log
