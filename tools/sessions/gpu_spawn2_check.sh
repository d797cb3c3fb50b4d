#!/bin/bash
# Native target respawn: spawn + fused/graph discovery GPU tests, then the C4 bench line.
set -u
mkdir -p gpurun_out/spawn2
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_spawn.py tests/test_fused.py tests/test_graph.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/spawn2/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/spawn2/tests.log; exit 1; }
tail -2 gpurun_out/spawn2/tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-steps 0 --scenario discovery --envs 16384 --n-agents 8 --substeps 0 --kw '{"use_agent_lidar": true}' > gpurun_out/spawn2/c4.json 2> gpurun_out/spawn2/c4.log || exit 1
python -c "import json; d=json.load(open('gpurun_out/spawn2/c4.json')); print(round(d['value']/1e6,2), d['ms_per_step'], d.get('step_mode'))"
TAG=c4 ARGS="--scenario discovery --envs 16384 --n-agents 8 --substeps 0 --kw {\"use_agent_lidar\":true}" bash tools/prof_c2.sh > gpurun_out/spawn2/prof_c4.txt 2>&1 || exit 1
head -8 gpurun_out/spawn2/prof_c4.txt
