#!/bin/bash
# Host-path changes: graph / fused / action GPU tests, then the step timeline and a host profile.
set -u
mkdir -p gpurun_out/host
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_graph.py tests/test_fused.py tests/test_actions.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/host/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/host/tests.log; exit 1; }
tail -2 gpurun_out/host/tests.log
timeout -k 10 300 python tools/step_timeline.py balance 32768 > gpurun_out/host/timeline.log 2>&1 || exit 1
tail -1 gpurun_out/host/timeline.log
timeout -k 10 300 python tools/host_profile.py balance 32768 > gpurun_out/host/hostprof.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/host/bench.json 2> gpurun_out/host/bench.log || exit 1
python -c "import json; d=json.load(open('gpurun_out/host/bench.json')); r=d['roofline']; print(r['kernel_us_per_launch'], r.get('kernel_us_event'), round(d['value']/1e6,1), d['ms_per_step'])"
