#!/bin/bash
# Host path (cached array addresses, random-action plan fast path): the GPU tests, host_micro, and
# three C2 bench runs.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/h3
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/h3/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/h3/tests.log; exit 1; }
tail -1 gpurun_out/h3/tests.log
timeout -k 10 300 python tools/host_micro.py > gpurun_out/h3/host_micro.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/h3/host_micro.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/h3/bench$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']/1e6,1), d['ms_per_step'], d['roofline']['kernel_us_per_launch'], d['roofline']['kernel_us_event'], d['roofline']['pmc_record'])" gpurun_out/h3/bench$r.json
done
