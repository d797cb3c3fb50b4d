#!/bin/bash
# Claim-protocol change: the fixed-point GPU tests, then the k_world probe (per-workgroup records)
# and a C2 bench line.
set -u
mkdir -p gpurun_out/claim
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_jit.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/claim/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/claim/tests.log; exit 1; }
tail -2 gpurun_out/claim/tests.log
VMAS_JIT_PROFILE=200 timeout -k 10 200 python tools/kworld_probe.py balance 32768 > gpurun_out/claim/probe.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 60 --warmup 10 --cpu-steps 0 > gpurun_out/claim/bench.json 2> gpurun_out/claim/bench.log || exit 1
python -c "import json; d=json.load(open('gpurun_out/claim/bench.json')); r=d['roofline']; print(r['kernel_us_per_launch'], r.get('kernel_us_event'), round(d['value']/1e6,1))"
