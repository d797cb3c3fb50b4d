#!/bin/bash
# Global-pass fixed point (no exit counter): the JIT / graph / parity GPU tests, then the k_world
# probe at C2 (batch and env broadphase) and a short bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_jit.py tests/test_graph.py tests/test_gpu_parity.py > gpurun_out/grid_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/grid_tests.log; exit 1; }
tail -2 gpurun_out/grid_tests.log
timeout -k 10 240 python tools/kworld_probe.py balance 32768 batch > gpurun_out/kp_batch2.log 2>&1 || exit 1
timeout -k 10 240 env VMAS_JIT_PROFILE=0 python tools/kworld_probe.py balance 32768 batch > gpurun_out/kp_batch2_prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/grid_bench.json 2> gpurun_out/grid_bench.err || exit 1
grep -v amdgpu.ids gpurun_out/kp_batch2.log | head -4
tail -1 gpurun_out/grid_bench.json
