#!/bin/bash
set -u
mkdir -p gpurun_out/sp
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_spawn.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sp/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/sp/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/spawn_probe.py 16384 > gpurun_out/sp/probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/sp/probe.log | tail -30; exit $rc
