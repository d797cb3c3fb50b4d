#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/raw
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graph.py tests/test_rng.py -m gpu -p no:cacheprovider > gpurun_out/raw/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/raw/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/step_timeline.py balance > gpurun_out/raw/tl_balance.json && cat gpurun_out/raw/tl_balance.json || exit 1
bash tools/ab_raw_launch.sh
