#!/bin/bash
set -u
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3d/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3d/$name.log | tail -c 300; echo
  case $rc in 124|134|137|139) exit $rc;; esac
}
run pytest_fused 600 python -u -m pytest tests/test_fused.py tests/test_scenarios_behaviour.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_c4 300 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
run stepk_disc 300 python tools/step_kernels.py discovery 16384 8
