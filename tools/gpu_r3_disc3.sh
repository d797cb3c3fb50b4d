#!/bin/bash
set -u
mkdir -p gpurun_out/r3d3
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3d3/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3d3/$name.log | tail -c 300; echo
  case $rc in 0) ;; *) exit $rc;; esac
}
run pytest_spawn 600 python -u -m pytest tests/test_spawn.py -k "respawn" -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run stepk_disc 300 python tools/step_kernels.py discovery 16384 8
run bench_c4 300 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
