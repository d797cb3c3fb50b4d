#!/bin/bash
set -u
mkdir -p gpurun_out/r3d6
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3d6/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3d6/$name.log | tail -c 400; echo
  case $rc in 0) ;; *) exit $rc;; esac
}
run pytest 900 python -u -m pytest tests/test_graph.py tests/test_spawn.py tests/test_fused.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run stepk_disc 300 python tools/step_kernels.py discovery 16384 8
run host_disc 300 python tools/host_profile.py discovery 16384
run bench_c4 300 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
run stepk_bal 300 python tools/step_kernels.py balance 32768 4
