#!/bin/bash
set -u
mkdir -p gpurun_out/r3pre
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3pre/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3pre/$name.log | tail -c 300; echo
  case $rc in 124|134|137|139) exit $rc;; esac
}
run pytest_graph 600 python -u -m pytest tests/test_graph.py tests/test_rng.py tests/test_actions.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2; do run bench_$i 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0; done
run stepk 300 python tools/step_kernels.py balance 32768 4
run stepk_flock 300 python tools/step_kernels.py flocking 32768 8
run stepk_disc 300 python tools/step_kernels.py discovery 16384 8
