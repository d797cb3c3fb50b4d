#!/bin/bash
set -u
mkdir -p gpurun_out/r3i
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3i/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3i/$name.log | tail -c 500; echo
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run tests 500 python -u -m pytest tests/test_fused.py tests/test_gpu_parity.py tests/test_graph.py -k "discovery" -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_c4_1 200 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
run bench_c4_2 200 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
TAG=c4b ARGS="--scenario discovery" bash tools/step_trace.sh
