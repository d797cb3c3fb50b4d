#!/bin/bash
set -u
mkdir -p gpurun_out/r3h
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3h/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3h/$name.log | tail -c 600; echo
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run tests 500 python -u -m pytest tests/test_copy_spans.py tests/test_graph.py tests/test_fused.py tests/test_spawn.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_c4 200 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
run bench_c5 200 python bench.py --scenario flocking --steps 100 --warmup 10 --cpu-steps 0
run bench_c2 200 python bench.py --steps 100 --warmup 10 --cpu-steps 0
