#!/bin/bash
# Round-3 session D: discovery after the spawn-word clear moved from a memset node to a kernel --
# the discovery GPU tests, the C4 bench (twice), then the whole GPU suite.  Stops at a timeout / crash.
set -u
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3d/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3d/$name.log | tail -c 700; echo
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run disc_tests 400 python -u -m pytest tests/test_fused.py tests/test_spawn.py tests/test_graph.py -k "discovery or spawn or flocking" -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_c4_1 200 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
run bench_c4_2 200 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
run suite 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_c5 200 python bench.py --scenario flocking --steps 100 --warmup 10 --cpu-steps 0
run clash 120 python tools/clash_probe.py flocking 4096 8
