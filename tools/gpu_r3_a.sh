#!/bin/bash
# Round-3 session A: the spawn-channel corruption probe, the graph / fused GPU tests, the C2 bench,
# the C2 step trace and the host micro-profile.  Stops at a timeout / crash.
set -u
mkdir -p gpurun_out/r3a
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3a/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3a/$name.log | tail -c 1500; echo
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run probe2 120 python tools/deferred_probe2.py 777
run tests 600 python -u -m pytest tests/test_graph.py tests/test_fused.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_c2 200 python bench.py --steps 100 --warmup 10 --cpu-steps 0
run host_micro 200 python tools/host_micro.py balance 32768
TAG=c2 bash tools/step_trace.sh
