#!/bin/bash
set -u
mkdir -p gpurun_out/r3g
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3g/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3g/$name.log | tail -c 1000; echo
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run spawn_c4 200 python tools/spawn_probe_c4.py 16384
run tests 500 python -u -m pytest tests/test_spawn.py tests/test_fused.py tests/test_graph.py -k "discovery or spawn" -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_c4 200 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
run clash_disc 120 python tools/clash_probe.py discovery 4096 8
run stepk_disc 200 python tools/step_kernels.py discovery 16384 8
