#!/bin/bash
set -u
mkdir -p gpurun_out/r3h
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3h/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3h/$name.log | tail -c 300; echo
  case $rc in 0) ;; *) exit $rc;; esac
}
run pytest 600 python -u -m pytest tests/test_spawn.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run probe 300 python tools/spawn_probe.py 16384
run host_flock 300 python tools/host_profile.py flocking 32768
run host_bal 300 python tools/host_profile.py balance 32768
run host_disc 300 python tools/host_profile.py discovery 16384
run pytest_fused 600 python -u -m pytest tests/test_fused.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run stepk_disc 300 python tools/step_kernels.py discovery 16384 8
run stepk_flock 300 python tools/step_kernels.py flocking 32768 8
