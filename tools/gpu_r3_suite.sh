#!/bin/bash
# The whole GPU suite without -x (every failure listed), then the discovery fused test alone
# (twice) with the spawn launch's per-item stamps.  Stops at a timeout / crash.
set -u
mkdir -p gpurun_out/r3s
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3s/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3s/$name.log | tail -c 600; echo
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run suite 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
run disc1 200 python -u -m pytest "tests/test_fused.py::test_fused_program_matches_torch_program_gpu[discovery]" -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
VMAS_SPAWN_CLAIMED=1 run disc_claimed 200 python -u -m pytest "tests/test_fused.py::test_fused_program_matches_torch_program_gpu[discovery]" -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
