#!/bin/bash
# Round 3: features full-size probe, k_world with runtime vs folded parameter values (A/B, C2),
# then the GPU test suite.  Stops at the first fatal step.
set -u
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3/$name.log | tail -c 400; echo
  case $rc in 124|134|137|139) exit $rc;; esac
}
run feat_probe 300 python tools/features_probe.py 16384
for i in 1 2 3; do
  run bench_runtime_$i 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0
  run bench_folded_$i 300 env VMAS_JIT_PRM_MASK=0 python bench.py --steps 100 --warmup 10 --cpu-steps 0
done
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
