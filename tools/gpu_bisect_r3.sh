#!/bin/bash
# Round 3 bisects: relaxed-math NaNs in the features world at 16 384 envs under runtime parameter
# values (VMAS_JIT_PRM_MASK: bit k = entity value field k an argument, bit 11 = world values), and
# the k_world cost of runtime values / the force export at C2.  Stops at the first fatal step.
set -u
mkdir -p gpurun_out/bisect
export TMPDIR=/tmp
run() {
  local name=$1; shift
  echo "=== $name"
  timeout -k 10 300 "$@" > gpurun_out/bisect/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/bisect/$name.log | tail -c 600
  case $rc in 124|134|137|139) exit $rc;; esac
}
for m in ${MASKS:-0xFFF 0x0 0x800 0x7FF 0x001 0x002 0x004}; do
  run feat_$m env VMAS_JIT_PRM_MASK=$m python tools/features_probe.py 16384
done
for i in 1 2; do
  run bench_runtime_$i python bench.py --steps 100 --warmup 10 --cpu-steps 0
  run bench_baked_$i env VMAS_JIT_PRM_MASK=0 python bench.py --steps 100 --warmup 10 --cpu-steps 0
done
