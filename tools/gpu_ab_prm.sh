#!/bin/bash
# A/B on one box: k_world with parameter values as arguments vs folded into the code, per field
# group (VMAS_JIT_PRM_MASK bits: 0 mass, 1 inertia, 2 drag, ..., 11 world), C2 balance.
set -u
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for i in 1 2; do
  for m in ${MASKS:-0xFFF 0x0 0xFFC 0xFFB 0x7FF}; do
    timeout -k 10 300 env VMAS_JIT_PRM_MASK=$m python bench.py --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/ab/m${m}_$i.log 2>&1
    rc=$?; echo "$m $i rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  done
done
