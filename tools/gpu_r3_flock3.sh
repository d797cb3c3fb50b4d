#!/bin/bash
# k_flocking variants: exact (VMAS_FUSED_EXACT_LIDAR=1) vs fast; PMC of the fast kernel.
set -u
mkdir -p gpurun_out/r3f3
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3f3/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep "/step" gpurun_out/r3f3/$name.log | head -3
  case $rc in 124|134|137|139) exit $rc;; esac
}
#run stepk_exact 300 env VMAS_FUSED_EXACT_LIDAR=1 python tools/step_kernels.py flocking 32768 8
run stepk_fast 300 python tools/step_kernels.py flocking 32768 8
run pmc1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/r3f3/pmc1 -o p --output-format csv -- python bench.py --scenario flocking --steps 5 --warmup 3 --cpu-steps 0 --event-launches 2
run pmc2 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r3f3/pmc2 -o p --output-format csv -- python bench.py --scenario flocking --steps 5 --warmup 3 --cpu-steps 0 --event-launches 2
run pmc3 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r3f3/pmc3 -o p --output-format csv -- python bench.py --scenario flocking --steps 5 --warmup 3 --cpu-steps 0 --event-launches 2
