#!/bin/bash
set -u
mkdir -p gpurun_out/r3f2
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3f2/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3f2/$name.log | tail -c 300; echo
  case $rc in 124|134|137|139) exit $rc;; esac
}
run bench_c5 300 python bench.py --scenario flocking --steps 100 --warmup 10 --cpu-steps 0
run pmc1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/r3f2/pmc1 -o p --output-format csv -- python bench.py --scenario flocking --steps 5 --warmup 3 --cpu-steps 0 --event-launches 2
run pmc2 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/r3f2/pmc2 -o p --output-format csv -- python bench.py --scenario flocking --steps 5 --warmup 3 --cpu-steps 0 --event-launches 2
