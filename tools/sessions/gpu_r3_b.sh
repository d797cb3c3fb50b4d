#!/bin/bash
# Round-3 session B: C5 flocking -- which call issues each dispatch (torch profiler), a PMC pass of
# k_flocking_fast, the C4 / C5 bench lines and the C4 step trace.  Stops at a timeout / crash.
set -u
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3b/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3b/$name.log | tail -c 1500; echo
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run stepk_flock 300 python tools/step_kernels.py flocking 32768 8
run bench_c5 200 python bench.py --scenario flocking --steps 100 --warmup 10 --cpu-steps 0
run bench_c4 200 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
run pmc_flock 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "k_flocking_fast" -d gpurun_out/r3b/pmc_flock -o p --output-format csv -- python bench.py --scenario flocking --steps 5 --warmup 3 --cpu-steps 0
TAG=c4 ARGS="--scenario discovery" bash tools/step_trace.sh
