#!/bin/bash
set -u
mkdir -p gpurun_out/r3d2
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $to "$@" > gpurun_out/r3d2/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/r3d2/$name.log | tail -c 300; echo
  case $rc in 0) ;; *) exit $rc;; esac
}
run pytest_spawn 600 python -u -m pytest tests/test_spawn.py tests/test_fused.py -k "spawn or respawn or discovery" -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_c4 300 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0
run stepk_disc 300 python tools/step_kernels.py discovery 16384 8
run pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM -d gpurun_out/r3d2/pmc_sq -o pmc -- python bench.py --scenario discovery --steps 10 --warmup 3 --cpu-steps 0
run pmc_tcc 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d gpurun_out/r3d2/pmc_tcc -o pmc -- python bench.py --scenario discovery --steps 10 --warmup 3 --cpu-steps 0
