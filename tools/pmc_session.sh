#!/bin/bash
# rocprofv3 PMC passes for the k_step kernel (one counter group per pass, kernel-trace only).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 10 --warmup 3 --cpu-steps 0}"
i=0
for counters in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_WAIT_ANY SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex "k_step" -d gpurun_out/pmc/p$i -o pmc --output-format csv -- python bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 3 gpurun_out/pmc/p$i.log
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
done
