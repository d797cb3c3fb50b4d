#!/bin/bash
# Round-3 evidence on one box: the GPU suite + smoke + C2 bench + rocprofv3 stats (gpu_session.sh),
# the PMC passes of k_world (-> tools/pmc_traffic.py record), then the C3-C5 bench lines with their
# rocprofv3 stats.  Stops at the first timeout / crash.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
SESSION_STEPS="tests smoke bench prof" bash tools/gpu_session.sh || exit $?
PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH" TAG=final bash tools/pmc_session.sh || exit $?
OUT=gpurun_out/matrix
mkdir -p $OUT
for cfg in "c3_transport --scenario transport" "c4_discovery --scenario discovery" "c5_flocking --scenario flocking"; do
  set -- $cfg; name=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0 "$@" > $OUT/$name.json 2> $OUT/$name.log
  rc=$?; echo "rc=$rc"; tail -c 300 $OUT/$name.json
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --cpu-steps 0 "$@" > $OUT/prof_$name.log 2>&1
  rc=$?; echo "prof rc=$rc"; rm -f $OUT/prof_$name/*_kernel_trace.csv
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
done
echo "evidence done"
