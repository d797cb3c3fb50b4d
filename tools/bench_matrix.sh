#!/bin/bash
# Bench lines + rocprofv3 kernel stats for the SURVEY §8(d) configs (C2-C5) on one GPU.
# Stops at the first timeout / crash.  Output: gpurun_out/matrix/<name>.{json,log}, prof_<name>/
set -u
export TMPDIR=/tmp
OUT=gpurun_out/matrix
mkdir -p $OUT
STEPS=${STEPS:-50}
run() {  # run <name> <bench args...>
  local name=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -k 10 300 python bench.py --steps $STEPS --warmup 10 --cpu-steps 0 "$@" > $OUT/$name.json 2> $OUT/$name.log
  local rc=$?; echo "rc=$rc"; tail -c 600 $OUT/$name.json
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --cpu-steps 0 "$@" > $OUT/prof_$name.log 2>&1
  rc=$?; echo "prof rc=$rc"; rm -f $OUT/prof_$name/*_kernel_trace.csv
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
}
run c2_balance_sub10
run c2_balance_sub1 --substeps 1
run c2_balance_sub10_envbp --broadphase env
run c3_transport --scenario transport
run c4_discovery --scenario discovery
run c5_flocking --scenario flocking
echo done
