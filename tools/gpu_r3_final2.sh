#!/bin/bash
# Round-3 closing evidence: GPU suite + smoke + C2 bench + rocprofv3 stats, then the C3-C5 bench
# lines with their rocprofv3 stats and the C2 / C4 / C5 step traces.  Stops at a timeout / crash.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
SESSION_STEPS="tests smoke bench prof" bash tools/gpu_session.sh || exit $?
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
TAG=c2 bash tools/step_trace.sh && TAG=c4 ARGS="--scenario discovery" bash tools/step_trace.sh && TAG=c5 ARGS="--scenario flocking" bash tools/step_trace.sh
echo "evidence done"
