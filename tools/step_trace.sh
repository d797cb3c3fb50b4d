#!/bin/bash
# rocprofv3 kernel trace of a bench config: every dispatch of the last 3 steps (the stretch from
# one k_world start to the next), with its duration and the gap before it, plus the per-step GPU
# busy time and the wall period.  TAG names the output (gpurun_out/steptrace/<TAG>), ARGS = bench args.
set -u
export TMPDIR=/tmp
TAG=${TAG:-c2}
ARGS=${ARGS:-}
OUT=gpurun_out/steptrace/$TAG
mkdir -p $OUT
rm -rf /tmp/st_$TAG
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/st_$TAG -o st --output-format csv -- python bench.py --steps 30 --warmup 10 --cpu-steps 0 $ARGS > $OUT/run.log 2>&1 || { echo "rc=$?"; exit 1; }
f=$(find /tmp/st_$TAG -name "*kernel_trace.csv" | head -1)
python tools/step_trace.py "$f" > $OUT/summary.txt
cat $OUT/summary.txt
