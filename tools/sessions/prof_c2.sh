#!/bin/bash
# rocprofv3 kernel stats of one bench config (default C2), CSV summaries only into gpurun_out/prof_<tag>/.
set -u
export TMPDIR=/tmp
TAG=${TAG:-c2}
ARGS=${ARGS:-}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --cpu-steps 0 $ARGS > gpurun_out/prof_$TAG/bench.log 2>&1 || exit 1
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$TAG/kernel_stats.csv \;
python tools/kstats.py gpurun_out/prof_$TAG/kernel_stats.csv
