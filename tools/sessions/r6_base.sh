#!/bin/bash
# Round 6 start: the committed tree's C2 bench and the rocprof summary of the same command.
set -u
OUT=${OUT:-gpurun_out/r6base}; mkdir -p $OUT
export TMPDIR=/tmp
step() {
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-600
    case $rc in 0) ;; *) echo "fatal rc=$rc, stopping"; exit $rc;; esac
}
step bench_c2 600 python bench.py
step prof_c2 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --cpu-steps 0
echo "session done"
