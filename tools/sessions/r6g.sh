#!/bin/bash
# Round 6: after the closing records -- the debug worlds under the default graph step, the
# write-back size limit (C5 shard / C5 full), the contended-respawn test; the default C2 bench with
# the committed rocprof / PMC records attached.
set -u
OUT=${OUT:-gpurun_out/r6g}; mkdir -p $OUT
export TMPDIR=/tmp
step() {
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600
    case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
}
step pytest 900 python -u -m pytest tests/test_graph.py tests/test_spawn.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
step bench_c2_recheck 600 python bench.py
step bench_c5 600 python bench.py --scenario flocking --cpu-steps 0
step bench_c5full 600 python bench.py --scenario flocking --envs 262144 --steps 30 --warmup 10 --cpu-steps 0
echo "session done"
