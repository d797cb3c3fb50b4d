#!/bin/bash
# Round 6 closing evidence on the committed tree: smoke, the whole -m gpu suite, the bench lines,
# rocprofv3 kernel trace of the default bench command, and the PMC passes of the same (graph-mode)
# command (10 warm-up steps: every timed step a replay) -- tools/pmc_traffic.py splits the timed steps'
# k_world launches from the fused-timer and plain ones.
set -u
OUT=${OUT:-gpurun_out/r6final}; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stops the session on a crash / timeout
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-400
    case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
}
PART=${1:-all}  # A: smoke, suite, bench lines; B: rocprof + PMC (gpurun caps one call at 20 min)
if [ "$PART" != B ]; then
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1100 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
step bench_c2 600 python bench.py
step bench_c3 600 python bench.py --scenario transport --cpu-steps 0
step bench_c4 600 python bench.py --scenario discovery --cpu-steps 0
step bench_c5 600 python bench.py --scenario flocking --cpu-steps 0
step bench_c5full 600 python bench.py --scenario flocking --envs 262144 --steps 30 --warmup 10 --cpu-steps 0
step bench_c2_eager 600 python bench.py --graph off --cpu-steps 0
fi
if [ "$PART" != A ]; then
step prof_c2 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --cpu-steps 0
TAG=${PMC_TAG:-r6final} BENCH_ARGS="--steps 10 --warmup 10 --cpu-steps 0" bash tools/pmc_session.sh || exit $?
fi
echo "session done"
