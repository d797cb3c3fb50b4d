#!/bin/bash
# Round 5 closing evidence, fourth pass (the chain launched by the post-replay call):
# smoke, the whole -m gpu suite, the bench lines and rocprofv3 of the default bench command (k_world's
# source is final3's: its PMC record stands).
set -u
OUT=${OUT:-gpurun_out/r5final4}; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stops the session on a crash / timeout
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-400
    case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1100 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
step bench_c2 600 python bench.py
step bench_c3 600 python bench.py --scenario transport --cpu-steps 0
step bench_c4 600 python bench.py --scenario discovery --cpu-steps 0
step bench_c5 600 python bench.py --scenario flocking --cpu-steps 0
step bench_c5full 600 python bench.py --scenario flocking --envs 262144 --steps 30 --warmup 10 --cpu-steps 0
step bench_c2_eager 600 python bench.py --graph off --cpu-steps 0
step rocprof_c2 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py
echo "session done"
