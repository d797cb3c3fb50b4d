#!/bin/bash
# Round 6, last check of the committed tree: smoke, the whole -m gpu suite, the default bench line.
set -u
OUT=${OUT:-gpurun_out/r6verify}; mkdir -p $OUT
export TMPDIR=/tmp
step() {
    local name=$1 to=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400
    case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
step bench_c2 600 python bench.py
echo "session done"
