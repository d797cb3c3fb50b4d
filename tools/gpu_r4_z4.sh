#!/bin/bash
# Round 4, final check of the tree as committed: smoke, the whole GPU suite, one C2 bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4z4
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; tail -1 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || exit $?
echo "C2: $(tail -1 $O/bench_c2.log | cut -c90-150)"
echo done
