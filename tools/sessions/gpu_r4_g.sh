#!/bin/bash
# Round 4, session g: direct outputs (all four fused scenarios) -- graph / fused tests, A/B direct
# on/off at C2, C3, C4, C5 (full size).
set -u
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_graph.py tests/test_fused.py tests/test_copy_spans.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_graph.log 2>&1; rc=$?
echo "graph tests rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest_graph.log | tail -8
case $rc in 0|1) ;; *) exit $rc;; esac
ab() {  # name, bench args, steps
  for i in 1 2; do
    for d in 1 0; do
      VMAS_GRAPH_DIRECT_OUTPUTS=$d timeout -k 10 300 python bench.py --cpu-steps 0 --steps $3 $2 > $O/ab_$1_${d}_$i.log 2>&1 || return $?
      echo "$1 direct=$d run $i: $(tail -1 $O/ab_$1_${d}_$i.log | cut -c90-130)"
    done
  done
}
ab c2 "" 200 || exit $?
ab c4 "--scenario discovery" 100 || exit $?
ab c5 "--scenario flocking --envs 262144" 40 || exit $?
ab c3 "--scenario transport" 200 || exit $?
echo done
