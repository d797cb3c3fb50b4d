#!/bin/bash
# Round 4, session c: the fixed draw-ahead test, a C2 dispatch trace, interleaved A/Bs (draw-ahead
# on/off at C2, non-temporal copy stores at C5 / C2), the C2 PMC passes of the current k_world and
# its rocprofv3 kernel stats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_graph.py tests/test_copy_spans.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_graph.log 2>&1; rc=$?
echo "graph tests rc=$rc"; tail -2 $O/pytest_graph.log
case $rc in 0|1) ;; *) exit $rc;; esac
TAG=c2 bash tools/step_trace.sh > $O/step_trace_c2.txt 2>&1 || exit $?
tail -3 $O/step_trace_c2.txt
for i in 1 2; do
  for da in 1 0; do
    VMAS_GRAPH_DRAW_AHEAD=$da timeout -k 10 200 python bench.py --cpu-steps 0 --steps 200 > $O/ab_drawahead_${da}_$i.log 2>&1 || exit $?
    echo "draw-ahead=$da run $i: $(tail -1 $O/ab_drawahead_${da}_$i.log | cut -c90-130)"
  done
done
for i in 1 2; do
  for nt in 0 1; do
    VMAS_COPY_NT=$nt timeout -k 10 300 python bench.py --scenario flocking --envs 262144 --steps 40 --cpu-steps 0 > $O/ab_nt_c5_${nt}_$i.log 2>&1 || exit $?
    echo "C5 nt=$nt run $i: $(tail -1 $O/ab_nt_c5_${nt}_$i.log | cut -c90-130)"
    VMAS_COPY_NT=$nt timeout -k 10 200 python bench.py --cpu-steps 0 --steps 200 > $O/ab_nt_c2_${nt}_$i.log 2>&1 || exit $?
    echo "C2 nt=$nt run $i: $(tail -1 $O/ab_nt_c2_${nt}_$i.log | cut -c90-130)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --steps 50 --cpu-steps 0 > $O/prof_c2.log 2>&1 || exit $?
TAG=r4c bash tools/pmc_session.sh || exit $?
echo done
