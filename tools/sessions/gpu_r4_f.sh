#!/bin/bash
# Round 4, session f: windowed respawn v4 (cluster-reduced tables, speculative chain) -- spawn
# parity, discovery graph tests, probe, C4 A/B, C4 dispatch trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_spawn.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_spawn.log 2>&1; rc=$?
echo "spawn tests rc=$rc"; tail -3 $O/pytest_spawn.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -m pytest tests/test_graph.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "discovery or respawn or spawn" > $O/pytest_graph_disc.log 2>&1; rc=$?
echo "graph discovery tests rc=$rc"; tail -2 $O/pytest_graph_disc.log
case $rc in 0|1|5) ;; *) exit $rc;; esac
for cov in 0 0.001 0.004; do
  timeout -k 10 120 python -u tools/spawn_probe.py 16384 $cov > $O/probe_$cov.log 2>&1 || exit $?
  echo "cov=$cov"; grep -A1 "T=7" $O/probe_$cov.log
done
for i in 1 2; do
  for k in window resident; do
    VMAS_SPAWN_KERNEL=$k timeout -k 10 200 python bench.py --scenario discovery --cpu-steps 0 --steps 100 > $O/ab_c4_${k}_$i.log 2>&1 || exit $?
    echo "C4 $k run $i: $(tail -1 $O/ab_c4_${k}_$i.log | cut -c90-130)"
  done
done
TAG=c4 ARGS="--scenario discovery" bash tools/step_trace.sh > $O/step_trace_c4.txt 2>&1 || exit $?
tail -12 $O/step_trace_c4.txt
echo done
