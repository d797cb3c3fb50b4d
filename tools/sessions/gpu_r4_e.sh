#!/bin/bash
# Round 4, session e: windowed respawn v2 (templated candidates kernel, packed tests) -- spawn
# parity, discovery graph tests, the spawn probe with per-phase stamps, C4 A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_spawn.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_spawn.log 2>&1; rc=$?
echo "spawn tests rc=$rc"; tail -3 $O/pytest_spawn.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -u tools/spawn_probe.py 16384 0.001 > $O/spawn_probe_window.log 2>&1 || exit $?
cat $O/spawn_probe_window.log
VMAS_SPAWN_WINDOW=96 timeout -k 10 120 python -u tools/spawn_probe.py 16384 0.001 > $O/spawn_probe_window96.log 2>&1 || exit $?
cat $O/spawn_probe_window96.log
for i in 1 2; do
  for k in window resident; do
    VMAS_SPAWN_KERNEL=$k timeout -k 10 200 python bench.py --scenario discovery --cpu-steps 0 --steps 100 > $O/ab_c4_${k}_$i.log 2>&1 || exit $?
    echo "C4 $k run $i: $(tail -1 $O/ab_c4_${k}_$i.log | cut -c90-130)"
  done
done
echo done
