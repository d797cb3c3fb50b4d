#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
for w in 128 96; do
  VMAS_SPAWN_WINDOW=$w timeout -k 10 120 python -u tools/spawn_probe.py 16384 0.001 > $O/probe_$w.log 2>&1 || exit $?
  echo "window=$w"; grep -A1 "T=7" $O/probe_$w.log
done
echo done
