#!/bin/bash
# Round 4, session k: adaptive window spread over every wave, the respawn's channel words staged by
# the reward launch (no clear kernel in graph mode) -- spawn / graph / fused tests, probe, C4.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_spawn.py tests/test_graph.py tests/test_fused.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest.log | tail -6
case $rc in 0|1) ;; *) exit $rc;; esac
for w in 128 96; do
  VMAS_SPAWN_WINDOW=$w timeout -k 10 120 python -u tools/spawn_probe.py 16384 0.001 > $O/probe_$w.log 2>&1 || exit $?
  echo "window=$w"; grep -A1 "T=7" $O/probe_$w.log
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --scenario discovery --cpu-steps 0 --steps 200 > $O/c4_$i.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('$O/c4_$i.log').read().strip().splitlines()[-1]); print('C4 run $i', round(d['value']/1e6,1), d['ms_per_step'], d['config'].get('respawn_handovers'))"
done
TAG=c4 ARGS="--scenario discovery" bash tools/step_trace.sh > $O/step_trace_c4.txt 2>&1 || exit $?
tail -10 $O/step_trace_c4.txt
for pk in 0 1 0 1; do
  VMAS_COPY_PACKED=$pk timeout -k 10 200 python bench.py --cpu-steps 0 > $O/ab_packed_c2_$pk.log 2>&1 || exit $?
  echo "C2 packed=$pk $(tail -1 $O/ab_packed_c2_$pk.log | cut -c1-120)"
  VMAS_COPY_PACKED=$pk timeout -k 10 200 python bench.py --scenario discovery --cpu-steps 0 --steps 200 > $O/ab_packed_c4_$pk.log 2>&1 || exit $?
  echo "C4 packed=$pk $(tail -1 $O/ab_packed_c4_$pk.log | cut -c1-120)"
done
for sc in discovery balance; do
  VMAS_COPY_TRACE=1 timeout -k 10 150 python bench.py --scenario $sc --cpu-steps 0 --steps 20 > $O/copytrace_$sc.out 2> $O/copytrace_$sc.log || exit $?
done
grep -c span $O/copytrace_discovery.log $O/copytrace_balance.log
timeout -k 10 200 python tools/host_profile.py discovery 16384 300 > $O/host_profile_c4.log 2>&1 || exit $?
echo done
