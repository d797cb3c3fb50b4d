#!/bin/bash
# Round 4, session h: C4 / C5-shard dispatch traces with direct outputs, C4 hand-over count,
# A/B of 16 waves per workgroup for balance's k_world.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --scenario discovery --cpu-steps 0 --steps 200 > $O/c4_$i.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('$O/c4_$i.log').read().strip().splitlines()[-1]); print('C4 run $i', round(d['value']/1e6,1), d['ms_per_step'], 'handovers', d['config'].get('respawn_handovers'))"
done
TAG=c4 ARGS="--scenario discovery" bash tools/step_trace.sh > $O/step_trace_c4.txt 2>&1 || exit $?
tail -11 $O/step_trace_c4.txt
timeout -k 10 200 python bench.py --scenario flocking --cpu-steps 0 --steps 200 > $O/c5shard.log 2>&1 || exit $?
echo "C5 shard: $(tail -1 $O/c5shard.log | cut -c90-160)"
TAG=c5shard ARGS="--scenario flocking" bash tools/step_trace.sh > $O/step_trace_c5shard.txt 2>&1 || exit $?
tail -9 $O/step_trace_c5shard.txt
for i in 1 2; do
  for w in 16 8; do
    VMAS_JIT_WAVES=$w timeout -k 10 200 python bench.py --cpu-steps 0 --steps 200 > $O/ab_waves_${w}_$i.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open('$O/ab_waves_${w}_$i.log').read().strip().splitlines()[-1]); print('C2 waves=$w run $i', round(d['value']/1e6,1), d['roofline']['kernel_us_per_launch'])"
  done
done
echo done
