#!/bin/bash
# Round 4, session i: discovery's host timeline (where the host waits), hand-overs in the timed region.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 200 python bench.py --scenario discovery --cpu-steps 0 --steps 200 > $O/c4.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open('$O/c4.log').read().strip().splitlines()[-1]); print('C4', round(d['value']/1e6,1), d['ms_per_step'], 'handovers', d['config'].get('respawn_handovers'))"
timeout -k 10 200 python -u tools/step_timeline.py discovery 16384 > $O/timeline_c4.log 2>&1 || exit $?
tail -2 $O/timeline_c4.log
timeout -k 10 200 python -u tools/step_timeline.py flocking 32768 > $O/timeline_c5shard.log 2>&1 || exit $?
tail -2 $O/timeline_c5shard.log
timeout -k 10 200 python -u tools/host_micro.py discovery 16384 > $O/host_micro_c4.log 2>&1 || exit $?
cat $O/host_micro_c4.log
echo done
