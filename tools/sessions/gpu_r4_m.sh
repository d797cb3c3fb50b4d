#!/bin/bash
# Round 4, session m: the packed copy grid's units per thread (A/B at C2 / C5 shard), C2 step trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_copy_spans.py tests/test_graph.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "copy or replay_matches or preapplied" > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
for u in 4 1 4 1; do
  VMAS_COPY_UNITS=$u timeout -k 10 200 python bench.py --cpu-steps 0 > $O/ab_units_c2_$u.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/ab_units_c2_$u.log').read().strip().splitlines()[-1]); print('C2 units=$u', round(d['value']/1e6,1), d['ms_per_step'])"
  VMAS_COPY_UNITS=$u timeout -k 10 200 python bench.py --scenario flocking --cpu-steps 0 --steps 200 > $O/ab_units_c5_$u.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/ab_units_c5_$u.log').read().strip().splitlines()[-1]); print('C5 shard units=$u', round(d['value']/1e6,1), d['ms_per_step'])"
done
TAG=c2 ARGS="" bash tools/step_trace.sh > $O/step_trace_c2.txt 2>&1 || exit $?
tail -5 $O/step_trace_c2.txt
echo done
