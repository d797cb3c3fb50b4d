#!/bin/bash
# Round 4, session q: a replay's outputs as raw storage views (no dispatcher / autograd view
# bookkeeping) -- graph / fused / copy GPU tests, A/B at C2 / C4, the post_draw phases.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_copy_spans.py tests/test_graph.py tests/test_fused.py tests/test_actions.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest.log | tail -6
case $rc in 0) ;; *) exit $rc;; esac
VMAS_HOST_TIMING=1 timeout -k 10 200 python tools/step_timeline.py balance 32768 > $O/timeline_c2.log 2>&1 || exit $?
grep -E "post_draw|wall" $O/timeline_c2.log | cut -c1-300
for rv in 0 1 0 1; do
  VMAS_HOST_RAW_VIEWS=$rv timeout -k 10 200 python bench.py --cpu-steps 0 > $O/ab_raw_c2_$rv.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/ab_raw_c2_$rv.log').read().strip().splitlines()[-1]); print('C2 raw=$rv', round(d['value']/1e6,1), d['ms_per_step'])"
  VMAS_HOST_RAW_VIEWS=$rv timeout -k 10 200 python bench.py --scenario discovery --cpu-steps 0 --steps 200 > $O/ab_raw_c4_$rv.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/ab_raw_c4_$rv.log').read().strip().splitlines()[-1]); print('C4 raw=$rv', round(d['value']/1e6,1), d['ms_per_step'])"
done
echo done
