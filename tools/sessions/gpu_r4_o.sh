#!/bin/bash
# Round 4, session o: one allocation per step for a replay's fresh outputs (A/B at C2 / C4), the
# merged copy/draw launch's own GPU test.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_copy_spans.py tests/test_graph.py tests/test_fused.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest.log | tail -6
case $rc in 0) ;; *) exit $rc;; esac
for one in 0 1 0 1; do
  VMAS_HOST_ONE_ALLOC=$one timeout -k 10 200 python bench.py --cpu-steps 0 > $O/ab_one_c2_$one.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/ab_one_c2_$one.log').read().strip().splitlines()[-1]); print('C2 one=$one', round(d['value']/1e6,1), d['ms_per_step'])"
  VMAS_HOST_ONE_ALLOC=$one timeout -k 10 200 python bench.py --scenario discovery --cpu-steps 0 --steps 200 > $O/ab_one_c4_$one.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/ab_one_c4_$one.log').read().strip().splitlines()[-1]); print('C4 one=$one', round(d['value']/1e6,1), d['ms_per_step'])"
done
timeout -k 10 200 python tools/step_timeline.py balance 32768 > $O/timeline_c2.log 2>&1 || exit $?
tail -1 $O/timeline_c2.log | cut -c1-330
echo done
