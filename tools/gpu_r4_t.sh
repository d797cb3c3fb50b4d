#!/bin/bash
# Round 4, session t: the range-assert kernel with 32-bit index math -- graph / action GPU tests,
# C5 shard and full benches, the C5 shard dispatch trace (k_assert_range was 6.0 us).
set -u
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_graph.py tests/test_actions.py tests/test_fused.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest.log | tail -6
case $rc in 0) ;; *) exit $rc;; esac
for i in 1 2; do
  timeout -k 10 200 python bench.py --scenario flocking --cpu-steps 0 --steps 200 > $O/bench_c5_shard_$i.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/bench_c5_shard_$i.log').read().strip().splitlines()[-1]); print('C5 shard', round(d['value']/1e6,1), d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --scenario flocking --envs 262144 --steps 40 --cpu-steps 0 > $O/bench_c5_full.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('$O/bench_c5_full.log').read().strip().splitlines()[-1]); print('C5 full', round(d['value']/1e6,1), d['ms_per_step'])"
TAG=c5t ARGS="--scenario flocking" bash tools/step_trace.sh > $O/step_trace_c5shard.txt 2>&1 || exit $?
tail -8 $O/step_trace_c5shard.txt
echo done
