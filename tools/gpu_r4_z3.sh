#!/bin/bash
# Round 4, closing evidence 3/3 (after the host-path changes): smoke, the whole GPU suite, bench
# lines of C2 (graph x3, eager), C3, C4, C5 (full size and shard), rocprofv3 stats of C2.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4z3
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; tail -1 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/bench_c2_$i.log 2>&1 || exit $?
  echo "C2 run $i: $(tail -1 $O/bench_c2_$i.log | cut -c90-150)"
done
timeout -k 10 300 python bench.py --graph off --cpu-steps 0 > $O/bench_c2_eager.log 2>&1 || exit $?
echo "C2 eager: $(tail -1 $O/bench_c2_eager.log | cut -c90-150)"
timeout -k 10 300 python bench.py --scenario transport --cpu-steps 0 --steps 200 > $O/bench_c3.log 2>&1 || exit $?
echo "C3: $(tail -1 $O/bench_c3.log | cut -c90-150)"
timeout -k 10 300 python bench.py --scenario discovery --cpu-steps 0 --steps 200 > $O/bench_c4.log 2>&1 || exit $?
echo "C4: $(tail -1 $O/bench_c4.log | cut -c90-150)"
timeout -k 10 300 python bench.py --scenario flocking --envs 262144 --steps 40 --cpu-steps 0 > $O/bench_c5_full.log 2>&1 || exit $?
echo "C5 full: $(tail -1 $O/bench_c5_full.log | cut -c90-150)"
timeout -k 10 300 python bench.py --scenario flocking --cpu-steps 0 --steps 200 > $O/bench_c5_shard.log 2>&1 || exit $?
echo "C5 shard: $(tail -1 $O/bench_c5_shard.log | cut -c90-150)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --steps 50 --cpu-steps 0 > $O/prof_c2.log 2>&1 || exit $?
echo done
