#!/bin/bash
# Round 4, session b: the C++ host path (_vmas_host), action-shadow and fresh-state changes:
# graph / fused / action / rng tests first, then the whole suite, the C2 bench (graph + eager),
# the host profile and the C5 full-size bench.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_graph.py tests/test_fused.py tests/test_actions.py tests/test_rng.py tests/test_spawn.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_graph.log 2>&1; rc=$?
echo "graph tests rc=$rc"; tail -3 $O/pytest_graph.log
case $rc in 0) ;; 1) grep -n "Error\|assert" $O/pytest_graph.log | head -20;; *) exit $rc;; esac
timeout -k 10 200 python tools/host_micro.py balance 32768 > $O/host_micro.log 2>&1 || exit $?
grep -v amdgpu.ids $O/host_micro.log | tail -11
for i in 1 2; do timeout -k 10 300 python bench.py > $O/bench_c2_$i.log 2>&1 || exit $?; tail -1 $O/bench_c2_$i.log | cut -c1-400; done
timeout -k 10 300 python bench.py --graph off --cpu-steps 0 > $O/bench_c2_eager.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --scenario flocking --envs 262144 --steps 50 --cpu-steps 0 > $O/bench_c5_full.log 2>&1 || exit $?
tail -1 $O/bench_c5_full.log | cut -c1-300
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 $O/pytest_gpu.log
timeout -k 10 200 python tools/jit_phase_profile.py balance 32768 > $O/phase_profile.log 2>&1 || exit $?
echo done
