#!/bin/bash
# Graph-mode check on the GPU: probe, graph + jit + actions tests, then bench with graph on / off.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python tools/graph_probe.py balance > gpurun_out/graph_probe.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/graph_probe.log
timeout -k 10 600 python -u -m pytest tests/test_graph.py tests/test_jit.py tests/test_actions.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_graph.log 2>&1
rc=$?; tail -n 30 gpurun_out/pytest_graph.log; echo "graph tests rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --cpu-steps 0 --graph on > gpurun_out/bench_graph.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_graph.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0 --graph off > gpurun_out/bench_eager.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_eager.log
