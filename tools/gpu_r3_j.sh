#!/bin/bash
set -u
mkdir -p gpurun_out/r3j
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_graph.py tests/test_actions.py tests/test_fused.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3j/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/r3j/tests.log; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python tools/host_micro.py balance 32768 > gpurun_out/r3j/host_micro.log 2>&1 || exit $?
grep "whole step\|get_random\|post_replay" gpurun_out/r3j/host_micro.log
for i in 1 2; do timeout -k 10 200 python bench.py --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/r3j/bench_c2_$i.log 2>&1 || exit $?; grep -o '"value": [0-9.]*' gpurun_out/r3j/bench_c2_$i.log; done
timeout -k 10 200 python bench.py --scenario flocking --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/r3j/bench_c5.log 2>&1 || exit $?; grep -o '"value": [0-9.]*' gpurun_out/r3j/bench_c5.log
