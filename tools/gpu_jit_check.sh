#!/bin/bash
# GPU check of the specialised step: tests, bench line, per-wave phase profile, kernel stats.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench.log 2>&1 || exit $?
tail -c 900 gpurun_out/bench.log
timeout -k 10 200 python tools/jit_phase_profile.py balance 32768 200 > gpurun_out/phase_balance.log 2>&1 || exit $?
head -14 gpurun_out/phase_balance.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-steps 0 > gpurun_out/rocprof.log 2>&1 || exit $?
rm -f gpurun_out/prof/*_kernel_trace.csv
grep -E "k_world|k_step" gpurun_out/prof/run_kernel_stats.csv
