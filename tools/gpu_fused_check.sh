#!/bin/bash
# Fused scenario programs: parity tests against the torch programs, then the bench matrix.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fused.py tests/test_graph.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; tail -n 30 gpurun_out/pytest_fused.log; [ $rc -eq 0 ] || exit $rc
for cfg in "balance|" "balance_torch|VMAS_FUSED_SCENARIOS=0"; do
  name=${cfg%%|*}; envs=${cfg#*|}
  env $envs timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/bench_$name.json')); print('$name', round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms', d['roofline']['kernel_us_per_launch'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-steps 0 > gpurun_out/prof_fused.log 2>&1 || exit $?
echo done
