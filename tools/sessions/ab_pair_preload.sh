#!/bin/bash
# A/B of the pair phase preload of other waves entity rows (VMAS_JIT_PAIR_PRELOAD=0|1), after the JIT tests.
set -u
mkdir -p gpurun_out/abq
timeout -k 10 600 python -u -m pytest tests/test_jit.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abq/tests.log 2>&1 || { tail -30 gpurun_out/abq/tests.log; exit 1; }
tail -1 gpurun_out/abq/tests.log
run() {  # tag, mode, bench args
  VMAS_JIT_PAIR_PRELOAD=$2 timeout -k 10 200 python bench.py --steps 60 --warmup 10 --cpu-steps 0 $3 > gpurun_out/abq/$1.json 2> gpurun_out/abq/$1.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/abq/$1.json')); r=d['roofline']; print('$1', r['kernel_us_per_launch'], r.get('kernel_us_event'), round(d['value']/1e6,1))"
}
for rep in 1 2; do
  for m in 0 1; do
    run bal_${m}_$rep $m ""
    run fl_${m}_$rep $m "--scenario flocking --n-agents 8 --substeps 0"
    run tr_${m}_$rep $m "--scenario transport --substeps 0"
  done
done
