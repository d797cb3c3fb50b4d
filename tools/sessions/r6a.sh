#!/bin/bash
# Round 6: k_world with two 64-env groups per workgroup in lockstep (VMAS_JIT_NG=2) -- the physics /
# JIT / fused / graph / scenario-oracle GPU tests under it, then an interleaved C2 A/B (+ C3, C5 shard).
set -u
OUT=gpurun_out/r6a; mkdir -p $OUT
export TMPDIR=/tmp
VMAS_JIT_NG=2 timeout -k 10 900 python -u -m pytest tests/test_jit.py tests/test_gpu_parity.py tests/test_fused.py tests/test_graph.py tests/test_scenario_oracle.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_ng2.log 2>&1; rc=$?
tail -3 $OUT/pytest_ng2.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
for i in 1 2 3; do
  for v in 1 2; do
    VMAS_JIT_NG=$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_ng${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c2_ng${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2 ng=$v', d['value'], d['ms_per_step'], r['kernel_us_per_launch'], r.get('kernel_us_timed_region'))"
  done
done
for sc in transport flocking; do
  for v in 1 2; do
    VMAS_JIT_NG=$v timeout -k 10 300 python bench.py --scenario $sc --cpu-steps 0 > $OUT/bench_${sc}_ng${v}.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_${sc}_ng${v}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$sc ng=$v', d['value'], d['ms_per_step'], r['kernel_us_per_launch'])"
  done
done
echo "session done"
