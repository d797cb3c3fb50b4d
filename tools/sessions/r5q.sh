#!/bin/bash
# Round 5: the scenario program's argument block copied into LDS at k_world's start
# (VMAS_JIT_EPI_LDS) -- parity of the fused programs, interleaved C2 / C3 A/B.
set -u
OUT=gpurun_out/r5q; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -v -m gpu"
timeout -k 10 900 $T tests/test_fused.py tests/test_graph.py "tests/test_scenario_oracle.py::test_scenario_programs_match_oracle_full_size_gpu" > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/tests.log | tail -8
case $rc in 124|134|137|139) exit $rc;; esac
for i in 1 2; do
  for v in 1 0; do
    for sc in balance transport; do
      VMAS_JIT_EPI_LDS=$v timeout -k 10 300 python bench.py --scenario $sc --cpu-steps 0 > $OUT/bench_${sc}_lds${v}_$i.log 2>&1 || { echo "bench rc=$?"; tail -3 $OUT/bench_${sc}_lds${v}_$i.log; exit 1; }
      tail -1 $OUT/bench_${sc}_lds${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc lds=$v', d['value'], d['ms_per_step'])"
    done
  done
done
