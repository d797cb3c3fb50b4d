#!/bin/bash
# Round 5: k_world code generation -- one group loop per wave (VMAS_JIT_LOOP_PER_WAVE) and the
# v_minimum3 / v_maximum3 NaN-propagating min / max in relaxed worlds.  Parity (physics + scenario
# oracle), interleaved C2 A/B, one PMC pass per variant (VALU / SALU instruction counts).
set -u
OUT=gpurun_out/r5m; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -v -m gpu"
timeout -k 10 1000 $T tests/test_gpu_parity.py tests/test_jit.py tests/test_graph.py "tests/test_scenario_oracle.py::test_scenario_programs_match_oracle_full_size_gpu" > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/tests.log | tail -14
case $rc in 124|134|137|139) exit $rc;; esac
for i in 1 2; do
  for v in 1 0; do
    VMAS_JIT_LOOP_PER_WAVE=$v timeout -k 10 300 python bench.py --cpu-steps 0 > $OUT/bench_c2_lpw${v}_$i.log 2>&1 || { echo "bench rc=$?"; tail -3 $OUT/bench_c2_lpw${v}_$i.log; exit 1; }
    tail -1 $OUT/bench_c2_lpw${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 lpw=$v', d['value'], d['ms_per_step'], d['roofline']['achieved'], d.get('kernel_us_eager_events'))"
  done
done
for v in 1 0; do
  VMAS_JIT_LOOP_PER_WAVE=$v timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-include-regex "^k_world$" -d $OUT/pmc_lpw$v -o pmc --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-steps 0 > $OUT/pmc_lpw$v.log 2>&1; echo "pmc lpw=$v rc=$?"
  f=$(find $OUT/pmc_lpw$v -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: round(sum(v) / max(1, len(set(r["Dispatch_Id"] for r in rows))), 1) for k, v in acc.items()})
PY
done
