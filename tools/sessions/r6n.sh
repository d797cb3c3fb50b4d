#!/bin/bash
# Round 6: the tail's store kind (VMAS_JIT_TAIL_STORE: 0 plain, 1 non-temporal, 2 agent-scope
# write-through) -- graph parity of balance / transport under each, C2 A/B/C x3, kernel traces.
# (The knob was measured without gain and removed: profiles/r06/run16_tail_stores.)
set -u
OUT=${OUT:-gpurun_out/r6n}; mkdir -p $OUT
export TMPDIR=/tmp
for m in 1 2; do
  VMAS_JIT_TAIL_STORE=$m timeout -k 10 400 python -u -m pytest tests/test_graph.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "preapplied and (balance or transport)" > $OUT/pytest_$m.log 2>&1 || { tail -30 $OUT/pytest_$m.log; exit 1; }
  echo "mode $m: $(tail -1 $OUT/pytest_$m.log)"
done
for i in 1 2 3; do
  for m in 0 1 2; do
    VMAS_JIT_TAIL_STORE=$m timeout -k 10 200 python bench.py --cpu-steps 0 --steps 300 > $OUT/c2_${m}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    python - $OUT/c2_${m}_$i.log $m <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("mode", sys.argv[2], round(d["value"] / 1e6, 1), "M", d["ms_per_step"] * 1e3, "us/step", "headline", d["roofline"]["kernel_us_per_launch"], d["config"].get("step_mode"))
PY
  done
done
echo "session done"
