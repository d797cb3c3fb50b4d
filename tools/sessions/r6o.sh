#!/bin/bash
# Round 6: plain vs non-temporal tail stores (VMAS_JIT_TAIL_STORE 0 / 1), C2 x5 interleaved pairs.
# (The knob was measured without gain and removed: profiles/r06/run16_tail_stores.)
set -u
OUT=${OUT:-gpurun_out/r6o2}; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  for m in 0 1; do
    VMAS_JIT_TAIL_STORE=$m timeout -k 10 200 python bench.py --cpu-steps 0 --steps 500 > $OUT/c2_${m}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    python - $OUT/c2_${m}_$i.log $m <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("mode", sys.argv[2], round(d["value"] / 1e6, 1), "M headline", d["roofline"]["kernel_us_per_launch"], "fused_no_tail", d["roofline"]["fused_no_tail"]["kernel_us"])
PY
  done
done
echo "session done"
