#!/bin/bash
# Round 6: what the tail's ~4.8 us is made of -- C2 kernel traces with the tail's copies or its draw
# dropped (VMAS_TAIL_DIAG, timing only: those steps' results are wrong), beside the full tail.
set -u
OUT=${OUT:-gpurun_out/r6k}; mkdir -p $OUT
export TMPDIR=/tmp
for v in full nocopy nodraw; do
  VMAS_TAIL_DIAG=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_$v -o run --output-format csv -- python bench.py --cpu-steps 0 --steps 40 --event-launches 0 > $OUT/prof_$v.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  python - "$OUT/prof_$v" "$v" <<'PY'
import csv, glob, statistics as st, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("k_world"))
d = [(e - s) / 1e3 for s, e in ks][10:50]
print(sys.argv[2], "in-step k_world median", round(st.median(d), 2), "mean", round(st.mean(d), 2), "n", len(d))
PY
done
echo "session done"
