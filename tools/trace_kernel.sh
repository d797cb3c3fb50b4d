#!/bin/bash
# rocprofv3 kernel trace of a bench config; prints the durations of KERNEL's dispatches of the
# last few steps with the gaps to the previous dispatch (TAG, ARGS, KERNEL).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/trace/$TAG
mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --kernel-trace -d /tmp/tr -o tr --output-format csv -- python bench.py --steps 10 --warmup 5 --cpu-steps 0 $ARGS > $OUT/run.log 2>&1 || { echo "rc=$?"; exit 1; }
f=$(find /tmp/tr -name "*kernel_trace.csv" | head -1)
python - "$f" "$KERNEL" > $OUT/summary.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
for i in sel[-21:]:
    r = rows[i]; p = rows[i - 1] if i else r
    print(f"{r['Kernel_Name'][:50]:50s} dur {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.2f} us  gap {(int(r['Start_Timestamp']) - int(p['End_Timestamp'])) / 1e3:8.2f} us after {p['Kernel_Name'][:40]}")
PY
cat $OUT/summary.txt
