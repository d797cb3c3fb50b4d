#!/bin/bash
# PMC passes of one named kernel during a bench config: KERNEL (regex), ARGS (bench args), TAG.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmck/$TAG
mkdir -p $OUT
i=0
for counters in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM" "FETCH_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --kernel-include-regex "$KERNEL" -d /tmp/pmck_$i -o pmc --output-format csv -- python bench.py --steps 5 --warmup 3 --cpu-steps 0 $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
  find /tmp/pmck_$i -name "*counter_collection.csv" -exec cp {} $OUT/p${i}.csv \;
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/p*.csv"):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(tot): print(f"{k:22s} per dispatch {tot[k] / max(len(n[k]), 1):14.1f}  ({len(n[k])} dispatches)")
PY
