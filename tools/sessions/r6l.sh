#!/bin/bash
# Round 6: what bounds k_flocking_fast at C5 shard (flocking 32 768 envs x 8 agents): kernel trace
# of the default C5 bench, then PMC passes on k_flocking_fast alone.
set -u
OUT=${OUT:-gpurun_out/r6l}; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--scenario flocking --cpu-steps 0 --steps 30 --warmup 10 --event-launches 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py $ARGS > $OUT/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
tail -1 $OUT/prof.log | cut -c1-160
f=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | cut -c1-150
i=0
for counters in "FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" "WRITE_SIZE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $counters --kernel-include-regex "k_flocking_fast" -d $OUT/p$i -o pmc --output-format csv -- python bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0|1|2) ;; *) exit $rc;; esac
  python - "$OUT/p$i" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/pmc_counter_collection.csv", recursive=True)
if not f: print("no csv"); sys.exit(0)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    v = v[-20:]
    print(f"  {k}: {sum(v)/len(v):.1f} per dispatch (n={len(v)})")
PY
done
echo "session done"
