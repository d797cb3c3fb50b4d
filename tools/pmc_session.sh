#!/bin/bash
# rocprofv3 PMC passes for the k_step kernel (one counter group per pass, kernel-trace only).
#   PASSES   ';'-separated counter groups (default: HBM bytes, then SQ instruction/stall groups)
#   TAG      output sub-directory name (gpurun_out/pmc/<TAG>)
#   BENCH_ARGS  arguments of bench.py
# A pass that fails with a plain error (e.g. an unknown counter, rc 1) is reported and skipped;
# a timeout / abort / crash (124, 134, 137, 139) stops the session.
set -u
export TMPDIR=/tmp
TAG="${TAG:-default}"
OUT="gpurun_out/pmc/$TAG"
mkdir -p "$OUT"
ARGS="${BENCH_ARGS:---steps 10 --warmup 3 --cpu-steps 0}"
PASSES="${PASSES:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_WAIT_ANY SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE}"
i=0
IFS=';' read -ra GROUPS_ <<< "$PASSES"
for counters in "${GROUPS_[@]}"; do
  i=$((i+1))
  echo "=== $TAG pass $i: $counters"
  # shellcheck disable=SC2086
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-include-regex "^(k_step|k_world)$" -d "$OUT/p$i" -o pmc --output-format csv -- python bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 2 "$OUT/p$i.log"
  case $rc in 0|1|2) ;; *) echo "stopping"; exit $rc;; esac
done
