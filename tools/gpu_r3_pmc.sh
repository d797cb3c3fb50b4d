#!/bin/bash
# The closing PMC record of k_world (the source hash changes with the header) plus the graph tests
# and the C2 bench / host profile of the final host path.  Stops at a timeout / crash.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3p
PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" TAG=final3 bash tools/pmc_session.sh || exit $?
timeout -k 10 400 python -u -m pytest tests/test_graph.py tests/test_fused.py tests/test_actions.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3p/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r3p/tests.log; case $rc in 0|1) ;; *) exit $rc;; esac
for i in 1 2; do timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/r3p/bench_$i.log 2>&1 || exit $?; done
timeout -k 10 200 python tools/host_micro.py balance 32768 > gpurun_out/r3p/host_micro.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r3p/host_micro.log | tail -11
echo done
