#!/bin/bash
# Round evidence on one box: the GPU test suite and smoke, the C2 bench line + rocprofv3 kernel
# stats, the PMC passes of k_world (-> pmc_traffic.py record), then the C2-C5 matrix.  Stops at the
# first timeout / crash.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
SESSION_STEPS="tests smoke bench prof" bash tools/gpu_session.sh || exit $?
grep -q " passed" gpurun_out/pytest_gpu.log || { echo "GPU tests did not pass"; exit 1; }
PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH" TAG=final bash tools/pmc_session.sh || exit $?
bash tools/bench_matrix.sh || exit $?
echo "evidence done"
