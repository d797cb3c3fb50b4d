#!/bin/bash
# Evidence for profiles/: PMC traffic + SQ counters of the step kernel, then the config matrix.
set -u
export TMPDIR=/tmp
PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH" TAG=final bash tools/pmc_session.sh || exit $?
bash tools/bench_matrix.sh || exit $?
