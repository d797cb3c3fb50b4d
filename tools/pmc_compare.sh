set -u
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
export PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH"
TAG=split_auto bash tools/pmc_session.sh || exit $?
VMAS_SPLIT_PAIRS=0 TAG=split_off bash tools/pmc_session.sh || exit $?
