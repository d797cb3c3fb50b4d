#!/bin/bash
# Round 4, first GPU session: the whole -m gpu suite (C5 at 262 144 envs, aggregate error
# guards, features exact vs relaxed), the C2 graph / eager bench lines, the C5 full-size bench
# with its rocprofv3 kernel stats, and two PMC passes of k_world at C2 (wait attribution).
set -u
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "rocprofv3 -L rc=$?"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || exit $?
tail -1 $O/bench_c2.log
timeout -k 10 300 python bench.py --graph off --cpu-steps 0 > $O/bench_c2_eager.log 2>&1 || exit $?
tail -1 $O/bench_c2_eager.log
timeout -k 10 300 python bench.py --scenario flocking --envs 262144 --steps 50 --cpu-steps 0 > $O/bench_c5_full.log 2>&1 || exit $?
tail -1 $O/bench_c5_full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --scenario flocking --envs 262144 --steps 20 --cpu-steps 0 > $O/prof_c5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --steps 50 --cpu-steps 0 > $O/prof_c2.log 2>&1 || exit $?
PASSES="SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM" TAG=r4a bash tools/pmc_session.sh || exit $?
echo done
