#!/bin/bash
# Round 4, closing evidence 2/2: the k_world PMC passes of the C2 bench (the bench line's traffic /
# issue record), bench lines of C3, C4, C5 (full size and the per-GPU shard) with C4 / C5 rocprof.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
TAG=r4z bash tools/pmc_session.sh > $O/pmc_session.log 2>&1 || exit $?
tail -4 $O/pmc_session.log
timeout -k 10 300 python bench.py --scenario transport --cpu-steps 0 --steps 200 > $O/bench_c3.log 2>&1 || exit $?
echo "C3: $(tail -1 $O/bench_c3.log | cut -c90-150)"
timeout -k 10 300 python bench.py --scenario discovery --cpu-steps 0 --steps 200 > $O/bench_c4.log 2>&1 || exit $?
echo "C4: $(tail -1 $O/bench_c4.log | cut -c90-150)"
timeout -k 10 300 python bench.py --scenario flocking --envs 262144 --steps 40 --cpu-steps 0 > $O/bench_c5_full.log 2>&1 || exit $?
echo "C5 full: $(tail -1 $O/bench_c5_full.log | cut -c90-150)"
timeout -k 10 300 python bench.py --scenario flocking --cpu-steps 0 --steps 200 > $O/bench_c5_shard.log 2>&1 || exit $?
echo "C5 shard: $(tail -1 $O/bench_c5_shard.log | cut -c90-150)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 --output-format csv -- python bench.py --scenario discovery --steps 50 --cpu-steps 0 > $O/prof_c4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --scenario flocking --envs 262144 --steps 20 --cpu-steps 0 > $O/prof_c5.log 2>&1 || exit $?
echo done
