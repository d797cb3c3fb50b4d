#!/bin/bash
# Round 6: flocking's program over two waves per (64 envs, agent) (VMAS_FLOCK_SPLIT=1,
# k_flocking_split): the bit-identity test, C5 shard A/B x3, kernel traces of both.
# (The variant measured slower and was reverted: profiles/r06/run14_flock_split.)
set -u
OUT=${OUT:-gpurun_out/r6m}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "flocking or lidar" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2 3; do
  for s in 0 1; do
    VMAS_FLOCK_SPLIT=$s timeout -k 10 200 python bench.py --scenario flocking --cpu-steps 0 --steps 200 > $OUT/c5_${s}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    echo "split=$s $(grep -o '"value": [0-9.]*' $OUT/c5_${s}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5_${s}_$i.log)"
  done
done
for s in 0 1; do
  VMAS_FLOCK_SPLIT=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$s -o run --output-format csv -- python bench.py --scenario flocking --cpu-steps 0 --steps 30 --event-launches 0 > $OUT/prof_$s.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  f=$(find $OUT/prof_$s -name 'run_kernel_stats.csv' | head -1); echo "split=$s"; grep -E "k_flocking|k_world|k_copy_draw" "$f" | cut -d, -f1-4 | cut -c1-140
done
echo "session done"
