#!/bin/bash
# Round 5: a wave per LIDAR (discovery) / per half of the rays (flocking) -- parity, then an
# interleaved A/B against the per-agent kernels; step traces of C2 / C4 / C5 shard.
set -u
OUT=gpurun_out/r5g; mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -v -m gpu"
timeout -k 10 900 $T tests/test_fused.py "tests/test_scenario_oracle.py::test_scenario_programs_match_oracle_full_size_gpu" "tests/test_scenario_oracle.py::test_scenario_programs_match_oracle_eager_gpu" > $OUT/tests.log 2>&1; echo "tests rc=$?"
grep -E "passed|failed" $OUT/tests.log | tail -2
for i in 1 2; do
  for v in 1 0; do
    VMAS_FLOCK_SPLIT=$v timeout -k 10 300 python bench.py --scenario flocking --steps 100 --warmup 10 --cpu-steps 0 > $OUT/bench_c5_split${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c5_split${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 split=$v', d['value'], d['ms_per_step'])"
    VMAS_DISC_OBS_SPLIT=$v timeout -k 10 300 python bench.py --scenario discovery --steps 100 --warmup 10 --cpu-steps 0 > $OUT/bench_c4_split${v}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    tail -1 $OUT/bench_c4_split${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 split=$v', d['value'], d['ms_per_step'])"
  done
done
for c in c5:flocking c4:discovery c2:balance; do
  tag=${c%%:*}; sc=${c##*:}
  TAG=r5g_$tag ARGS="--scenario $sc" bash tools/step_trace.sh > /dev/null 2>&1; cp gpurun_out/steptrace/r5g_$tag/summary.txt $OUT/step_trace_$tag.txt; tail -14 $OUT/step_trace_$tag.txt
done
