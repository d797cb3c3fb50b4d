#!/bin/bash
# Round 5: (1) discovery's respawn chain inside the candidates launch (VMAS_SPAWN_FUSED_CHAIN,
# default 1) vs two launches; (2) a pre-applied replay's kernel chain launched by the post-replay
# C++ call (VMAS_GRAPH_CHAIN_IN_POST, default 1) vs its own ctypes call.  Spawn / graph / scenario
# GPU tests first, then interleaved A/Bs and the respawn phase probe.
set -u
OUT=gpurun_out/r5y; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_spawn.py tests/test_graph.py tests/test_scenario_oracle.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
b() {  # b <tag> <env assignment> <bench args...>
  local tag=$1 v=$2; shift 2
  env $v timeout -k 10 300 python bench.py --cpu-steps 0 "$@" > $OUT/bench_$tag.log 2>&1 || { echo "bench $tag rc=$?"; exit 1; }
  tail -1 $OUT/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d.get('respawn_handovers'))"
}
for i in 1 2; do
  b c4_fused1_$i VMAS_SPAWN_FUSED_CHAIN=1 --scenario discovery
  b c4_fused0_$i VMAS_SPAWN_FUSED_CHAIN=0 --scenario discovery
  for sc in transport flocking; do
    b ${sc}_inpost1_$i VMAS_GRAPH_CHAIN_IN_POST=1 --scenario $sc
    b ${sc}_inpost0_$i VMAS_GRAPH_CHAIN_IN_POST=0 --scenario $sc
  done
done
b c2_inpost1 VMAS_GRAPH_CHAIN_IN_POST=1 --scenario balance
b c2_inpost0 VMAS_GRAPH_CHAIN_IN_POST=0 --scenario balance
timeout -k 10 300 python -u tools/spawn_phase_probe.py > $OUT/spawn_phases_c4.txt 2>&1 || { echo "probe rc=$?"; tail -20 $OUT/spawn_phases_c4.txt; exit 1; }
cat $OUT/spawn_phases_c4.txt
