#!/bin/bash
# Round 6: where the state write-back's time goes -- per-step dispatch traces of C2 with and without
# it, C5 shard; and why (or whether) flocking's replay takes it.
set -u
OUT=gpurun_out/r6c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python - > $OUT/wb_probe.log 2>&1 <<'PY'
import torch
from vectorizedmultiagentsimulator_amd import make_env
for name, kw in (("balance", dict(n_agents=4)), ("flocking", dict(n_agents=8)), ("transport", dict(n_agents=4))):
    env = make_env(name, num_envs=32768, device="cuda:0", seed=0, **kw)
    if name == "balance":
        env.world._substeps = 10; env.world._sub_dt = env.world._dt / 10
    for _ in range(12):
        env.step(env.get_random_actions())
    g = env._graph
    ch = g._chain
    print(name, "status", env.graph_status, "chain", None if ch is None else (ch.n_nodes, ch.fused), g.chain_why,
          "wb", None if g._wb is None else (g._wb if g._wb is False else "on"), "state_idx", g._state_idx,
          "carry", g._carry_names, "other", len(g._carry_other), "preapplied", env.preapplied_steps, flush=True)
PY
cat $OUT/wb_probe.log | tail -5
TAG=c2_wb1 bash tools/step_trace.sh > $OUT/c2_wb1.txt 2>&1 || exit 1
VMAS_GRAPH_WRITEBACK=0 TAG=c2_wb0 bash tools/step_trace.sh > $OUT/c2_wb0.txt 2>&1 || exit 1
TAG=c5_wb1 ARGS="--scenario flocking" bash tools/step_trace.sh > $OUT/c5_wb1.txt 2>&1 || exit 1
head -30 $OUT/c2_wb1.txt; head -30 $OUT/c2_wb0.txt; head -30 $OUT/c5_wb1.txt
echo "session done"
