"""Probe: the graph-mode discovery step with the deferred respawn (test_fused's sequence), dumping
the spawn words of a failing launch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402
from vectorizedmultiagentsimulator_amd import _native as N  # noqa: E402

envs = int(sys.argv[1]) if len(sys.argv) > 1 else 777
env = make_env("discovery", num_envs=envs, device="cuda:0", seed=3, graph_step=True, n_agents=5, use_agent_lidar=True)
for t in range(14):
    if t == 5:
        env.reset_at(7)
    if t == 9:
        env.reset()
    try:
        acts = env.get_random_actions()
        if os.environ.get("PROBE_CLONE", "1") == "1":  # test_fused's form: cloned actions (the speculative path)
            acts = [a.clone() for a in acts]
        env.step(acts)
    except Exception as ex:  # noqa: BLE001
        g = env._graph
        print(f"step {t}: {type(ex).__name__}: {ex}", flush=True)
        for d in g._deferred:
            torch.cuda.synchronize()
            w = d.mx.tolist()
            T = d.T
            print("maxima", w[:T], "unresolved", w[T], "claim", w[32], "err", w[64],
                  "done", [w[96 + 32 * i] for i in range(T)], flush=True)
            rep = d.mx[96 + 32 * T:].view(torch.int64).tolist()
            print("replicas", [(r >> 32, r & 0xFFFFFFFF) for r in rep[::16]], flush=True)
        raise
    print(f"step {t}: ok, graph {env.graph_status}, deferred {len(env._graph._deferred)}", flush=True)
