"""Probe: who overwrites the spawn channel's words in test_fused's discovery sequence (speculative
graph steps with cloned actions).  After every stage of each graph step the stream is synchronised
and the channel words are checked; the first stage that leaves words outside the launch's layout is
reported with the data pointers of every candidate buffer."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402
from vectorizedmultiagentsimulator_amd.simulator.environment import _graph  # noqa: E402
from vectorizedmultiagentsimulator_amd.simulator.environment.environment import Environment  # noqa: E402

envs = int(sys.argv[1]) if len(sys.argv) > 1 else 777
env = make_env("discovery", num_envs=envs, device="cuda:0", seed=3, graph_step=True, n_agents=5, use_agent_lidar=True)
stage = ["init"]


def words():
    ch = getattr(env.scenario, "_spawn_channel", None)
    if ch is None:
        return None, None
    torch.cuda.synchronize()
    return ch.mx, ch.mx.tolist()


def check(where):
    mx, w = words()
    if w is None:
        return
    bad = [i for i, v in enumerate(w) if v < 0 or v > 1 << 20]
    print(f"  [{where}] mx@{mx.data_ptr():#x} bad words {len(bad)} first {bad[:6]} w0..8 {w[:8]}", flush=True)
    if bad:
        v = w[bad[0]] & 0xFFFFFFFF
        hi = w[bad[0] + 1] & 0xFFFFFFFF if bad[0] + 1 < len(w) else 0
        print(f"  value {hi:#x}{v:08x}", flush=True)
        cands = {}
        for i, a in enumerate(env.agents):
            cands[f"agent{i}.u"] = a.action.u
            cands[f"agent{i}.u_range_t"] = a.action._u_range_tensor
            cands[f"agent{i}.u_mult_t"] = a.action._u_multiplier_tensor
        up = env._u_persist
        if up is not None:
            cands["u_persist"] = up[1]
        g = env._graph
        for i, t in enumerate(g._bk_dst):
            cands[f"bk_dst{i}"] = t
        for i, t in enumerate(g._bk_src):
            cands[f"bk_src{i}"] = t
        for i, t in enumerate(env.scenario._targets):
            cands[f"target{i}.pos"] = t.state.pos
        for k, t in cands.items():
            if isinstance(t, torch.Tensor):
                print(f"    {k:16s} {t.data_ptr():#x} .. {t.data_ptr() + t.numel() * t.element_size():#x}", flush=True)
        raise SystemExit(f"corrupted at {where}")


G = _graph.StepGraph
for name in ("backup", "_launch", "_post_replay", "_finish_deferred", "before_actions"):
    orig = getattr(G, name)

    def wrap(self, *a, _orig=orig, _name=name, **k):
        check(f"before {_name}")
        r = _orig(self, *a, **k)
        if _name != "_finish_deferred":
            check(f"after {_name}")
        return r

    setattr(G, name, wrap)
orig_apply = Environment._apply_continuous_actions


def apply_wrap(self, *a, **k):
    r = orig_apply(self, *a, **k)
    check("after _apply_continuous_actions")
    return r


Environment._apply_continuous_actions = apply_wrap
for t in range(8):
    print(f"step {t}", flush=True)
    acts = [a.clone() for a in env.get_random_actions()]
    env.step(acts)
print("no corruption seen")
