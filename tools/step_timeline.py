"""Where a graph-mode step's wall time goes (no profiler: its serialisation distorts tiny kernels).

Host phases of `env.step(env.get_random_actions())` by perf_counter stamps (monkeypatched around
the StepGraph / Environment methods), and the GPU time of the replayed graph and of the action
kernel by HIP events recorded on the stream around them (outside the graph).
Usage: python tools/step_timeline.py [scenario] [envs]
"""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402
from vectorizedmultiagentsimulator_amd.simulator.environment import _graph  # noqa: E402
from vectorizedmultiagentsimulator_amd.simulator.environment.environment import Environment  # noqa: E402

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
kw = {"n_agents": 8 if scenario in ("discovery", "flocking") else 4}
if scenario == "discovery":  # (bench.py's C4)
    kw["use_agent_lidar"] = True
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, graph_step=True, **kw)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
import os  # noqa: E402

if os.environ.get("SKIP_PHYSICS") == "1":  # diagnostic: the step without World.step (scenario nodes only)
    env.world.step = lambda: None
for _ in range(10):
    env.step(env.get_random_actions())
assert env.graph_status == "graph", env.graph_reason

stamps = {}
events = []


def stamp(name):
    stamps.setdefault(name, []).append(time.perf_counter())


def wrap(cls, meth, before, after):
    orig = getattr(cls, meth)

    def f(*a, **k):
        stamp(before)
        r = orig(*a, **k)
        stamp(after)
        return r

    setattr(cls, meth, f)


wrap(_graph.StepGraph, "before_actions", "before_actions0", "before_actions1")
wrap(Environment, "_apply_continuous_actions", "apply0", "apply1")
G = env._graph
orig_launch = _graph.StepGraph._launch


def launch(self, *a, **k):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    stamp("replay0")
    r = orig_launch(self, *a, **k)  # (a deferred kernel chain: launched later, by _post_replay)
    stamp("replay1")
    e1.record()
    events.append((e0, e1))
    return r


_graph.StepGraph._launch = launch
wrap(_graph.StepGraph, "_post_replay", "clone0", "clone1")
wrap(_graph.StepGraph, "_finish_deferred", "deferred0", "deferred1")

N = 100
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    stamp("draw0")
    a = env.get_random_actions()
    stamp("draw1")
    env.step(a)
    stamp("step1")
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / N * 1e6


def mean_us(a, b):
    if a not in stamps or b not in stamps:
        return float("nan")  # (the path did not run: e.g. pre-applied actions skip the action launch)
    return sum(y - x for x, y in zip(stamps[a], stamps[b])) / len(stamps[a]) * 1e6


gpu_graph = sum(e0.elapsed_time(e1) for e0, e1 in events) / len(events) * 1e3
out = {
    "scenario": scenario, "envs": n_envs, "wall_us_per_step": round(wall, 1),
    "host_us": {
        "draw_random_actions": round(mean_us("draw0", "draw1"), 1),
        "step_before_actions": round(mean_us("before_actions0", "before_actions1"), 1),
        "apply_actions_incl_wait": round(mean_us("apply0", "apply1"), 1),
        "graph_replay_launch": round(mean_us("replay0", "replay1"), 1),
        "post_replay_copies": round(mean_us("clone0", "clone1"), 1),
        "deferred_finish_incl_wait": round(mean_us("deferred0", "deferred1"), 1),
        "whole_step_call": round(mean_us("draw1", "step1"), 1),
    },
    "gpu_us": {"graph_replay": round(gpu_graph, 1)},
    "inplace_backed_up": [list(t.shape) for t in G._inplace],
    "speculative": bool(env._can_speculate()),
    "raw_graph_launch": G._raw_exec is not None,
}
print(json.dumps(out), flush=True)
