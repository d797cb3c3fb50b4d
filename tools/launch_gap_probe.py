"""Is the idle gap after a replayed step graph a host-issue delay or a graph -> stream transition?

1. A one-kernel graph (x += 1 over 32 768 floats) replayed back to back: (a) alone, (b) followed by
   the same kernel launched on the stream, (c) followed by a second one-kernel graph, (d) alone
   but launched through vmas_graph_launch (the product's raw launch).  HIP events around 500
   iterations: us per iteration.  (b) - (a) - one kernel = the transition cost.
2. The bench step (make_env + env.step(env.get_random_actions())): the host's issue time of K
   steps (perf_counter, no sync) vs the wall time to the final synchronize.  Issue ~ wall: the
   step is host-bound.
usage: python tools/launch_gap_probe.py [scenario] [envs]
"""
import ctypes
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402
from vectorizedmultiagentsimulator_amd import _native as N  # noqa: E402

dev = torch.device("cuda:0")
res = {}


def timed(fn, n=500):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    t1 = time.perf_counter()
    e1.synchronize()
    t2 = time.perf_counter()
    return {"gpu_us": round(1e3 * e0.elapsed_time(e1) / n, 2), "issue_us": round(1e6 * (t1 - t0) / n, 2),
            "wall_us": round(1e6 * (t2 - t0) / n, 2)}


s = torch.cuda.Stream()
x = torch.zeros(32768, device=dev)
y = torch.zeros(32768, device=dev)
with torch.cuda.stream(s):
    for _ in range(3):
        x.add_(1)
        y.add_(1)
    torch.cuda.synchronize()
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, stream=s):
        x.add_(1)
    with torch.cuda.graph(g2, stream=s):
        y.add_(1)
    torch.cuda.synchronize()
    res["stream_kernel_only"] = timed(lambda: y.add_(1))
    res["graph_only"] = timed(g1.replay)
    res["graph_then_stream_kernel"] = timed(lambda: (g1.replay(), y.add_(1)))
    res["graph_then_graph"] = timed(lambda: (g1.replay(), g2.replay()))
    lib = N.load_library()
    raw = ctypes.c_void_p(g1.raw_cuda_graph_exec())
    sp = ctypes.c_void_p(s.cuda_stream)
    res["raw_graph_only"] = timed(lambda: lib.vmas_graph_launch(raw, sp))
    res["raw_graph_then_stream_kernel"] = timed(lambda: (lib.vmas_graph_launch(raw, sp), y.add_(1)))
print(json.dumps({"probe": "transition", **res}), flush=True)

# GPU-bound variant: a ~25 us kernel (16 M floats scaled in place) in the graph, a small kernel
# after it on the stream vs inside the same graph.  (graph+stream) - (graph with both) = the
# GPU-side cost of the graph -> stream transition.
h = torch.ones(1 << 24, device=dev)
res = {}
with torch.cuda.stream(s):
    heavy = lambda: h.mul_(1.0000001)  # noqa: E731
    small = lambda: y.add_(1)  # noqa: E731
    for _ in range(3):
        heavy()
        small()
    torch.cuda.synchronize()
    gh, gb, gs = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gh, stream=s):
        heavy()
    with torch.cuda.graph(gb, stream=s):
        heavy()
        small()
    with torch.cuda.graph(gs, stream=s):
        small()
    torch.cuda.synchronize()
    res["heavy_stream"] = timed(heavy, 300)
    res["heavy_small_stream"] = timed(lambda: (heavy(), small()), 300)
    res["graph_heavy"] = timed(gh.replay, 300)
    res["graph_both"] = timed(gb.replay, 300)
    res["graph_heavy_then_stream_small"] = timed(lambda: (gh.replay(), small()), 300)
    res["graph_heavy_then_graph_small"] = timed(lambda: (gh.replay(), gs.replay()), 300)
    res["stream_small_then_graph_heavy"] = timed(lambda: (small(), gh.replay()), 300)
print(json.dumps({"probe": "transition_gpu_bound", **res}), flush=True)

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
kw = {"n_agents": 8 if scenario in ("discovery", "flocking") else 4}
if scenario == "discovery":
    kw["use_agent_lidar"] = True
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, **kw)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
for _ in range(20):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
out = {"probe": "step", "scenario": scenario, "envs": n_envs, "graph_status": env.graph_status}
for K in (50, 200):
    out[f"K{K}"] = timed(lambda: env.step(env.get_random_actions()), n=K)
print(json.dumps(out), flush=True)
