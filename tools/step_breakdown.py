"""Per-step breakdown on the GPU: host cProfile of env.step + GPU kernel time per step (torch
profiler), for the bench workload (balance 32k, 10 substeps by default)."""
import cProfile
import pstats
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
n_agents = int(sys.argv[3]) if len(sys.argv) > 3 else (8 if scenario in ("discovery", "flocking") else 4)
kw = {"n_agents": n_agents}
if scenario == "discovery":
    kw["use_agent_lidar"] = True
import os  # noqa: E402

env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, graph_step=os.environ.get("GRAPH", "1") == "1", **kw)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
for _ in range(10):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(100):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
print(f"{scenario} {n_envs}: {(time.perf_counter() - t) / 100 * 1e3:.3f} ms/step, step mode {env.graph_status}")

from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(20):
        env.step(env.get_random_actions())
    torch.cuda.synchronize()
ka = prof.key_averages()
gpu_total = sum(e.self_device_time_total for e in ka) / 20
print(f"GPU kernel time per step (torch profiler): {gpu_total:.1f} us")
print(ka.table(sort_by="self_device_time_total", row_limit=25))

pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumtime").print_stats(30)
