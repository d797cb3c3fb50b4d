"""cProfile of the bench loop (host-side cost of env.step on the GPU)."""
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
kw = {"n_agents": 4} if scenario != "discovery" else {"n_agents": 8, "use_agent_lidar": True}
import os  # noqa: E402

env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, graph_step=os.environ.get("GRAPH", "1") == "1", **kw)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
for _ in range(10):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(50):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
print(f"{scenario} {n_envs}: {(time.perf_counter() - t) / 50 * 1e3:.3f} ms/step")
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumtime").print_stats(40)
