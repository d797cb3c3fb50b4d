"""Host-side profile of graph-mode steps (cProfile over `env.step(env.get_random_actions())`): which
Python / native calls the host spends a step's wall time in when the step is host-bound.
Usage: python tools/host_profile.py [scenario] [envs] [steps] [graph|eager]
(eager: the reference API's default path, make_env without graph_step)
"""
import cProfile
import pstats
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

scenario = sys.argv[1] if len(sys.argv) > 1 else "discovery"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 300
mode = sys.argv[4] if len(sys.argv) > 4 else "graph"
kw = {"n_agents": 8, "use_agent_lidar": True} if scenario == "discovery" else {}  # (bench.py's C4)
if scenario == "balance":
    kw = {"n_agents": 4}
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, graph_step=mode == "graph", **kw)
if scenario == "balance":  # C2: 10 substeps
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
for _ in range(10):
    env.step(env.get_random_actions())
if mode == "graph":
    assert env.graph_status == "graph", env.graph_reason
torch.cuda.synchronize()


def run():
    for _ in range(steps):
        env.step(env.get_random_actions())
    torch.cuda.synchronize()


pr = cProfile.Profile()
pr.enable()
run()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(40)
