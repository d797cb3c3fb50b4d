"""Host-side cost of env.step(env.get_random_actions()) on the GPU: wall per step, GPU-synchronised
per step, and a cProfile of the steady state (python tools/host_profile.py SCENARIO ENVS [N_AGENTS])."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "flocking"
envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
preset = dict(bench.PRESETS[name])
kw = dict(preset.get("kw", {}))
if len(sys.argv) > 3:
    kw["n_agents"] = int(sys.argv[3])
elif "n_agents" in preset:
    kw["n_agents"] = preset["n_agents"]
env = make_env(name, num_envs=envs, device="cuda:0", seed=0, graph_step=os.environ.get("GRAPH", "1") == "1", **kw)
for _ in range(30):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
n = 200
t0 = time.perf_counter()
for _ in range(n):
    env.step(env.get_random_actions())
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"{name} {envs}: host {1e6 * (t1 - t0) / n:.1f} us/step issued, {1e6 * (t2 - t0) / n:.1f} us/step with the GPU drained",
      flush=True)
t0 = time.perf_counter()
for _ in range(n):
    a = env.get_random_actions()
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"get_random_actions alone: {1e6 * (t1 - t0) / n:.1f} us", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    env.step(env.get_random_actions())
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
