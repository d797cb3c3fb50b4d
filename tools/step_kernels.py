"""Which Python call issues each GPU kernel / copy of one bench step: torch.profiler over a few
graph-mode steps of a bench config, every device event attributed to the innermost frame of this
package (or bench.py) on its launching op's stack.
usage: python tools/step_kernels.py [scenario] [envs] [n_agents]
"""
import sys
from collections import defaultdict
from pathlib import Path

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
n_agents = int(sys.argv[3]) if len(sys.argv) > 3 else 4
import os  # noqa: E402

graph = os.environ.get("STEP_GRAPH", "1") != "0"  # STEP_GRAPH=0: the eager step (the graph's body)
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, n_agents=n_agents, graph_step=graph)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
for _ in range(10):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
print("graph status:", env.graph_status, env.graph_reason)
steps = 5
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for _ in range(steps):
        env.step(env.get_random_actions())
    torch.cuda.synchronize()
agg = defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    if ev.device_type != torch.autograd.DeviceType.CUDA:
        continue
    frame = "?"
    parent = ev.cpu_parent if hasattr(ev, "cpu_parent") else None
    node = parent
    while node is not None:
        st = [s for s in (node.stack or []) if "vectorizedmultiagentsimulator_amd" in s or "bench.py" in s]
        if st:
            frame = st[0].split("/")[-1][:90]
            break
        node = node.cpu_parent
    key = (ev.name[:60], frame)
    agg[key][0] += 1
    agg[key][1] += ev.device_time_total if hasattr(ev, "device_time_total") else ev.cuda_time_total
for (name, frame), (n, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{n / steps:5.1f}/step {us / max(n, 1):8.2f} us  {name:60s}  {frame}")
