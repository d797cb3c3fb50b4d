"""k_world diagnostics on the bench workload: fixed-point passes per step, per-launch event time,
and (with VMAS_JIT_PROFILE=<block>) the profiled workgroup's cycle span, whose ratio to the event
time is the effective shader clock.
usage: python tools/kworld_probe.py [scenario] [envs] [broadphase]
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
bp = sys.argv[3] if len(sys.argv) > 3 else "batch"
kw = {"n_agents": 8 if scenario in ("discovery", "flocking") else 4}
if scenario == "discovery":
    kw["use_agent_lidar"] = True
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, **kw)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
env.world.broadphase = bp
eng = env.world.engine
for _ in range(5):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
print("kernel:", eng.kernel_name, "grid:", eng.jit_grid, eng.jit_error or "")
passes = []
eng.set_timing(True)
eng.get_timing(reset=True)
for _ in range(30):
    env.step(env.get_random_actions())
    passes.append(eng.last_iterations)
ms, n = eng.get_timing(reset=True)
print(f"passes per step: {np.bincount(passes).tolist()} (index = passes)")
print(f"event time per launch: {1e3 * ms / max(n, 1):.2f} us over {n} launches")
if os.environ.get("VMAS_JIT_PROFILE"):
    t = eng.jit_profile().astype(np.int64)
    ms_sub = eng._max_substeps
    S = env.world._substeps
    nw = int((t[ms_sub * 4 + 1] != 0).sum())
    t = t[:, :nw]
    span = t[S * 4 - 1].max() - t[ms_sub * 4].min()
    print(f"profiled workgroup: {span} cycles from prologue end to last release; "
          f"{span / (1e3 * ms / max(n, 1)) / 1e3:.2f} GHz at the event time")
