"""Per-workgroup timeline of one k_world launch (VMAS_JIT_PROFILE builds): when each workgroup
started, claimed its group, finished it and left, relative to the first start (s_memrealtime,
100 MHz); where the launch's span goes beyond one workgroup's own work (dispatch spread, tail).
usage: python tools/kworld_wg_timeline.py [scenario] [envs]
"""
import os
import sys
from pathlib import Path

import numpy as np

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
os.environ["VMAS_JIT_PROFILE"] = "0"

import torch  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

kw = {"n_agents": 8 if scenario in ("discovery", "flocking") else 4}
if scenario == "discovery":
    kw["use_agent_lidar"] = True
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, graph_step=False, **kw)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
for _ in range(6):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
eng = env.world.engine
flat = eng.jit_profile().reshape(-1).astype(np.int64)
ms = eng._max_substeps
K_NW, K_REC = 16, 24
base = (ms * 4 + 2) * K_NW
nwg = (n_envs + 63) // 64
rec = flat[base: base + nwg * K_REC].reshape(nwg, K_REC)
ran = rec[:, 0] != 0
rec = rec[ran]
t0 = rec[:, 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731 (100 MHz s_memrealtime)
start, leave = us(rec[:, 0]), us(rec[:, 3])
g_start, g_end = us(rec[:, 4]), us(rec[:, 5])
c0, c1 = us(rec[:, 6]), us(rec[:, 7])  # around the first claim's compare-and-swap
xcc = rec[:, 2] & 0xF


def pct(v):
    q = np.percentile(v, [0, 10, 50, 90, 100])
    return " ".join(f"{x:7.2f}" for x in q)


print(f"{scenario} {n_envs} envs: {len(rec)} workgroups recorded (launch span {leave.max():.2f} us from first start)")
print("                      min     p10     p50     p90     max   (us)")
print(f"start              {pct(start)}")
print(f"claim CAS issued   {pct(c0)}")
print(f"claim CAS returned {pct(c1)}")
print(f"last group start   {pct(g_start)}")
print(f"last group end     {pct(g_end)}")
print(f"leave group loop   {pct(leave)}")
print(f"own span (leave - start) {pct(leave - start)}")
print(f"group work (end - start) {pct(g_end - g_start)}")
for x in sorted(set(xcc.tolist())):
    m = xcc == x
    print(f"  XCC {x}: {int(m.sum())} wg, start p50 {np.median(start[m]):.2f}, leave max {leave[m].max():.2f}")
