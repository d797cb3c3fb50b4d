"""Per-wave phase timing of the world-specialised step kernel (k_world) inside one workgroup.

Sets VMAS_JIT_PROFILE=<block> so the generated kernel stamps s_memtime at every phase boundary
of that workgroup, runs a few steps of the bench workload and prints, per wave and averaged over
the substeps of the last launch: pair-phase busy cycles, barrier wait after it, entity-phase busy
cycles, barrier wait after it.
usage: python tools/jit_phase_profile.py [scenario] [envs] [block]
"""
import os
import sys
from pathlib import Path

import numpy as np

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
block = int(sys.argv[3]) if len(sys.argv) > 3 else 200
os.environ["VMAS_JIT_PROFILE"] = str(block)

import torch  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

kw = {"n_agents": 8 if scenario in ("discovery", "flocking") else 4}
if scenario == "discovery":
    kw["use_agent_lidar"] = True
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, **kw)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
for _ in range(5):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
eng = env.world.engine
print("kernel:", eng.kernel_name, eng.jit_error or "")
t = eng.jit_profile().astype(np.int64)  # [max_substeps*4 + 2, 16]
S = env.world._substeps
ms = eng._max_substeps
nw = int((t[ms * 4 + 1] != 0).sum())  # waves that stamped the prologue release
t = t[:, :nw]
pro_done, pro_rel = t[ms * 4], t[ms * 4 + 1]
st = t[: S * 4].reshape(S, 4, nw)
start = np.concatenate([pro_rel[None], st[:-1, 3]], 0)  # each substep starts at the previous release
pair = (st[:, 0] - start).mean(0)
wait1 = (st[:, 1] - st[:, 0]).mean(0)
ent = (st[:, 2] - st[:, 1]).mean(0)
wait2 = (st[:, 3] - st[:, 2]).mean(0)
print(f"prologue: busy {(pro_done - pro_done.min()).tolist()} release at {int(pro_rel.max() - pro_done.min())}")
print("wave | pair busy | wait | entity busy | wait   (cycles per substep, mean over substeps)")
for w in range(nw):
    print(f"{w:4d} | {pair[w]:9.0f} | {wait1[w]:6.0f} | {ent[w]:11.0f} | {wait2[w]:6.0f}")
per_sub = (st[-1, 3].max() - pro_rel.min()) / S
print(f"substep period {per_sub:.0f} cycles; pair makespan {pair.max():.0f}, entity makespan {ent.max():.0f}")
print("source wave assignment:")
src = eng.jit_source()
for line in src.splitlines():
    if line.startswith("template <> __device__") or "// pair " in line or "// entity " in line:
        print("  ", line.strip()[:100])
