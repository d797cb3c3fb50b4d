"""Probe: the phases of discovery's windowed respawn (k_spawn_cands + k_spawn_chain) inside the C4
workload (16 384 envs, 8 agents, agent LIDAR), graph mode, from the VMAS_SPAWN_PROFILE=1 stamps
(s_memrealtime, 100 MHz) of the last launch: group 0's draw / sweep / table phases, every group's
start and end, the chain kernel's stamps (csrc/vmas_spawn.hip, k_spawn_cands / k_spawn_chain)."""
import ctypes
import os
import sys

os.environ.setdefault("VMAS_SPAWN_PROFILE", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorizedmultiagentsimulator_amd import _native as N  # noqa: E402
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
lib = N.load_library()
G = (B + 63) // 64
env = make_env("discovery", num_envs=B, device="cuda:0", seed=0, n_agents=8, use_agent_lidar=True)
t = len(env.scenario._targets)
buf = np.zeros(max(t * G * 6, 32 + 2 * G), dtype=np.uint64)
rows = []
for k in range(40):
    env.step(env.get_random_actions())
    torch.cuda.synchronize()
    if k < 8:
        continue
    n = lib.vmas_spawn_profile(buf.ctypes.data, buf.size)
    assert n == buf.size, n
    s = buf.astype(np.int64)
    t0 = s[0]
    start = (s[32 + G:32 + 2 * G] - t0) / 100.0
    end = (s[32:32 + G] - t0) / 100.0
    chain = (s[1:6] - t0) / 100.0
    rows.append([(s[30] - t0) / 100.0, (s[31] - t0) / 100.0, (s[29] - t0) / 100.0, end[0], start.max(),
                 np.median(end), end.max(), *chain])
r = np.median(np.array(rows), axis=0)
print(f"status {env.graph_status}; median over {len(rows)} steps, us from group 0's start:")
print(f"  group 0: pairs drawn + tested {r[0]:.2f}, sweep {r[1]:.2f}, table stored + counted {r[2]:.2f}, done {r[3]:.2f}")
print(f"  groups: last start {r[4]:.2f}, median end {r[5]:.2f}, last end {r[6]:.2f}")
print(f"  chain: start {r[7]:.2f}, reduced {r[8]:.2f}, clean chain {r[9]:.2f}, list {r[10]:.2f}, end {r[11]:.2f}")
