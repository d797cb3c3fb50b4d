"""Probe: the per-item timeline of discovery's target respawn launch inside the C4 workload
(16 384 envs, 8 agents, agent LIDAR), eager and graph mode (VMAS_SPAWN_PROFILE=1 stamps of the
last launch; see tools/spawn_probe.py for the columns)."""
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
lib.vmas_spawn_profile.restype = ctypes.c_int32
lib.vmas_spawn_profile.argtypes = [ctypes.c_void_p, ctypes.c_int64]
G = (B + 63) // 64
for graph in (False, True):
    env = make_env("discovery", num_envs=B, device="cuda:0", seed=0, graph_step=graph, n_agents=8, use_agent_lidar=True)
    for _ in range(8):
        env.step(env.get_random_actions())
    torch.cuda.synchronize()
    t = len(env.scenario._targets)
    buf = np.zeros(t * G * 6, dtype=np.uint64)
    n = lib.vmas_spawn_profile(buf.ctypes.data, buf.size)
    st = buf[:n].reshape(-1, 6).astype(np.int64)
    t0 = st[:, 0].min()
    rel = (st[:, :5] - t0) / 100.0
    print(f"graph={graph} T={t} min_dist={env.scenario._min_dist_between_entities}: span {rel[:, 4].max():.1f} us "
          f"(status {env.graph_status})", flush=True)
    for i in range(t):
        r = rel[i * G:(i + 1) * G]
        print(f"  target {i}: start {r[:, 0].min():7.1f}-{r[:, 0].max():7.1f}  wait over {r[:, 1].min():7.1f}-{r[:, 1].max():7.1f}"
              f"  tried +{np.median(r[:, 3] - r[:, 2]):.2f} (max {np.max(r[:, 3] - r[:, 2]):.2f})"
              f"  done +{np.median(r[:, 4] - r[:, 3]):.2f}  last done {r[:, 4].max():7.1f}", flush=True)
    del env
