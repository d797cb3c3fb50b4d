"""Time the flocking fused program's launch variants (what = REWARD|OBS, OBS, REWARD; exact vs
fast LIDAR) with HIP events over repeated launches on a 32 768-env, 8-agent world."""
import sys

import torch

sys.path.insert(0, ".")
from vectorizedmultiagentsimulator_amd import _native as N  # noqa: E402
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402
from vectorizedmultiagentsimulator_amd.simulator import _fused  # noqa: E402

env = make_env("flocking", num_envs=32768, device="cuda:0", seed=0, n_agents=8)
for _ in range(3):
    env.step(env.get_random_actions())
sc = env.scenario
for exact in (False, True):
    _fused.EXACT_LIDAR = exact
    for name, what in (("rew+obs", N.VMAS_SCN_REWARD | N.VMAS_SCN_OBS), ("obs", N.VMAS_SCN_OBS),
                       ("rew", N.VMAS_SCN_REWARD)):
        for _ in range(3):
            sc._run_fused(what)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        n = 50
        for _ in range(n):
            sc._run_fused(what)
        e1.record()
        e1.synchronize()
        print(f"exact={exact} {name}: {e0.elapsed_time(e1) / n * 1e3:.1f} us per launch (incl. host gaps)", flush=True)
