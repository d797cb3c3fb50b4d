"""Features world at full size: parity of one teacher-forced step, per entity / field worst env
(bisecting a GPU parity failure).  python tools/features_probe.py [envs]"""
import sys

import torch

sys.path.insert(0, ".")
from oracle import vmas_oracle as O  # noqa: E402
from tests._parity import make  # noqa: E402

envs = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
env = make("features", dict(n_agents=8), None, "cuda:0", num_envs=envs, seed=0)
for step in range(2):
    env.step(env.get_random_actions())
    w = env.world
    snap = O.snapshot(w)
    exp, ow = O.oracle_step(w, snap)
    w.step()
    got = O.snapshot(w)
    print("step", step, "kernel", w.engine.kernel_name, "export", w.export_forces)
    for i, e in enumerate(w.entities):
        for k in got[i]:
            d = (got[i][k] - exp[i][k]).abs()
            bad = ~torch.isfinite(got[i][k]).all(-1) | (d > 1e-3).any(-1)
            if bad.any():
                j = int(bad.nonzero()[0, 0])
                print(f"  {e.name} {k}: {int(bad.sum())} envs, env {j}: got {got[i][k][j].tolist()} exp {exp[i][k][j].tolist()} "
                      f"in {snap[i][k][j].tolist()} margin {float(ow.cutoff_margin[j]):.3g}")
