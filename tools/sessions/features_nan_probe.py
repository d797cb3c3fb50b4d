"""Relaxed-math NaN in the features world (VMAS_JIT_PRM_MASK=0x2): teacher-force the failing step
with 1..S substeps and the force export on, print the first entity / substep going non-finite."""
import sys

import torch

sys.path.insert(0, ".")
from oracle import vmas_oracle as O  # noqa: E402
from tests._parity import make  # noqa: E402

env = make("features", dict(n_agents=8), None, "cuda:0", num_envs=16384, seed=0)
env.step(env.get_random_actions())
env.step(env.get_random_actions())
w = env.world
snap = O.snapshot(w)
w.export_forces = True
S = w._substeps
for sub in range(1, S + 1):
    O.load_snapshot(w, snap)
    w._substeps = sub
    w.step()
    got = O.snapshot(w)
    bad = torch.zeros(w.batch_dim, dtype=torch.bool)
    for i in got:
        for k, v in got[i].items():
            bad |= ~torch.isfinite(v).reshape(v.shape[0], -1).all(-1)
    print("substeps", sub, "non-finite envs", int(bad.sum()), bad.nonzero().flatten()[:8].tolist())
    if bad.any():
        j = int(bad.nonzero()[0, 0])
        for i, e in enumerate(w.entities):
            f = w.forces_dict[e][j].tolist()
            t = w.torques_dict[e][j].tolist()
            print(f"  {e.name}: in pos {snap[i]['pos'][j].tolist()} rot {snap[i]['rot'][j].tolist()} vel {snap[i]['vel'][j].tolist()} "
                  f"angv {snap[i]['ang_vel'][j].tolist()} | out pos {got[i]['pos'][j].tolist()} angv {got[i]['ang_vel'][j].tolist()} "
                  f"| F {f} T {t}")
        break
w._substeps = S
