"""Which outputs of a captured step lie inside a carry destination (the post-replay launch is then
split in two, _graph._post_replay's "clash"): output index / shape / dtype against the carry spans.
usage: python tools/clash_probe.py [scenario] [envs] [n_agents]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "flocking"
envs = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
na = int(sys.argv[3]) if len(sys.argv) > 3 else 8
env = make_env(name, num_envs=envs, device="cuda:0", seed=0, graph_step=True, n_agents=na)
for _ in range(5):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
g = env._graph
t = g._post_table()
print("status", env.graph_status, "clash", t["clash"], "plain", t["plain"], "n_out", t["n_out"], "n_all", t["n_all"])
carry = [(y.data_ptr(), x.data_ptr(), x.numel()) for x, y in zip(g._carry_dst, g._carry_src)]
for i, o in enumerate(g._out_tensors):
    lo, nb = o.data_ptr(), o.numel() * o.element_size()
    for y, x, cn in carry:
        if lo < x + cn and x < lo + nb:
            print(f"output {i} {tuple(o.shape)} {o.dtype} @{lo:#x}+{nb} inside carry X @{x:#x}+{cn}")
print("carry spans", [(hex(x), cn) for _, x, cn in carry])
