"""What a graph-mode step's post-replay launch moves (StepGraph._post_table): output clones, the
carry of re-bound state (Y -> X, with the attribute names), the next step's rollback backups, the
direct-output offset words; bytes per row kind.
usage: python tools/post_table_probe.py [scenario] [envs]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
kw = {"n_agents": 8 if scenario in ("discovery", "flocking") else 4}
if scenario == "discovery":
    kw["use_agent_lidar"] = True
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, **kw)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
for _ in range(8):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
g = env._graph
print(f"{scenario} {n_envs}: graph {env.graph_status} ({env.graph_reason})")
t = g._post_table()
tbl = t["tbl"]
n_out, n_all = t["n_out"], t["n_all"]
out_b = int(sum(int(r["nbytes"]) for r in tbl[:n_out] if int(r["nbytes"]) > 0))
rest = tbl[n_out:n_all]
n_bk = t["n_bk"]
carry_rows = rest[:len(rest) - n_bk] if n_bk else rest
bk_rows = rest[len(rest) - n_bk:] if n_bk else rest[:0]
print(f"rows: {n_out} output (+ direct words / step counter), {len(carry_rows)} carry, {len(bk_rows)} backup; plain={t['plain']}")
print(f"bytes: outputs {out_b / 1e6:.2f} MB, carry {sum(int(r['nbytes']) for r in carry_rows) / 1e6:.2f} MB, "
      f"backups {sum(int(r['nbytes']) for r in bk_rows) / 1e6:.2f} MB")
print("carried attributes:", getattr(g, "_carry_names", "?"))
from vectorizedmultiagentsimulator_amd.simulator.environment._graph import _own_scenario  # noqa: E402
print("own scenario:", _own_scenario(env.scenario), "; agent dynamics:",
      sorted({type(getattr(a, "dynamics", None)).__module__ + "." + type(getattr(a, "dynamics", None)).__name__
              for a in env.world.agents}), "; write-only ys:", len(g._write_only_ys))
print("in-place (backed up) tensors:", len(g._inplace), [tuple(x.shape) for x in g._inplace][:12])
print("direct categories:", len(g._direct.enabled) if g._direct is not None else 0,
      "; clone groups:", [(str(dt), tuple(sh), n) for dt, sh, n in g._clone_groups])
