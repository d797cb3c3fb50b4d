"""Graph-mode diagnostics: step a graph_step env and print the capture status / reason."""
import sys
import traceback
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "balance"
env = make_env(name, num_envs=32768, device="cuda:0", seed=0, graph_step=True, n_agents=4)
env.world._substeps = 10
env.world._sub_dt = env.world._dt / 10
env.step(env.get_random_actions())
env.world.engine.set_timing(True)
for t in range(6):
    try:
        env.step(env.get_random_actions())
        torch.cuda.synchronize()
        print(t, "ok", env.graph_status, env.graph_reason, flush=True)
    except Exception:
        print(t, "FAILED", env.graph_status, env.graph_reason, flush=True)
        traceback.print_exc()
        break
eng = env.world.engine
eng.device_timing(reset=True)
import time
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"{1e3 * dt / 50:.3f} ms/step; device timer:", eng.device_timing(reset=True), env.graph_status, flush=True)
try:
    print("passes:", eng.last_iterations, "grid:", eng.jit_grid)
except Exception as ex:
    print("fixed point error:", ex)
