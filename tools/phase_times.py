"""Host wall time per phase of env.step (no profiler overhead: perf_counter wrappers on the
phase functions), for the bench workload.  Usage: python tools/phase_times.py [scenario] [envs]"""
import functools
import sys
import time
from collections import defaultdict
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402
from vectorizedmultiagentsimulator_amd.simulator.environment import environment as envmod  # noqa: E402

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, n_agents=4)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10

acc = defaultdict(float)
cnt = defaultdict(int)


def wrap(obj, name, label):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[label] += time.perf_counter() - t
            cnt[label] += 1

    setattr(obj, name, g)


sc = env.scenario
for n in ("observation", "reward", "done", "info"):
    wrap(sc, n, "scenario." + n)
wrap(env, "_set_action", "env._set_action")
wrap(env, "_validate_continuous_actions", "env._validate_actions")
wrap(env.world, "step", "world.step")
wrap(env.world.engine, "step", "engine.step")
wrap(env.world.engine, "_query", "engine._query (distance)")
wrap(env, "_get_from_scenario", "env._get_from_scenario")
wrap(env, "_done", "env._done")

for _ in range(20):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
acc.clear()
cnt.clear()
K = 200
t_act = t_step = 0.0
for _ in range(K):
    t0 = time.perf_counter()
    a = env.get_random_actions()
    t1 = time.perf_counter()
    env.step(a)
    t2 = time.perf_counter()
    t_act += t1 - t0
    t_step += t2 - t1
torch.cuda.synchronize()
print(f"{scenario} {n_envs}: get_random_actions {t_act / K * 1e6:.1f} us, env.step {t_step / K * 1e6:.1f} us")
for k in sorted(acc, key=lambda k: -acc[k]):
    print(f"  {k:34s} {acc[k] / K * 1e6:8.1f} us/step  ({cnt[k] / K:.0f} calls)")
