"""Host cost of the pieces of a graph-mode step, each called alone in a loop (µs per call):
the random-action draw, before_actions, the speculative action launch, the raw graph launch and
the post-replay copies.  GPU work they enqueue runs meanwhile; the stream is synchronised every
50 calls so that the queue stays short.
usage: python tools/host_micro.py [scenario] [envs]"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, n_agents=4, graph_step=True)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
for _ in range(12):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
G = env._graph
assert G.graph is not None, G.why


def bench(name, fn, n=400):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t = 0.0
    for i in range(n):
        t0 = time.perf_counter()
        fn()
        t += time.perf_counter() - t0
        if i % 50 == 49:
            torch.cuda.synchronize()
    print(f"{name:34s} {t / n * 1e6:8.1f} us")


acts = env.get_random_actions()
bench("get_random_actions", env.get_random_actions)
bench("before_actions", G.before_actions)
bench("apply (speculative launch)", lambda: env._apply_continuous_actions(acts, persistent=True, speculative=True))
bench("graph launch (raw)", G._launch)
bench("post_replay", G._post_replay)
bench("check_device_errors", env.world.engine.check_device_errors)
bench("_still_valid", G._still_valid)
bench("current_stream", lambda: torch.cuda.current_stream(0))
bench("torch.empty (4096,16)", lambda: torch.empty((4, 32768, 16), device="cuda:0"))
bench("whole step", lambda: env.step(env.get_random_actions()), n=200)
