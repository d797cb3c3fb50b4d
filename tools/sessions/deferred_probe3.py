"""Probe: test_fused's discovery sequence (graph mode, cloned actions) without extra syncs; when a
step fails, decode the 64-bit value found in the spawn channel's words and name every live CUDA
tensor whose storage contains that address or the channel words' address."""
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

envs = int(sys.argv[1]) if len(sys.argv) > 1 else 777
env = make_env("discovery", num_envs=envs, device="cuda:0", seed=3, graph_step=True, n_agents=5, use_agent_lidar=True)
if os.environ.get("PROBE_SPEC", "1") == "0":
    env._SPECULATE = False


def owners(addr):
    hits = []
    for o in gc.get_objects():
        try:
            if isinstance(o, torch.Tensor) and o.is_cuda:
                st = o.untyped_storage()
                lo = st.data_ptr()
                if lo <= addr < lo + st.nbytes():
                    hits.append((tuple(o.shape), str(o.dtype), hex(o.data_ptr()), hex(lo), st.nbytes()))
        except Exception:  # noqa: BLE001
            pass
    return hits


for t in range(14):
    try:
        acts = [a.clone() for a in env.get_random_actions()]
        env.step(acts)
        print(f"step {t}: ok ({env.graph_status})", flush=True)
    except Exception as ex:  # noqa: BLE001
        print(f"step {t}: {type(ex).__name__}: {ex}", flush=True)
        torch.cuda.synchronize()
        ch = env.scenario._spawn_channel
        w = ch.mx.view(torch.int64).tolist()
        vals = sorted(set(w))
        print("channel words @", hex(ch.mx.data_ptr()), "distinct u64 values:", [hex(v & (2**64 - 1)) for v in vals[:8]], flush=True)
        print("first 16 u64:", [hex(v & (2**64 - 1)) for v in w[:16]], flush=True)
        for v in vals[:4]:
            v &= 2**64 - 1
            if v > 1 << 32:
                print(f"owners of {v:#x}:", owners(v)[:6], flush=True)
        print("owners of the channel words:", owners(ch.mx.data_ptr())[:6], flush=True)
        g = env._graph
        print("graph raw exec", g._raw_exec, "replays", g.replays, flush=True)
        raise
print("no failure")
