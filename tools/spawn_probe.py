"""Probe: vmas_spawn_targets kernel time vs targets / min_dist (run under rocprofv3 --stats)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vectorizedmultiagentsimulator_amd.scenarios.discovery import respawn_targets_native

dev = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
for t, md in [(1, 0.0), (1, 0.2), (7, 0.0), (7, 0.2)]:
    torch.manual_seed(0)
    agents = torch.empty((B, 8, 2), device=dev).uniform_(-1, 1)
    tpos = [torch.empty((B, 2), device=dev).uniform_(-1, 1) for _ in range(t)]
    covered = torch.rand(B, t, device=dev) < 0.3
    for rep in range(20):
        mx = respawn_targets_native(agents, covered, md, 1.0, 1.0, *tpos)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for rep in range(20):
        mx = respawn_targets_native(agents, covered, md, 1.0, 1.0, *tpos)
    e.record()
    torch.cuda.synchronize()
    print(f"T={t} min_dist={md}: {s.elapsed_time(e) / 20 * 1e3:.1f} us/call (host incl.), words {mx.tolist()[:t + 1]}",
          flush=True)
