"""Probe: vmas_spawn_targets timeline (VMAS_SPAWN_PROFILE=1) at discovery's C4 shape.

Windowed kernel (default): phase 1 from workgroup 0's start to the last group's table (arrivals),
the tables' reduction, the chain.  Per-target kernels (VMAS_SPAWN_KERNEL=resident): per-item
stamps per target.  usage: python tools/spawn_probe.py [B] [covered probability]"""
import ctypes
import os
import sys
import time

os.environ.setdefault("VMAS_SPAWN_PROFILE", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorizedmultiagentsimulator_amd import _native as N  # noqa: E402
from vectorizedmultiagentsimulator_amd.scenarios.discovery import respawn_targets_native  # noqa: E402

dev = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
cov_p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.001
window = os.environ.get("VMAS_SPAWN_KERNEL", "window") == "window"
lib = N.load_library()
G = (B + 63) // 64
for t, md in [(1, 0.2), (7, 0.2)]:
    torch.manual_seed(0)
    agents = torch.empty((B, 8, 2), device=dev).uniform_(-1, 1)
    tpos = [torch.empty((B, 2), device=dev).uniform_(-1, 1) for _ in range(t)]
    covered = torch.rand(B, t, device=dev) < cov_p
    # one words buffer across the calls, as a graph's spawn channel keeps it (the windowed kernels
    # size each call's window from the previous call's consumption)
    mx = torch.zeros(N.spawn_words(t), dtype=torch.int32, device=dev)
    for rep in range(20):
        respawn_targets_native(agents, covered, md, 1.0, 1.0, *tpos, out=mx)
    torch.cuda.synchronize()
    # wall time per call (the call's one host read included)
    t0 = time.perf_counter()
    for rep in range(50):
        respawn_targets_native(agents, covered, md, 1.0, 1.0, *tpos, out=mx)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 50 * 1e6
    words = mx.tolist()
    n = max(t * G * 6, 8 + G)
    buf = np.zeros(n, dtype=np.uint64)
    got = lib.vmas_spawn_profile(buf.ctypes.data, buf.size)
    print(f"T={t} min_dist={md} cov={cov_p}: maxima {words[:t]} unresolved {words[t]} listed {words[33]}"
          f" window next {words[38]}"
          f" call {wall:.1f} us (host read included)", flush=True)
    if window:
        st = buf[:32 + G].astype(np.int64)
        us = lambda a, b: (st[b] - st[a]) / 100.0  # noqa: E731
        ends = (st[32:32 + G] - st[0]) / 100.0
        print(f"  cands: group 0 drew its pairs in {us(0, 30):.2f} us; groups done {ends.min():.2f}-{ends.max():.2f}"
              f" (median {np.median(ends):.2f}) | chain starts +{(st[1] - st[0]) / 100.0 - ends.max():.2f}:"
              f" rows + list {us(1, 2):.2f}, clean chain + listed candidates {us(2, 3):.2f},"
              f" listed walks + check {us(3, 4):.2f}, rebuild from target {st[6]} + writes {us(4, 5):.2f}"
              f" | span {us(0, 5):.2f} us", flush=True)
    else:
        st = buf[:t * G * 6].reshape(-1, 6).astype(np.int64)
        t0 = st[:, 0].min()
        rel = (st[:, :5] - t0) / 100.0  # s_memrealtime 100 MHz ticks -> us
        print(f"  span {rel[:, 4].max():.1f} us", flush=True)
        for i in range(t):
            r = rel[i * G:(i + 1) * G]
            print(f"  target {i}: wait over {r[:, 1].min():7.1f}-{r[:, 1].max():7.1f}"
                  f"  tried +{np.median(r[:, 3] - r[:, 2]):.2f} (max {np.max(r[:, 3] - r[:, 2]):.2f})"
                  f"  last done {r[:, 4].max():7.1f}", flush=True)
