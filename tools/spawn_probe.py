"""Probe: vmas_spawn_targets per-item timeline (VMAS_SPAWN_PROFILE=1) vs targets / min_dist."""
import ctypes
import os
import sys

os.environ.setdefault("VMAS_SPAWN_PROFILE", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vectorizedmultiagentsimulator_amd import _native as N  # noqa: E402
from vectorizedmultiagentsimulator_amd.scenarios.discovery import respawn_targets_native  # noqa: E402

dev = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
lib = N.load_library()
lib.vmas_spawn_profile.restype = ctypes.c_int32
lib.vmas_spawn_profile.argtypes = [ctypes.c_void_p, ctypes.c_int64]
G = (B + 63) // 64
for t, md in [(1, 0.0), (7, 0.0), (7, 0.2)]:
    torch.manual_seed(0)
    agents = torch.empty((B, 8, 2), device=dev).uniform_(-1, 1)
    tpos = [torch.empty((B, 2), device=dev).uniform_(-1, 1) for _ in range(t)]
    covered = torch.rand(B, t, device=dev) < 0.3
    for rep in range(20):
        mx = respawn_targets_native(agents, covered, md, 1.0, 1.0, *tpos)
    torch.cuda.synchronize()
    buf = np.zeros(t * G * 6, dtype=np.uint64)
    n = lib.vmas_spawn_profile(buf.ctypes.data, buf.size)
    st = buf[:n].reshape(-1, 6).astype(np.int64)
    t0 = st[:, 0].min()
    rel = (st[:, :5] - t0) / 100.0  # s_memrealtime 100 MHz ticks -> us
    print(f"T={t} min_dist={md}: words {mx.tolist()[:t + 1]}, span {rel[:, 4].max():.1f} us", flush=True)
    for i in range(t):
        r = rel[i * G:(i + 1) * G]
        print(f"  target {i}: claimed {r[:, 0].min():7.1f}-{r[:, 0].max():7.1f}  wait over {r[:, 1].min():7.1f}-{r[:, 1].max():7.1f}"
              f"  loaded +{np.median(r[:, 2] - r[:, 1]):.2f}  tried +{np.median(r[:, 3] - r[:, 2]):.2f} (max {np.max(r[:, 3] - r[:, 2]):.2f})"
              f"  done +{np.median(r[:, 4] - r[:, 3]):.2f}  last done {r[:, 4].max():7.1f}", flush=True)
