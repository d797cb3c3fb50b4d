"""k_world diagnostics on the bench workload: fixed-point passes per step, per-launch event time,
and (with VMAS_JIT_PROFILE=<block>) the profiled workgroup's cycle span, whose ratio to the event
time is the effective shader clock.
usage: python tools/kworld_probe.py [scenario] [envs] [broadphase]
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vectorizedmultiagentsimulator_amd import make_env  # noqa: E402

scenario = sys.argv[1] if len(sys.argv) > 1 else "balance"
n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
bp = sys.argv[3] if len(sys.argv) > 3 else "batch"
kw = {"n_agents": 8 if scenario in ("discovery", "flocking") else 4}
if scenario == "discovery":
    kw["use_agent_lidar"] = True
env = make_env(scenario, num_envs=n_envs, device="cuda:0", seed=0, **kw)
if scenario == "balance":
    env.world._substeps = 10
    env.world._sub_dt = env.world._dt / 10
env.world.broadphase = bp
eng = env.world.engine
for _ in range(5):
    env.step(env.get_random_actions())
torch.cuda.synchronize()
print("kernel:", eng.kernel_name, "grid:", eng.jit_grid, eng.jit_error or "")
passes = []
eng.set_timing(True)
eng.get_timing(reset=True)
for _ in range(30):
    env.step(env.get_random_actions())
    passes.append(eng.last_iterations)
ms, n = eng.get_timing(reset=True)
print(f"passes per step: {np.bincount(passes).tolist()} (index = passes)")
print(f"event time per launch: {1e3 * ms / max(n, 1):.2f} us over {n} launches")
if os.environ.get("VMAS_JIT_PROFILE"):
    t = eng.jit_profile().astype(np.int64)
    ms_sub = eng._max_substeps
    S = env.world._substeps
    nw = int((t[ms_sub * 4 + 1] != 0).sum())
    t = t[:, :nw]
    span = t[S * 4 - 1].max() - t[ms_sub * 4].min()
    print(f"profiled workgroup: {span} cycles from prologue end to last release; "
          f"{span / (1e3 * ms / max(n, 1)) / 1e3:.2f} GHz at the event time")
    # per-workgroup records (start / group start / group end / leave, s_memrealtime; HW_ID, XCC_ID)
    base = (ms_sub * 4 + 2) * 16
    rec = t_full = eng.jit_profile().astype(np.int64)
    blk = t_full.reshape(-1)[base:].reshape(-1, 24)
    G = abs(eng.jit_grid)
    blk = blk[:G]
    t0 = blk[:, 0].min()
    mhz = 100.0  # s_memrealtime ticks at 100 MHz
    start, gs, ge, leave = [(blk[:, k] - t0) / mhz for k in (0, 4, 5, 3)]
    hw, xcc = blk[:, 1], blk[:, 2]
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    print(f"workgroups {G}: start spread {start.min():.2f}-{start.max():.2f} us; group time "
          f"{np.percentile(ge - gs, [0, 50, 100]).round(2).tolist()} us; leave {leave.min():.2f}-{leave.max():.2f} us")
    keys = xcc * 1000 + se * 100 + cu
    _, counts = np.unique(keys, return_counts=True)
    print(f"distinct (xcc, se, cu): {len(counts)}; workgroups per CU histogram: {np.bincount(counts).tolist()}")
    order = np.argsort(start)
    print("start times (us) by decile:", np.percentile(start, [0, 10, 25, 50, 75, 90, 100]).round(2).tolist())
    print("group start (us) deciles:", np.percentile(gs, [0, 10, 25, 50, 75, 90, 100]).round(2).tolist())
    print("group end (us) deciles:", np.percentile(ge, [0, 10, 25, 50, 75, 90, 100]).round(2).tolist())
    gt = ge - gs
    c0, c1 = [(blk[:, k] - t0) / mhz for k in (6, 7)]
    print("claim CAS (us) deciles:", np.percentile(c1 - c0, [0, 10, 50, 90, 100]).round(2).tolist(),
          "; start -> claim issue:", np.percentile(c0 - start, [0, 50, 100]).round(2).tolist(),
          "; claim done -> group start:", np.percentile(gs - c1, [0, 50, 100]).round(2).tolist())
    for x in np.unique(xcc):
        m = xcc == x
        print(f"  xcc {x}: {int(m.sum())} workgroups, group time mean {gt[m].mean():.2f} max {gt[m].max():.2f} us, "
              f"group start mean {gs[m].mean():.2f} us")
    slow = np.argsort(gt)[-8:]
    print("slowest groups (block, start, time):", [(int(i), round(float(gs[i]), 2), round(float(gt[i]), 2)) for i in slow])
    # the two workgroups sharing a CU: their group times
    pair_t = {}
    for i, k in enumerate(keys):
        pair_t.setdefault(int(k), []).append(float(gt[i]))
    both = np.array([sorted(v) for v in pair_t.values() if len(v) == 2])
    if len(both):
        print(f"CU pairs: faster member mean {both[:, 0].mean():.2f}, slower member mean {both[:, 1].mean():.2f} us")
    simd = (blk[:, 8:16] >> 4) & 3
    print("SIMD of waves 0-7, first 4 workgroups:", simd[:4].tolist())
    cnt = {}
    for row in simd:
        cnt[tuple(row.tolist())] = cnt.get(tuple(row.tolist()), 0) + 1
    print("wave->SIMD patterns:", sorted(cnt.items(), key=lambda x: -x[1])[:4])
