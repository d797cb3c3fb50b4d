"""Shared parity drivers: native engine (host backend or gfx950 kernels) vs the CPU oracle."""
from __future__ import annotations

import torch

from oracle import vmas_oracle as O
from vectorizedmultiagentsimulator_amd import make_env

# (scenario, kwargs, substeps override) -- every narrowphase class, joints and LIDAR types occur
SCENARIOS = [
    ("balance", dict(n_agents=4), 10),       # S-S, L-S, B-S, B-L, world gravity, y semidim
    ("transport", dict(n_agents=4), None),   # B-S, S-S, heavy box, semidims
    ("discovery", dict(n_agents=4, use_agent_lidar=True), None),  # S-S, 2 LIDARs
    ("flocking", dict(n_agents=4), None),    # S-S, scripted agent, LIDAR on obstacles
    ("pollock", dict(n_agents=4, n_lines=3, n_boxes=3, lidar=True), None),  # all 6 classes + box/line rays
    ("waterfall", dict(n_agents=5), None),   # joints (rotate / fixed rotation), L-L, B-L, B-B
    # friction (world + entity), force/torque clamps, max_speed / v_range, [B,2] entity gravity,
    # hollow + solid boxes vs spheres / lines / boxes, dim_c > 0 (scenarios/debug/features.py)
    ("features", dict(n_agents=4), None),
]


def make(name, kw, substeps, device, num_envs, seed):
    env = make_env(name, num_envs=num_envs, device=device, seed=seed, **kw)
    if substeps is not None:
        env.world._substeps = substeps
        env.world._sub_dt = env.world._dt / substeps
    return env


def step_parity(env, n_steps, broadphase="batch", max_bad_frac=0.0, certify=True):
    """Free-run the engine on random actions; after each step compare one teacher-forced step.
    certify=False: no cut-off certification (every env outside the tolerance counts as bad)."""
    reports = []
    for _ in range(n_steps):
        env.step(env.get_random_actions())
        rep = O.compare_one_step(env.world, broadphase=broadphase, max_bad_frac=max_bad_frac, certify=certify)
        reports.append(rep)
    return reports


# Parity numbers of this session, printed as one "PARITY {json}" line per config at the end of
# the run (tests/conftest.py pytest_terminal_summary), so that they land in the driver's log tail.
SUMMARY = []


def summarize(config, env, reps, lidar=None):
    """Fold the per-step reports of one config into one record (and keep it for the summary)."""
    w = env.world
    eng = getattr(w, "engine", None)
    src = eng.jit_source() if (eng is not None and eng.kernel_name == "k_world") else ""
    rec = {
        "config": config,
        "device": str(w.device),
        "kernel": getattr(eng, "kernel_name", None),
        "math": ("relaxed" if "VMAS_PHYS_RELAXED" in src else "exact") if src else "exact",
        "envs": reps[0]["n_envs"] if reps else 0,
        "steps": len(reps),
        "substeps": w._substeps,
        "bad_envs": sum(r["bad_envs"] for r in reps),
        "certified_envs": sum(r.get("certified_envs", 0) for r in reps),
        "uncertified_envs": sum(r["uncertified_envs"] for r in reps),
        "certified_max_margin": max((r.get("certified_max_margin", 0.0) for r in reps), default=0.0),
        "certified_max_bound_frac": max((r.get("certified_max_bound_frac", 0.0) for r in reps), default=0.0),
        "max_abs": {k: max(r["max_abs"].get(k, 0.0) for r in reps) for k in reps[0]["max_abs"]} if reps else {},
        # aggregate guards (max over the steps): p99.9 and mean over envs of the per-env max |diff|
        "p999_abs": {k: max(r.get("p999_abs", {}).get(k, 0.0) for r in reps) for k in reps[0].get("p999_abs", {})}
        if reps else {},
        "mean_abs": {k: max(r.get("mean_abs", {}).get(k, 0.0) for r in reps) for k in reps[0].get("mean_abs", {})}
        if reps else {},
        "band_max": {k: max(r.get("band_max", {}).get(k, 0.0) for r in reps) for k in reps[0].get("band_max", {})}
        if reps else {},
        "passes": [r.get("iterations") for r in reps],
    }
    if lidar is not None:
        rec["lidar"] = {k: lidar[k] for k in ("rows", "bad_rows", "uncertified_rows", "max_abs")}
    SUMMARY.append(rec)
    return rec


# ray perturbations that certify a LIDAR mismatch as a hit/miss boundary case: the engine's value
# must equal the oracle's for a ray turned by a few 1e-7 rad (a last-bit difference of the
# angle's sin/cos) -- a tangent ray, a slab edge of a box, a line end point
_RAY_CERT_DELTAS = (-1e-6, -3e-7, 3e-7, 1e-6)


def lidar_parity(env, atol=2e-5, rtol=2e-5, max_bad_frac=0.0, measured=False):
    """Every agent sensor: engine measure() vs the oracle's cast_rays on the same state/angles.
    A (env, ray) outside atol/rtol passes only when certified as a boundary case (see above).
    measured=True: check each sensor's last measurement (what the step's observation program
    produced, e.g. a fused scenario program's LIDAR) instead of a fresh measure()."""
    w = env.world
    snap = O.snapshot(w)
    ow = O.OracleWorld(w, snap)
    worst, n_bad, n_unc, n_tot = 0.0, 0, 0, 0
    for agent in w.agents:
        ai = w.entities.index(agent)
        for sensor in agent.sensors:
            got = (sensor._last_measurement if measured else sensor.measure()).detach().cpu()
            angles = sensor._angles.detach().cpu() + snap[ai]["rot"]
            exp = ow.cast_rays(ai, angles, sensor._max_range, sensor.entity_filter)
            diff = (got - exp).abs()
            bad = diff > atol + rtol * exp.abs()
            worst = max(worst, float(diff.max()))
            n_bad += int(bad.any(-1).sum())
            if bad.any():
                cert = torch.zeros_like(bad)
                for d in _RAY_CERT_DELTAS:
                    e2 = ow.cast_rays(ai, angles + d, sensor._max_range, sensor.entity_filter)
                    cert |= (got - e2).abs() <= atol + rtol * e2.abs()
                n_unc += int((bad & ~cert).any(-1).sum())
            n_tot += got.shape[0]
    return {"ok": n_unc <= max_bad_frac * max(n_tot, 1), "max_abs": worst, "bad_rows": n_bad,
            "uncertified_rows": n_unc, "rows": n_tot}


def distance_parity(env, atol=2e-5):
    """get_distance / is_overlapping for every entity pair: engine vs oracle."""
    w = env.world
    snap = O.snapshot(w)
    ow = O.OracleWorld(w, snap)
    worst, mism = 0.0, 0
    ents = w.entities
    for i, a in enumerate(ents):
        for j, b in enumerate(ents):
            if j <= i:
                continue
            got = w.get_distance(a, b).detach().cpu()
            exp = ow.get_distance(ow.ents[i], ow.ents[j])
            worst = max(worst, float((got - exp).abs().max()))
            go = w.is_overlapping(a, b).detach().cpu()
            eo = ow.is_overlapping(ow.ents[i], ow.ents[j])
            mism += int((go != eo).sum())
    return {"ok": worst <= atol and mism == 0, "max_abs": worst, "overlap_mismatch": mism}


def assert_aggregate(rec, p999_bound, mean_bound):
    """Aggregate error guard over envs: the per-step tolerance admits a
    contact-cut-off env's large error, so a systematic error of 100x could pass it; the 99.9th
    percentile and the mean over envs of the per-env max |diff| cannot move that far without a
    real regression.  Bounds are ~10x the values measured on gfx950."""
    for k, bnd in p999_bound.items():
        assert rec["p999_abs"].get(k, 0.0) <= bnd, (rec["config"], "p99.9", k, rec["p999_abs"].get(k), bnd)
    for k, bnd in mean_bound.items():
        assert rec["mean_abs"].get(k, 0.0) <= bnd, (rec["config"], "mean", k, rec["mean_abs"].get(k), bnd)
