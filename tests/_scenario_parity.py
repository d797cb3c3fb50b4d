"""Parity driver for what env.step computes around World.step: the action path (u, state.force)
and the benchmark scenarios' reward / observation / done / info programs, product vs the CPU oracle
(oracle/vmas_scenario_oracle.py) on the same states and actions.

Per step: the state before the step and the actions are copied to the CPU, the product steps, the
state after it is copied, and the oracle's programs run on those copies (teacher forcing: the
oracle carries only its own shaping state, set from the reset state).  Tolerances (fp32):
  * u / state.force of policy agents: bit-exact (a clamp and one fp32 product per element);
    a scripted agent's u (cos / sin of t / 30): 2e-6;
  * observations outside LIDAR columns: 1e-6 + 1e-6 |x| (copies and differences of state;
    ``rot % pi`` is one remainder);
  * rewards / infos: 1e-4 + 1e-5 |x| (differences of two norms scaled by the shaping factor 100);
  * dones: exact; LIDAR columns: tests/_parity.py's LIDAR tolerance (2e-5 + 2e-5 |x|) with its
    ray-turn certification, then (_scan_certify; counted as scan_certified_rows) a scan over rays
    turned by up to SCAN_DELTA and the oracle's own 1-ulp conditioning band at the row, for
    near-grazing hits of the fast LIDAR (hardware sin / cos); strict=True (the exact LIDAR,
    _fused.EXACT_LIDAR) turns every certification tier off.
An env outside these passes only when the oracle certifies it sits on a flag threshold: some
distance the programs compared with a threshold (overlap, coverage, collision) lies within
MARGIN_TOL of it, so a last-bit difference of that distance flips the flag.
"""
from __future__ import annotations

import torch

from oracle import vmas_oracle as O
from oracle import vmas_scenario_oracle as SO
from tests import _parity

MARGIN_TOL = 4e-6
OBS_ATOL, OBS_RTOL = 1e-6, 1e-6
REW_ATOL, REW_RTOL = 1e-4, 1e-5
LIDAR_ATOL, LIDAR_RTOL = 2e-5, 2e-5
SCRIPTED_U_ATOL = 2e-6


def _cpu(t):
    return t.detach().to("cpu")


# The fast LIDAR's ray direction is (v_cos_f32, v_sin_f32) of the fp32 angle a (|a| < 16 rad,
# vmas_scenarios.hip kFastTrigMaxAngle).  The instructions take revolutions: the product
# a * fl(1 / 2 pi) rounds once (relative 2^-24) and fl(1 / 2 pi) carries another 2^-24, so the angle
# they see is off by at most |a| * 2^-23 rad (1.9e-6 at 16 rad, 7.5e-7 at 2 pi: the LIDAR angles
# of a non-rotating agent), plus the instructions' own output error.  FAST_TRIG_DIR_ERR bounds the
# whole direction error |(cos', sin') - (cos a, sin a)| over |a| < 16; the GPU test
# test_fast_trig_direction_error_is_bounded_gpu (tests/test_scenario_oracle.py) measures it over
# 2^24 angles against float64 and asserts it stays below.  SCAN_DELTA -- how far the scan
# certification turns the oracle's ray -- is that bound (VERDICT r5 "Next" #3).
FAST_TRIG_DIR_ERR = 2.5e-6
SCAN_DELTA, SCAN_POINTS = FAST_TRIG_DIR_ERR, 41
CERT_DETAIL_ROWS = 12  # scan-certified rows listed in the PARITY line (ray, grazing |d - r|, delta)


def _scan_certify(world, snap, idx, ai, rays, spec, got, bad):
    """A LIDAR value outside the tolerance that no single ray turn of tests/_parity.py reproduces:
    a near-grazing hit, where dist = |foot - o| - sqrt(r^2 - d^2) turns steep as d -> r, so that
    last-bit differences of d (hardware sin / cos of the fast LIDAR, ~1e-6 rad) move it by more
    than the tolerance.  Certified when the oracle, scanned over rays turned by up to SCAN_DELTA
    (SCAN_POINTS angles), takes the engine's value: equal within the tolerance at a scanned angle,
    or between the values at two neighbouring scanned angles that both hit (the hit distance is
    continuous there, so an angle in between gives it exactly).  Returns, per row of ``idx``,
    whether every bad ray of it is certified."""
    from oracle import vmas_oracle as O

    sub = {i: {k: v[idx] for k, v in d.items()} for i, d in snap.items()}
    ow = O.OracleWorld(world, sub)
    ow.batch_dim = len(idx)
    r0, gv, bd = rays[idx], got[idx], bad[idx]
    scan = torch.stack([ow.cast_rays(ai, r0 + dl, spec.max_range, spec.entity_filter)
                        for dl in torch.linspace(-SCAN_DELTA, SCAN_DELTA, SCAN_POINTS).tolist()])  # [K, n, R]
    tol = LIDAR_ATOL + LIDAR_RTOL * gv.abs()
    eq = ((scan - gv).abs() <= tol).any(0)
    hit = scan < spec.max_range
    lo, hi = torch.minimum(scan[:-1], scan[1:]), torch.maximum(scan[:-1], scan[1:])
    between = (hit[:-1] & hit[1:] & (lo - tol <= gv) & (gv <= hi + tol)).any(0)
    # the oracle's own conditioning at the row (as the step parity's 1-ulp band, vmas_oracle.compare):
    # near a grazing hit m = sqrt(r^2 - d^2) cancels, and last-bit changes of the positions move
    # the distance by far more than the tolerance; accepted within 4x the spread of the oracle
    # over LIDAR_BAND_N random ~1-ulp relative perturbations of every position
    e0 = ow.cast_rays(ai, r0, spec.max_range, spec.entity_filter)
    g = torch.Generator().manual_seed(4321)
    band = torch.zeros_like(e0)
    for _ in range(LIDAR_BAND_N):
        pert = {i: {k: (v * (1 + 1.2e-7 * torch.randn(v.shape, generator=g)) if k == "pos" else v)
                    for k, v in d.items()} for i, d in sub.items()}
        ow2 = O.OracleWorld(world, pert)
        ow2.batch_dim = len(idx)
        e2 = ow2.cast_rays(ai, r0, spec.max_range, spec.entity_filter)
        band = torch.maximum(band, torch.where((e2 < spec.max_range) & (e0 < spec.max_range), (e2 - e0).abs(), 0.0))
    banded = (gv - e0).abs() <= tol + 4 * band
    return ((eq | between | banded) | ~bd).all(-1)


LIDAR_BAND_N = 8


def _grazing(world, snap, b, ai, theta, spec):
    """|d - r| of the sphere target the ray (agent ai, angle theta, env b) passes closest to: d the
    target centre's distance from the ray's line, r its radius (near 0: a grazing ray)."""
    from oracle import vmas_oracle as O

    sub = {i: {k: v[b:b + 1] for k, v in d.items()} for i, d in snap.items()}
    ow = O.OracleWorld(world, sub)
    ow.batch_dim = 1
    o = ow.ents[ai].state.pos[0].double()
    u = torch.tensor([torch.cos(torch.tensor(theta, dtype=torch.float64)),
                      torch.sin(torch.tensor(theta, dtype=torch.float64))], dtype=torch.float64)
    best = float("inf")
    for e in ow.ents:
        if e is ow.ents[ai] or not spec.entity_filter(e.e) or not hasattr(e.shape, "radius"):
            continue
        c = e.state.pos[0].double() - o
        if float(c @ u) <= 0:
            continue
        d = abs(float(c[0] * u[1] - c[1] * u[0]))
        best = min(best, abs(d - float(e.shape.radius)))
    return best


def _env_err(got, exp, atol, rtol):
    """Per env: max |diff| and whether any element is outside atol + rtol |exp| (NaN mismatch bad)."""
    g, e = _cpu(got).float(), exp.float()
    if g.dim() == 1:
        g, e = g.unsqueeze(-1), e.unsqueeze(-1)
    diff = (g - e).abs()
    nan = torch.isnan(g) != torch.isnan(e)
    bad = ((diff > atol + rtol * e.abs()) | nan).any(-1)
    return diff.nan_to_num(0.0).amax(-1), bad


class ScenarioParity:
    """Runs ``steps`` random-action steps of ``env`` (fresh from make_env) against the oracle."""

    def __init__(self, env, name: str, kw: dict, strict: bool = False):
        self.env, self.name = env, name
        self.strict = strict  # (no LIDAR certification tier at all: every row outside the tolerance fails)
        self.prog = SO.program(name, env.world, **kw)
        self.prog.reset(O.snapshot(env.world))
        B = env.world.batch_dim
        self.rec = {"bad_envs": 0, "certified_envs": 0, "uncertified_envs": 0, "certified_max_margin": 0.0,
                    "max_abs": {}, "lidar": {"rows": 0, "bad_rows": 0, "uncertified_rows": 0, "max_abs": 0.0},
                    "actions": {"u_bad": 0, "force_bad": 0, "scripted_max_abs": 0.0}, "steps": 0, "envs": B}
        self.failures = []

    def _worst(self, key, v):
        m = self.rec["max_abs"]
        m[key] = max(m.get(key, 0.0), float(v.max()) if v.numel() else 0.0)

    def step(self, actions=None):
        env, w, prog = self.env, self.env.world, self.prog
        pre = O.snapshot(w)
        if actions is None:
            actions = env.get_random_actions()
        acts = [_cpu(a).clone() for a in actions]
        scripted_u = prog.scripted_u() if hasattr(prog, "scripted_u") else None
        out = env.step(actions)
        post = O.snapshot(w)
        self._check_actions(acts, scripted_u)
        exp = prog.step(pre, post)
        self._check_outputs(out, exp, pre, post)
        self.rec["steps"] += 1
        return out, exp

    # ---- the action path ------------------------------------------------------------------------
    def _check_actions(self, acts, scripted_u):
        env, w = self.env, self.env.world
        a_rec = self.rec["actions"]
        for a, ag in zip(acts, env.agents):
            u, _ = SO.set_action(a, action_size=ag.action_size, u_range=ag.action.u_range,
                                 u_multiplier=ag.action.u_multiplier, dim_p=w.dim_p, dim_c=w.dim_c, silent=ag.silent,
                                 clamp_action=bool(env.clamp_action))
            f = SO.apply_action_force(SO.holonomic_process_action(u), ag.max_f, ag.f_range)
            if not torch.equal(_cpu(ag.action.u), u):
                a_rec["u_bad"] += 1
                self.failures.append(("u", ag.name))
            if not torch.equal(_cpu(ag.state.force), f):
                a_rec["force_bad"] += 1
                self.failures.append(("force", ag.name))
        for ag in w.agents:
            if ag.action_script is None:
                continue
            SO.check_scripted_action(scripted_u, ag.action.u_multiplier, ag.action.u_range, ag.action_size)
            d = (_cpu(ag.action.u) - scripted_u).abs().max()
            f = SO.apply_action_force(SO.holonomic_process_action(scripted_u), ag.max_f, ag.f_range)
            d = max(float(d), float((_cpu(ag.state.force) - f).abs().max()))
            a_rec["scripted_max_abs"] = max(a_rec["scripted_max_abs"], d)
            if d > SCRIPTED_U_ATOL:
                self.failures.append(("scripted u", ag.name, d))

    # ---- the scenario program -------------------------------------------------------------------
    def _check_outputs(self, out, exp, pre, post):
        env, w = self.env, self.env.world
        obs, rews, dones, infos = out[0], out[1], out[2], out[-1]
        B = w.batch_dim
        bad = torch.zeros(B, dtype=torch.bool)
        # LIDAR columns, certified row by row
        lidar_cols = {}
        lr = self.rec["lidar"]
        ow = O.OracleWorld(w, post)
        lidar_bad_rows = torch.zeros(B, dtype=torch.bool)
        for (k, c0, c1, ai, rays, spec) in exp["lidar"]:
            lidar_cols.setdefault(k, []).append((c0, c1))
            g = _cpu(obs[k][:, c0:c1])
            e = exp["obs"][k][:, c0:c1]
            diff = (g - e).abs()
            rb = diff > LIDAR_ATOL + LIDAR_RTOL * e.abs()
            lr["max_abs"] = max(lr["max_abs"], float(diff.max()))
            lr["rows"] += B
            lr["bad_rows"] += int(rb.any(-1).sum())
            if rb.any() and self.strict:
                unc = rb.any(-1)
                lr["uncertified_rows"] += int(unc.sum())
                lidar_bad_rows |= unc
                for b in unc.nonzero().flatten()[:4].tolist():
                    r = rb[b].nonzero().flatten().tolist()
                    self.failures.append(("lidar row (strict)", self.rec["steps"], k, c0, b, r, g[b, r].tolist(),
                                          e[b, r].tolist(), rays[b, r].tolist()))
            elif rb.any():
                cert = torch.zeros_like(rb)
                for d in _parity._RAY_CERT_DELTAS:
                    e2 = ow.cast_rays(ai, rays + d, spec.max_range, spec.entity_filter)
                    cert |= (g - e2).abs() <= LIDAR_ATOL + LIDAR_RTOL * e2.abs()
                left = rb & ~cert
                if left.any():  # near-grazing hits: the scan certification (see _scan_certify)
                    idx = left.any(-1).nonzero().flatten()
                    ok = _scan_certify(self.env.world, post, idx, ai, rays, spec, g, left)
                    lr["scan_certified_rows"] = lr.get("scan_certified_rows", 0) + int(ok.sum())
                    det = lr.setdefault("certified", [])
                    for b in idx[ok].tolist():  # what a reader needs to judge a certified row
                        if len(det) >= CERT_DETAIL_ROWS:
                            break
                        for r in left[b].nonzero().flatten().tolist()[:2]:
                            th = float(rays[b, r])
                            det.append({"step": self.rec["steps"], "env": b, "ray": r, "angle": round(th, 7),
                                        "grazing": float(f"{_grazing(self.env.world, post, b, ai, th, spec):.3g}"),
                                        "delta": float(f"{abs(float(g[b, r]) - float(e[b, r])):.3g}")})
                    left[idx[ok]] = False
                unc = left.any(-1)
                lr["uncertified_rows"] += int(unc.sum())
                lidar_bad_rows |= unc
                for b in unc.nonzero().flatten()[:4].tolist():  # what a reader needs to judge the row
                    r = left[b].nonzero().flatten().tolist()
                    self.failures.append(("lidar row", self.rec["steps"], k, c0, b, r, g[b, r].tolist(),
                                          e[b, r].tolist(), rays[b, r].tolist()))
        # the rest of the observations
        assert len(obs) == len(exp["obs"]), (len(obs), len(exp["obs"]))
        for k, (g, e) in enumerate(zip(obs, exp["obs"])):
            assert g.shape == e.shape, ("obs shape", k, tuple(g.shape), tuple(e.shape))
            keep = torch.ones(e.shape[1], dtype=torch.bool)
            for c0, c1 in lidar_cols.get(k, []):
                keep[c0:c1] = False
            m, b = _env_err(_cpu(g)[:, keep], e[:, keep], OBS_ATOL, OBS_RTOL)
            self._worst("obs", m)
            bad |= b
        assert len(rews) == len(exp["rew"])
        for g, e in zip(rews, exp["rew"]):
            assert g.shape == e.shape, ("rew shape", tuple(g.shape), tuple(e.shape))
            m, b = _env_err(g, e, REW_ATOL, REW_RTOL)
            self._worst("rew", m)
            bad |= b
        d_exp = exp["done"]
        assert dones.shape == d_exp.shape and dones.dtype == torch.bool, (dones.shape, dones.dtype)
        bad |= _cpu(dones) != d_exp
        assert len(infos) == len(exp["info"])
        for g, e in zip(infos, exp["info"]):
            assert set(g) == set(e), (sorted(g), sorted(e))
            for key in e:
                gv, ev = g[key], e[key]
                assert gv.shape == ev.shape, ("info", key, tuple(gv.shape), tuple(ev.shape))
                assert gv.dtype.is_floating_point == ev.dtype.is_floating_point, ("info dtype", key, gv.dtype, ev.dtype)
                m, b = _env_err(gv, ev, REW_ATOL, REW_RTOL)
                self._worst("info", m)
                bad |= b
        cert = bad & (exp["margin"] <= MARGIN_TOL)
        unc = (bad & ~cert) | lidar_bad_rows
        if "covered" in exp:  # discovery's respawn, outside certified envs
            rs = self.prog.check_respawn(pre, post, exp["covered"], exp["agents_pos"], skip=cert)
            r = self.rec.setdefault("respawn", {"bad_envs": 0, "respawned": 0, "threshold_envs": 0})
            for k2 in r:
                r[k2] += rs[k2]
            if rs["bad_envs"]:
                self.failures.append(("respawn", rs))
        self.rec["bad_envs"] += int(bad.sum())
        self.rec["certified_envs"] += int(cert.sum())
        self.rec["uncertified_envs"] += int(unc.sum())
        if cert.any():
            self.rec["certified_max_margin"] = max(self.rec["certified_max_margin"], float(exp["margin"][cert].max()))
        if unc.any():
            idx = unc.nonzero().flatten()[:8].tolist()
            self.failures.append(("outputs", self.rec["steps"], idx))

    def record(self, config: str):
        rec = dict(self.rec)
        rec["config"] = config
        rec["device"] = str(self.env.world.device)
        rec["program"] = "scenario+actions vs oracle"
        _parity.SUMMARY.append(rec)
        return rec

    @property
    def ok(self) -> bool:
        return not self.failures and self.rec["uncertified_envs"] == 0
