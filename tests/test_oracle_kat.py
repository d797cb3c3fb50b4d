"""Analytic known-answer tests (SURVEY.md §8c "How the build pins parity").

The reference ships no numeric golden vectors, so the oracle (and, through it, the engine) is
pinned by closed-form cases of every building block: soft contact force, free-body drag +
integration, gravity, friction, closest points, ray casts, joint torque.  Each step case is
checked on the oracle AND on the native engine, on three targets:
  * ``cpu``: the library's host backend, one env;
  * ``gpu-relaxed``: the gfx950 world kernel k_world in its default relaxed fp32 math (hardware
    rcp / sqrt / exp / log / sin / cos -- the kernel bench.py times), the case replicated over
    64 envs (one full wavefront; every env must give the closed-form answer);
  * ``gpu-exact``: the same with VMAS_JIT_MATH=exact (IEEE div / sqrt, ocml transcendentals).
"""
import math
from dataclasses import dataclass

import numpy as np
import pytest
import torch

from oracle import vmas_oracle as O
from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Box, Landmark, Line, Sphere, World

K = 1e-3  # contact_margin


@dataclass
class Target:
    device: str
    batch: int
    math: str | None


TARGETS = [
    pytest.param(("cpu", 1, None), id="cpu"),
    pytest.param(("cuda", 64, "relaxed"), id="gpu-relaxed", marks=pytest.mark.gpu),
    pytest.param(("cuda", 64, "exact"), id="gpu-exact", marks=pytest.mark.gpu),
]


@pytest.fixture(params=TARGETS)
def tgt(request, monkeypatch):
    dev, batch, mode = request.param
    if dev == "cuda":
        if not torch.cuda.is_available():
            pytest.skip("no ROCm GPU visible")
        monkeypatch.setenv("VMAS_JIT_MATH", mode)  # read when the world kernel is generated
        dev = "cuda:0"
    return Target(dev, batch, mode)


def softplus_pen(x):
    return K * (max(0.0, x / K) + math.log1p(math.exp(-abs(x / K))))


def world_with(*entities, tgt=None, **kw):
    tgt = tgt or Target("cpu", 1, None)
    w = World(tgt.batch, tgt.device, **kw)
    for e in entities:
        (w.add_agent if isinstance(e, Agent) else w.add_landmark)(e)
    w._kat_target = tgt
    return w


def set_state(e, pos, vel=(0.0, 0.0), rot=0.0, ang=0.0, tgt=None):
    tgt = tgt or Target("cpu", 1, None)
    rep = lambda v: torch.tensor([v] * tgt.batch, dtype=torch.float32, device=tgt.device)  # noqa: E731
    e.state.pos = rep(pos)
    e.state.vel = rep(vel)
    e.state.rot = rep([rot])
    e.state.ang_vel = rep([ang])


def step_both(w):
    """(oracle result, engine result) of one step from the current state (CPU tensors)."""
    expected, _ = O.oracle_step(w)
    w.step()
    t = w._kat_target
    if t.device != "cpu":
        assert w.engine.kernel_name == "k_world", "GPU KATs run the world-specialised kernel"
        assert ("VMAS_PHYS_RELAXED" in w.engine.jit_source()) == (t.math == "relaxed")
    return expected, O.snapshot(w)


def allclose(t, value, rel=0.0, abs_=0.0):
    """Every env of a [B, k] result equals the closed-form value (pytest.approx semantics)."""
    t = t.detach().cpu().reshape(t.shape[0], -1)
    want = torch.tensor(value, dtype=torch.float64).reshape(1, -1)
    err = (t.double() - want).abs()
    return bool((err <= torch.maximum(rel * want.abs(), torch.tensor(abs_, dtype=torch.float64))).all())


def test_sphere_sphere_contact_force(tgt):
    a = Landmark("a", shape=Sphere(0.05), movable=True)
    b = Landmark("b", shape=Sphere(0.05), movable=False)
    w = world_with(a, b, drag=0.0, tgt=tgt)
    set_state(a, (0.09, 0.0), tgt=tgt)
    set_state(b, (0.0, 0.0), tgt=tgt)
    f = 100 * softplus_pen(0.1 - 0.09)  # F = c * pen along delta_hat (+x)
    v_exp = f / 1.0 * 0.1
    exp, got = step_both(w)
    for res in (exp, got):
        assert allclose(res[0]["vel"][:, :1], [v_exp], rel=1e-5)
        assert allclose(res[0]["vel"][:, 1:], [0.0], abs_=1e-9)
        assert allclose(res[0]["pos"][:, :1], [0.09 + v_exp * 0.1], rel=1e-6)


def test_no_force_outside_contact(tgt):
    a = Landmark("a", shape=Sphere(0.05), movable=True)
    b = Landmark("b", shape=Sphere(0.05), movable=False)
    w = world_with(a, b, drag=0.0, tgt=tgt)
    set_state(a, (0.1001, 0.0), tgt=tgt)
    set_state(b, (0.0, 0.0), tgt=tgt)
    exp, got = step_both(w)
    for res in (exp, got):
        assert (res[0]["vel"] == 0.0).all()


@pytest.mark.parametrize("substeps", [1, 4])
def test_free_body_drag_gravity_integration(tgt, substeps):
    # v1 = (1 - drag) v0 + F/m dt_sub per substep (drag at substep 0 only); p += v dt_sub
    a = Landmark("a", shape=Sphere(0.05), movable=True, mass=2.0)
    w = world_with(a, drag=0.25, gravity=(0.0, -0.5), substeps=substeps, tgt=tgt)
    set_state(a, (0.0, 1.0), vel=(1.0, 0.0), tgt=tgt)
    dt = 0.1 / substeps
    v = np.array([1.0, 0.0]) * 0.75
    p = np.array([0.0, 1.0])
    for _ in range(substeps):
        v = v + np.array([0.0, -0.5]) * dt  # F/m = g
        p = p + v * dt
    exp, got = step_both(w)
    for res in (exp, got):
        assert allclose(res[0]["vel"], v.tolist(), abs_=1e-6)
        assert allclose(res[0]["pos"], p.tolist(), abs_=1e-6)


def test_linear_friction_stops_slow_body(tgt):
    # friction force magnitude min(mu*m, |v|/dt*m) per component: a slow body stops exactly
    a = Landmark("a", shape=Sphere(0.05), movable=True, linear_friction=10.0)
    w = world_with(a, drag=0.0, tgt=tgt)
    set_state(a, (0.0, 0.0), vel=(0.05, 0.0), tgt=tgt)
    exp, got = step_both(w)
    for res in (exp, got):
        assert allclose(res[0]["vel"][:, :1], [0.0], abs_=1e-7)


def test_agent_force_clamps(tgt):
    ag = Agent("ag", shape=Sphere(0.05), max_f=0.5, f_range=0.3)
    w = world_with(ag, drag=0.0, tgt=tgt)
    set_state(ag, (0.0, 0.0), tgt=tgt)
    ag.state.force = torch.tensor([[3.0, 4.0]] * tgt.batch, device=tgt.device)
    exp, got = step_both(w)
    # clamp_with_norm -> (0.3, 0.4), then clamp +-0.3 -> (0.3, 0.3)
    for res in (exp, got):
        assert allclose(res[0]["force"], [0.3, 0.3], abs_=1e-7)
        assert allclose(res[0]["vel"], [0.03, 0.03], abs_=1e-7)


def test_line_sphere_torque_sign(tgt):
    # sphere pressing down on the +x end of a horizontal line: line gets negative torque
    line = Landmark("line", shape=Line(1.0), movable=True, rotatable=True)
    s = Landmark("s", shape=Sphere(0.05), movable=False)
    w = world_with(line, s, drag=0.0, tgt=tgt)
    set_state(line, (0.0, 0.0), tgt=tgt)
    set_state(s, (0.4, 0.05), tgt=tgt)
    exp, got = step_both(w)
    for res in (exp, got):
        assert (res[0]["ang_vel"] < 0).all()
        assert (res[0]["vel"][:, 1] < 0).all()
    # and the engine agrees with the oracle's magnitudes (stated fp32 tolerance)
    assert O.compare(got, exp, w)["ok"]


def test_box_sphere_closest_point_and_inner_point():
    # oracle geometry: sphere at (1, 0), axis-aligned box 1 x 0.5 at origin -> closest (0.5, 0)
    cp = O.get_closest_point_box(torch.zeros(1, 2), torch.zeros(1, 1), 0.5, 1.0, torch.tensor([[1.0, 0.0]]))
    # (f32 cos(pi/2) = -4.4e-8 leaves a ~1e-8 residue in y)
    assert torch.allclose(cp, torch.tensor([[0.5, 0.0]]), atol=1e-6)
    inner, d = O.get_inner_point_box(torch.tensor([[1.0, 0.0]]), cp, torch.zeros(1, 2))
    assert torch.allclose(inner, torch.tensor([[0.0, 0.0]]), atol=1e-6)
    assert torch.allclose(d, torch.tensor([0.5]), atol=1e-6)


def test_box_sphere_contact_step(tgt):
    """A sphere resting 0.02 inside the right face of a fixed, solid, axis-aligned box: the
    closest point is (0.5, 0), the inner point the box centre, so dist = 0.53 from the centre vs
    d_min = r + LINE_MIN_DIST + 0.5 (core.py:2458-2551): F = c * pen along +x."""
    box = Landmark("box", shape=Box(length=1.0, width=0.5), movable=False)
    s = Landmark("s", shape=Sphere(0.05), movable=True)
    w = world_with(box, s, drag=0.0, tgt=tgt)
    set_state(box, (0.0, 0.0), tgt=tgt)
    set_state(s, (0.53, 0.0), tgt=tgt)
    d_min = 0.05 + 4 / 600 + 0.5
    f = 100 * softplus_pen(d_min - 0.53)
    exp, got = step_both(w)
    for res in (exp, got):
        assert allclose(res[1]["vel"][:, :1], [f * 0.1], rel=1e-4)
        assert allclose(res[1]["vel"][:, 1:], [0.0], abs_=1e-6)


def test_line_line_intersection():
    pa, pb = O.get_closest_points_line_line(
        torch.zeros(1, 2), torch.zeros(1, 1), 1.0, torch.zeros(1, 2), torch.full((1, 1), math.pi / 2), 1.0
    )
    assert torch.allclose(pa, torch.zeros(1, 2), atol=1e-7) and torch.allclose(pb, pa)


def test_ray_casts_analytic(tgt):
    # ray from the origin along +x: sphere (0.5,0) r=0.1 -> 0.4; box centred 0.5, L=0.2 -> 0.4;
    # vertical line at x=0.5 -> 0.5; max_range when nothing is hit
    cases = ((lambda: Sphere(0.1), (0.5, 0.0), 0.0, 0.4), (lambda: Box(length=0.2, width=0.2), (0.5, 0.0), 0.0, 0.4),
             (lambda: Line(length=0.4), (0.5, 0.0), math.pi / 2, 0.5), (lambda: Sphere(0.1), (0.5, 0.5), 0.0, 1.0))
    for shape, pos, rot, expected in cases:
        ag = Agent("ag", shape=Sphere(0.01))
        target = Landmark("t", shape=shape())
        w = world_with(ag, target, tgt=tgt)
        set_state(ag, (0.0, 0.0), tgt=tgt)
        set_state(target, pos, rot=rot, tgt=tgt)
        angles = torch.zeros(tgt.batch, 1, device=tgt.device)
        got = w.cast_rays(ag, angles, max_range=1.0, entity_filter=lambda e: e is target)
        ow = O.OracleWorld(w, O.snapshot(w))
        exp = ow.cast_rays(w.entities.index(ag), angles.cpu(), 1.0, lambda e: e is target)
        assert allclose(got, [expected], abs_=1e-6)
        assert allclose(exp, [expected], abs_=1e-6)


def test_joint_fixed_rotation_torque():
    # _get_constraint_torques: tau = -/+ c * sign(drot) * (exp(|drot|) - 1)
    ow = O.OracleWorld.__new__(O.OracleWorld)
    ta, tb = O.OracleWorld._get_constraint_torques(ow, torch.tensor([[0.3]]), torch.tensor([[0.1]]), 1.0)
    assert ta.item() == pytest.approx(-(math.exp(0.2) - 1), rel=1e-6)
    assert tb.item() == pytest.approx(math.exp(0.2) - 1, rel=1e-6)


def test_distance_queries_analytic(tgt):
    a = Landmark("a", shape=Sphere(0.1))
    b = Landmark("b", shape=Box(length=1.0, width=0.5))
    c = Landmark("c", shape=Line(length=1.0))
    w = world_with(a, b, c, tgt=tgt)
    set_state(a, (1.0, 0.0), tgt=tgt)
    set_state(b, (0.0, 0.0), tgt=tgt)
    set_state(c, (0.0, 2.0), tgt=tgt)
    # sphere to box: |(1,0)-(0.5,0)| - LINE_MIN_DIST - r
    assert allclose(w.get_distance(a, b).reshape(-1, 1), [0.5 - 4 / 600 - 0.1], abs_=1e-6)
    # box to line: the line is 1.75 above the box top
    assert allclose(w.get_distance(b, c).reshape(-1, 1), [1.75 - 4 / 600], abs_=1e-6)
    assert not bool(w.is_overlapping(a, b).any())
    set_state(a, (0.3, 0.0), tgt=tgt)
    assert bool(w.is_overlapping(a, b).all()) and bool((w.get_distance(a, b) == -1).all())
