"""Analytic known-answer tests (SURVEY.md §8c "How the build pins parity").

The reference ships no numeric golden vectors, so the oracle (and, through it, the engine) is
pinned by closed-form cases of every building block: soft contact force, free-body drag +
integration, gravity, friction, closest points, ray casts, joint torque.  Each case is checked
on the oracle AND on the native engine (host backend of libvmas_mi355x.so).
"""
import math

import numpy as np
import pytest
import torch

from oracle import vmas_oracle as O
from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Box, Landmark, Line, Sphere, World

K = 1e-3  # contact_margin


def softplus_pen(x):
    return K * (max(0.0, x / K) + math.log1p(math.exp(-abs(x / K))))


def world_with(*entities, **kw):
    w = World(1, "cpu", **kw)
    for e in entities:
        (w.add_agent if isinstance(e, Agent) else w.add_landmark)(e)
    return w


def set_state(e, pos, vel=(0.0, 0.0), rot=0.0, ang=0.0):
    e.state.pos = torch.tensor([pos], dtype=torch.float32)
    e.state.vel = torch.tensor([vel], dtype=torch.float32)
    e.state.rot = torch.tensor([[rot]], dtype=torch.float32)
    e.state.ang_vel = torch.tensor([[ang]], dtype=torch.float32)


def step_both(w):
    """(oracle result, engine result) of one step from the current state."""
    expected, _ = O.oracle_step(w)
    w.step()
    return expected, O.snapshot(w)


def test_sphere_sphere_contact_force():
    a = Landmark("a", shape=Sphere(0.05), movable=True)
    b = Landmark("b", shape=Sphere(0.05), movable=False)
    w = world_with(a, b, drag=0.0)
    set_state(a, (0.09, 0.0))
    set_state(b, (0.0, 0.0))
    f = 100 * softplus_pen(0.1 - 0.09)  # F = c * pen along delta_hat (+x)
    v_exp = f / 1.0 * 0.1
    exp, got = step_both(w)
    for res in (exp, got):
        assert res[0]["vel"][0, 0].item() == pytest.approx(v_exp, rel=1e-5)
        assert res[0]["vel"][0, 1].item() == pytest.approx(0.0, abs=1e-9)
        assert res[0]["pos"][0, 0].item() == pytest.approx(0.09 + v_exp * 0.1, rel=1e-6)


def test_no_force_outside_contact():
    a = Landmark("a", shape=Sphere(0.05), movable=True)
    b = Landmark("b", shape=Sphere(0.05), movable=False)
    w = world_with(a, b, drag=0.0)
    set_state(a, (0.1001, 0.0))
    set_state(b, (0.0, 0.0))
    exp, got = step_both(w)
    for res in (exp, got):
        assert res[0]["vel"][0, 0].item() == 0.0


@pytest.mark.parametrize("substeps", [1, 4])
def test_free_body_drag_gravity_integration(substeps):
    # v1 = (1 - drag) v0 + F/m dt_sub per substep (drag at substep 0 only); p += v dt_sub
    a = Landmark("a", shape=Sphere(0.05), movable=True, mass=2.0)
    w = world_with(a, drag=0.25, gravity=(0.0, -0.5), substeps=substeps)
    set_state(a, (0.0, 1.0), vel=(1.0, 0.0))
    dt = 0.1 / substeps
    v = np.array([1.0, 0.0]) * 0.75
    p = np.array([0.0, 1.0])
    for _ in range(substeps):
        v = v + np.array([0.0, -0.5]) * dt  # F/m = g
        p = p + v * dt
    exp, got = step_both(w)
    for res in (exp, got):
        assert np.allclose(res[0]["vel"][0].numpy(), v, atol=1e-6)
        assert np.allclose(res[0]["pos"][0].numpy(), p, atol=1e-6)


def test_linear_friction_stops_slow_body():
    # friction force magnitude min(mu*m, |v|/dt*m) per component: a slow body stops exactly
    a = Landmark("a", shape=Sphere(0.05), movable=True, linear_friction=10.0)
    w = world_with(a, drag=0.0)
    set_state(a, (0.0, 0.0), vel=(0.05, 0.0))
    exp, got = step_both(w)
    for res in (exp, got):
        assert abs(res[0]["vel"][0, 0].item()) < 1e-7


def test_agent_force_clamps():
    ag = Agent("ag", shape=Sphere(0.05), max_f=0.5, f_range=0.3)
    w = world_with(ag, drag=0.0)
    set_state(ag, (0.0, 0.0))
    ag.state.force = torch.tensor([[3.0, 4.0]])
    exp, got = step_both(w)
    # clamp_with_norm -> (0.3, 0.4), then clamp +-0.3 -> (0.3, 0.3)
    for res in (exp, got):
        assert np.allclose(res[0]["force"][0].numpy(), [0.3, 0.3], atol=1e-7)
        assert np.allclose(res[0]["vel"][0].numpy(), [0.03, 0.03], atol=1e-7)


def test_line_sphere_torque_sign():
    # sphere pressing down on the +x end of a horizontal line: line gets negative torque
    line = Landmark("line", shape=Line(1.0), movable=True, rotatable=True)
    s = Landmark("s", shape=Sphere(0.05), movable=False)
    w = world_with(line, s, drag=0.0)
    set_state(line, (0.0, 0.0))
    set_state(s, (0.4, 0.05))
    exp, got = step_both(w)
    for res in (exp, got):
        assert res[0]["ang_vel"][0, 0].item() < 0
        assert res[0]["vel"][0, 1].item() < 0


def test_box_sphere_closest_point_and_inner_point():
    # oracle geometry: sphere at (1, 0), axis-aligned box 1 x 0.5 at origin -> closest (0.5, 0)
    cp = O.get_closest_point_box(torch.zeros(1, 2), torch.zeros(1, 1), 0.5, 1.0, torch.tensor([[1.0, 0.0]]))
    # (f32 cos(pi/2) = -4.4e-8 leaves a ~1e-8 residue in y)
    assert torch.allclose(cp, torch.tensor([[0.5, 0.0]]), atol=1e-6)
    inner, d = O.get_inner_point_box(torch.tensor([[1.0, 0.0]]), cp, torch.zeros(1, 2))
    assert torch.allclose(inner, torch.tensor([[0.0, 0.0]]), atol=1e-6)
    assert torch.allclose(d, torch.tensor([0.5]), atol=1e-6)


def test_line_line_intersection():
    pa, pb = O.get_closest_points_line_line(
        torch.zeros(1, 2), torch.zeros(1, 1), 1.0, torch.zeros(1, 2), torch.full((1, 1), math.pi / 2), 1.0
    )
    assert torch.allclose(pa, torch.zeros(1, 2), atol=1e-7) and torch.allclose(pb, pa)


def test_ray_casts_analytic():
    # ray from the origin along +x: sphere (0.5,0) r=0.1 -> 0.4; box centred 0.5, L=0.2 -> 0.4;
    # vertical line at x=0.5 -> 0.5; max_range when nothing is hit
    cases = ((lambda: Sphere(0.1), (0.5, 0.0), 0.0, 0.4), (lambda: Box(length=0.2, width=0.2), (0.5, 0.0), 0.0, 0.4),
             (lambda: Line(length=0.4), (0.5, 0.0), math.pi / 2, 0.5), (lambda: Sphere(0.1), (0.5, 0.5), 0.0, 1.0))
    for shape, pos, rot, expected in cases:
        ag = Agent("ag", shape=Sphere(0.01))
        target = Landmark("t", shape=shape())
        w = world_with(ag, target)
        set_state(ag, (0.0, 0.0))
        set_state(target, pos, rot=rot)
        angles = torch.zeros(1, 1)
        got = w.cast_rays(ag, angles, max_range=1.0, entity_filter=lambda e: e is target)
        ow = O.OracleWorld(w, O.snapshot(w))
        exp = ow.cast_rays(w.entities.index(ag), angles, 1.0, lambda e: e is target)
        assert got.item() == pytest.approx(expected, abs=1e-6)
        assert exp.item() == pytest.approx(expected, abs=1e-6)


def test_joint_fixed_rotation_torque():
    # _get_constraint_torques: tau = -/+ c * sign(drot) * (exp(|drot|) - 1)
    ow = O.OracleWorld.__new__(O.OracleWorld)
    ta, tb = O.OracleWorld._get_constraint_torques(ow, torch.tensor([[0.3]]), torch.tensor([[0.1]]), 1.0)
    assert ta.item() == pytest.approx(-(math.exp(0.2) - 1), rel=1e-6)
    assert tb.item() == pytest.approx(math.exp(0.2) - 1, rel=1e-6)


def test_distance_queries_analytic():
    a = Landmark("a", shape=Sphere(0.1))
    b = Landmark("b", shape=Box(length=1.0, width=0.5))
    c = Landmark("c", shape=Line(length=1.0))
    w = world_with(a, b, c)
    set_state(a, (1.0, 0.0))
    set_state(b, (0.0, 0.0))
    set_state(c, (0.0, 2.0))
    # sphere to box: |(1,0)-(0.5,0)| - LINE_MIN_DIST - r
    assert w.get_distance(a, b).item() == pytest.approx(0.5 - 4 / 600 - 0.1, abs=1e-6)
    # box to line: the line is 1.75 above the box top
    assert w.get_distance(b, c).item() == pytest.approx(1.75 - 4 / 600, abs=1e-6)
    assert not bool(w.is_overlapping(a, b)[0])
    set_state(a, (0.3, 0.0))
    assert bool(w.is_overlapping(a, b)[0]) and w.get_distance(a, b).item() == -1
