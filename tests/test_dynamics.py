"""Dynamics models and the velocity controller (ref vmas/simulator/dynamics/*.py,
controllers/velocity_controller.py): the reference's scenario-side action programs, which feed the
physics step its force / torque inputs.  Closed-form checks of the forces they produce, a world of
each stepped through the engine (host backend; gfx950 with -m gpu), and the reference module
names through the ``vmas`` alias."""
import math

import pytest
import torch

from vectorizedmultiagentsimulator_amd.simulator.controllers.velocity_controller import VelocityController
from vectorizedmultiagentsimulator_amd.simulator.core import Agent, World
from vectorizedmultiagentsimulator_amd.simulator.dynamics.diff_drive import DiffDrive
from vectorizedmultiagentsimulator_amd.simulator.dynamics.drone import Drone
from vectorizedmultiagentsimulator_amd.simulator.dynamics.kinematic_bicycle import KinematicBicycle

DEVICES = [pytest.param("cpu", id="cpu"), pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


@pytest.fixture(params=DEVICES)
def device(request):
    if request.param == "cuda":
        if not torch.cuda.is_available():
            pytest.skip("no ROCm GPU visible")
        return "cuda:0"
    return "cpu"


def _world(device, B, dyn, **agent_kw):
    w = World(B, device, substeps=10)
    a = Agent("a", dynamics=dyn(w), **agent_kw)
    w.add_agent(a)
    for e in w.entities:
        e.state.pos = torch.zeros(B, 2, device=device)
        e.state.vel = torch.zeros(B, 2, device=device)
        e.state.rot = torch.zeros(B, 1, device=device)
        e.state.ang_vel = torch.zeros(B, 1, device=device)
    a.state.force = torch.zeros(B, 2, device=device)
    a.state.torque = torch.zeros(B, 1, device=device)
    return w, a


def test_reference_module_names():
    import vmas  # noqa: F401
    from vmas.simulator.controllers.velocity_controller import VelocityController as V
    from vmas.simulator.dynamics.diff_drive import DiffDrive as D
    from vmas.simulator.dynamics.roatation import Rotation  # (sic, the reference's module name)
    from vmas.simulator.dynamics.rotation import Rotation as R2

    assert V is VelocityController and D is DiffDrive and Rotation is R2


@pytest.mark.parametrize("integration", ["euler", "rk4"])
def test_diff_drive_straight_line_force(device, integration):
    """omega = 0: both integrators give the exact displacement (v dt cos th, v dt sin th, 0), so
    F = m (v dt cos th - vx dt) / dt^2 and no torque (diff_drive.py:60-88)."""
    B = 64
    w, a = _world(device, B, lambda w: DiffDrive(w, integration=integration), u_range=[1, 1], u_multiplier=[1, 1])
    th = torch.linspace(-3, 3, B, device=device).unsqueeze(-1)
    a.state.rot = th
    a.state.vel = torch.full((B, 2), 0.1, device=device)
    a.action.u = torch.stack([torch.full((B,), 0.5, device=device), torch.zeros(B, device=device)], -1)
    a.dynamics.process_action()
    dt = w.dt
    fx = a.mass * ((0.5 * dt * torch.cos(th[:, 0])) - 0.1 * dt) / dt ** 2
    assert torch.allclose(a.state.force[:, 0], fx, atol=1e-4)
    assert torch.allclose(a.state.torque, torch.zeros_like(a.state.torque), atol=1e-5)


def test_kinematic_bicycle_clamps_steering_and_turns(device):
    B = 32
    w, a = _world(device, B, lambda w: KinematicBicycle(w, width=0.1, l_f=0.1, l_r=0.1, max_steering_angle=0.3),
                  u_range=[1, 1], u_multiplier=[1, 1])
    a.action.u = torch.tensor([[1.0, 5.0]] * B, device=device)  # steering far beyond the limit
    a.dynamics.process_action()
    # from rest: beta = atan(tan(0.3) / 2), theta' = v / 0.2 * cos(beta) tan(0.3) > 0 -> positive torque
    beta = math.atan(math.tan(0.3) * 0.5)
    rate = 1.0 / 0.2 * math.cos(beta) * math.tan(0.3)
    assert (a.state.torque > 0).all()
    # Euler would give exactly I * rate * dt / dt^2; RK4 integrates the same constant rate
    assert torch.allclose(a.state.torque[:, 0], torch.full((B,), a.moment_of_inertia * rate / w.dt, device=device), rtol=1e-3)


def test_drone_hover_and_step(device):
    """Zero action = hover: thrust + m g balances gravity, so no planar force from rest."""
    B = 16
    w, a = _world(device, B, lambda w: Drone(w), u_range=[1, 1, 1, 1], u_multiplier=[1, 1, 1, 1])
    a.action.u = torch.zeros(B, 4, device=device)
    a.dynamics.process_action()
    assert torch.allclose(a.state.force, torch.zeros_like(a.state.force), atol=1e-5)
    assert not a.dynamics.needs_reset().any()
    w.step()
    assert torch.isfinite(a.state.pos).all()


def test_velocity_controller_pid(device):
    B = 8
    w, a = _world(device, B, lambda w: __import__(
        "vectorizedmultiagentsimulator_amd.simulator.dynamics.holonomic", fromlist=["Holonomic"]).Holonomic(),
        f_range=2.0, mass=2.0)
    c = VelocityController(a, w, ctrl_params=(2.0, 0.5, 0.1), pid_form="standard")
    a.action.u = torch.ones(B, 2, device=device)
    c.process_force()
    # err = 1; I = (dt * err) / Ti; D = Td * err / dt; u = kP (err + I + D) * m
    dt = w.dt
    want = 2.0 * (1 + dt / 0.5 + 0.1 / dt) * 2.0
    assert torch.allclose(a.action.u, torch.full((B, 2), want, device=device), rtol=1e-5)
    # anti-windup at 0.5 * f_max * Ti / (dt * kP)
    assert c.integrator_windup_cutoff == pytest.approx(0.5 * 2.0 * 0.5 / (dt * 2.0))
    c.reset(0)
    assert (c.prev_err[0] == 0).all() and (c.prev_err[1:] == 1).all()
