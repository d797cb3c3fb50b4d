# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Shared pieces of the kinematic dynamics models (DiffDrive, KinematicBicycle, Drone): the
explicit Euler / classic RK4 state increment and the force / torque that make the physics step
reproduce a desired one-step displacement.  The float operations and their order are the
reference's (dynamics/diff_drive.py:33-46, 60-88; kinematic_bicycle.py:57-70, 88-112;
drone.py:110-121, 130-160), so the increments equal the reference's tensor program bit for bit."""
import torch

from .. import utils


def increment(f, state, dt: float, integration: str, *cmd):
    """dt * f (Euler) or the RK4 combination (dt / 6) * (k1 + 2 k2 + 2 k3 + k4)."""
    if integration == "euler":
        return dt * f(state, *cmd)
    k1 = f(state, *cmd)
    k2 = f(state + dt * k1 / 2, *cmd)
    k3 = f(state + dt * k2 / 2, *cmd)
    k4 = f(state + dt * k3, *cmd)
    return (dt / 6) * (k1 + 2 * k2 + 2 * k3 + k4)


def check_integration(integration: str) -> None:
    assert integration in ("rk4", "euler"), "Integration method must be 'euler' or 'rk4'."


def apply_displacement(agent, dx, dy, dtheta, dt: float) -> None:
    """Force and torque such that one step of the (drag-free) integrator moves the agent by
    (dx, dy) and turns it by dtheta from its current velocities: a = (delta - v dt) / dt^2,
    F = m a, tau = I alpha.  The force is written into the agent's force tensor in place, the
    torque re-bound (as the reference does)."""
    vel, ang = agent.state.vel, agent.state.ang_vel
    ax = (dx - vel[:, 0] * dt) / dt ** 2
    ay = (dy - vel[:, 1] * dt) / dt ** 2
    aw = (dtheta - ang[:, 0] * dt) / dt ** 2
    fx = agent.mass * ax
    fy = agent.mass * ay
    tq = agent.moment_of_inertia * aw
    agent.state.force[:, utils.X] = fx
    agent.state.force[:, utils.Y] = fy
    agent.state.torque = tq.unsqueeze(-1)


def pose(agent) -> torch.Tensor:
    """[B, 3] (x, y, theta)."""
    return torch.cat((agent.state.pos, agent.state.rot), dim=1)
