# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Quadrotor (vmas/simulator/dynamics/drone.py:16-160): a 12-dimensional rigid-body state
(roll, pitch, yaw, their rates, linear velocity, position) driven by (thrust, torque x/y/z),
integrated over one step (Euler or RK4); the planar part (x, y velocity change, yaw rate change)
becomes the force / torque of the 2-D physics step.  The thrust action is offset by m g so a
zero action hovers."""
from typing import Union

import torch
from torch import Tensor

from .. import utils
from . import _integrators as I
from .common import Dynamics

# drone_state columns
PHI, THETA, PSI, P, Q, R, VX, VY, VZ, X, Y, Z = range(12)


class Drone(Dynamics):
    def __init__(self, world, I_xx: float = 8.1e-3, I_yy: float = 8.1e-3, I_zz: float = 14.2e-3,
                 integration: str = "rk4"):
        super().__init__()
        assert integration in ("rk4", "euler")
        self.integration = integration
        self.I_xx, self.I_yy, self.I_zz = I_xx, I_yy, I_zz
        self.world = world
        self.g = 9.81
        self.dt = world.dt
        self.reset()

    def reset(self, index: Union[Tensor, int] = None):
        if index is None:
            self.drone_state = torch.zeros(self.world.batch_dim, 12, device=self.world.device)
        else:
            self.drone_state = utils.TorchUtils.where_from_index(index, 0.0, self.drone_state)

    def zero_grad(self):
        self.drone_state = self.drone_state.detach()

    def f(self, state, thrust_command, torque_command):
        phi, theta, psi = state[:, PHI], state[:, THETA], state[:, PSI]
        p, q, r = state[:, P], state[:, Q], state[:, R]
        c_phi, s_phi = torch.cos(phi), torch.sin(phi)
        c_theta, s_theta = torch.cos(theta), torch.sin(theta)
        c_psi, s_psi = torch.cos(psi), torch.sin(psi)
        m = self.agent.mass
        x_ddot = (c_phi * s_theta * c_psi + s_phi * s_psi) * thrust_command / m
        y_ddot = (c_phi * s_theta * s_psi - s_phi * c_psi) * thrust_command / m
        z_ddot = (c_phi * c_theta) * thrust_command / m - self.g
        p_dot = (torque_command[:, 0] - (self.I_yy - self.I_zz) * q * r) / self.I_xx
        q_dot = (torque_command[:, 1] - (self.I_zz - self.I_xx) * p * r) / self.I_yy
        r_dot = (torque_command[:, 2] - (self.I_xx - self.I_yy) * p * q) / self.I_zz
        return torch.stack([p, q, r, p_dot, q_dot, r_dot, x_ddot, y_ddot, z_ddot,
                            state[:, VX], state[:, VY], state[:, VZ]], dim=-1)

    def needs_reset(self) -> Tensor:
        """Roll or pitch beyond +-30 degrees."""
        return torch.any(self.drone_state[:, :2].abs() > 30 * (torch.pi / 180), dim=-1)

    def euler(self, state, thrust, torque):
        return I.increment(self.f, state, self.dt, "euler", thrust, torque)

    def runge_kutta(self, state, thrust, torque):
        return I.increment(self.f, state, self.dt, "rk4", thrust, torque)

    @property
    def needed_action_size(self) -> int:
        return 4

    def process_action(self):
        u = self.agent.action.u
        thrust = u[:, 0]
        torque = u[:, 1:4]
        thrust += self.agent.mass * self.g  # (in place on the action, as the reference)
        self.drone_state[:, X] = self.agent.state.pos[:, 0]
        self.drone_state[:, Y] = self.agent.state.pos[:, 1]
        self.drone_state[:, PSI] = self.agent.state.rot[:, 0]
        delta = I.increment(self.f, self.drone_state, self.dt, self.integration, thrust, torque)
        self.drone_state = self.drone_state + delta
        I.apply_displacement(self.agent, delta[:, VX], delta[:, VY], delta[:, R], self.dt)
