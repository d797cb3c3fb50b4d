# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Differential drive (vmas/simulator/dynamics/diff_drive.py:13-89): the action is (forward speed,
angular speed); the unicycle model x' = v cos(theta), y' = v sin(theta), theta' = omega is
integrated over one step (Euler or RK4) and turned into the force / torque that make the
physics step follow it."""
import torch

from . import _integrators as I
from .common import Dynamics


class DiffDrive(Dynamics):
    def __init__(self, world, integration: str = "rk4"):
        super().__init__()
        I.check_integration(integration)
        self.dt = world.dt
        self.integration = integration
        self.world = world

    def f(self, state, u_command, ang_vel_command):
        theta = state[:, 2]
        return torch.stack((u_command * torch.cos(theta), u_command * torch.sin(theta), ang_vel_command), dim=-1)

    def euler(self, state, u_command, ang_vel_command):
        return I.increment(self.f, state, self.dt, "euler", u_command, ang_vel_command)

    def runge_kutta(self, state, u_command, ang_vel_command):
        return I.increment(self.f, state, self.dt, "rk4", u_command, ang_vel_command)

    @property
    def needed_action_size(self) -> int:
        return 2

    def process_action(self):
        u = self.agent.action.u
        delta = I.increment(self.f, I.pose(self.agent), self.dt, self.integration, u[:, 0], u[:, 1])
        I.apply_displacement(self.agent, delta[:, 0], delta[:, 1], delta[:, 2], self.dt)
