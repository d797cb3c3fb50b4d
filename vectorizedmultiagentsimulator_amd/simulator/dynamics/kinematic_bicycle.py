# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Kinematic bicycle (vmas/simulator/dynamics/kinematic_bicycle.py:13-112; Polack et al., IEEE IV
2017, eq. 2): the action is (speed, steering angle), the steering clamped to
+-max_steering_angle; slip angle beta = atan2(tan(delta) l_r / (l_f + l_r), 1), then
x' = v cos(theta + beta), y' = v sin(theta + beta), theta' = v / (l_f + l_r) cos(beta) tan(delta),
integrated over one step and turned into force / torque."""
import torch

from . import _integrators as I
from .common import Dynamics


class KinematicBicycle(Dynamics):
    def __init__(self, world, width: float, l_f: float, l_r: float, max_steering_angle: float,
                 integration: str = "rk4"):
        super().__init__()
        I.check_integration(integration)
        self.width = width
        self.l_f = l_f  # front axle to centre of gravity
        self.l_r = l_r  # rear axle to centre of gravity
        self.max_steering_angle = max_steering_angle
        self.dt = world.dt
        self.integration = integration
        self.world = world

    def f(self, state, steering_command, v_command):
        theta = state[:, 2]
        wheelbase = self.l_f + self.l_r
        beta = torch.atan2(torch.tan(steering_command) * self.l_r / wheelbase,
                           torch.tensor(1, device=self.world.device))
        dx = v_command * torch.cos(theta + beta)
        dy = v_command * torch.sin(theta + beta)
        dtheta = v_command / wheelbase * torch.cos(beta) * torch.tan(steering_command)
        return torch.stack((dx, dy, dtheta), dim=1)

    def euler(self, state, steering_command, v_command):
        return I.increment(self.f, state, self.dt, "euler", steering_command, v_command)

    def runge_kutta(self, state, steering_command, v_command):
        return I.increment(self.f, state, self.dt, "rk4", steering_command, v_command)

    @property
    def needed_action_size(self) -> int:
        return 2

    def process_action(self):
        u = self.agent.action.u
        steer = torch.clamp(u[:, 1], -self.max_steering_angle, self.max_steering_angle)
        delta = I.increment(self.f, I.pose(self.agent), self.dt, self.integration, steer, u[:, 0])
        I.apply_displacement(self.agent, delta[:, 0], delta[:, 1], delta[:, 2], self.dt)
