# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Holonomic dynamics with a torque input (dynamics/holonomic_with_rot.py:8-15): the action is
(fx, fy, torque); force and torque go to the physics step as the agent's action inputs."""
from .common import Dynamics


class HolonomicWithRotation(Dynamics):
    @property
    def needed_action_size(self) -> int:
        return 3

    def process_action(self):
        u = self.agent.action.u
        self.agent.state.force = u[:, :2]
        self.agent.state.torque = u[:, 2].unsqueeze(-1)
