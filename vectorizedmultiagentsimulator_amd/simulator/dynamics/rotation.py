# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Rotation-only dynamics (dynamics/roatation.py:8-15): the action is a torque."""
from .common import Dynamics


class Rotation(Dynamics):
    @property
    def needed_action_size(self) -> int:
        return 1

    def process_action(self):
        self.agent.state.torque = self.agent.action.u[:, 0].unsqueeze(-1)
