"""Rotation-only dynamics (dynamics/roatation.py:8-15): the action is a torque."""
from .common import Dynamics


class Rotation(Dynamics):
    @property
    def needed_action_size(self) -> int:
        return 1

    def process_action(self):
        self.agent.state.torque = self.agent.action.u[:, 0].unsqueeze(-1)
