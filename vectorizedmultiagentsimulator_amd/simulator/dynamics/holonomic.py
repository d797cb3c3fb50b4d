"""Holonomic dynamics (dynamics/holonomic.py:13-14): the force is the first two action entries."""
from .common import Dynamics


class Holonomic(Dynamics):
    @property
    def needed_action_size(self) -> int:
        return 2

    def process_action(self):
        self.agent.state.force = self.agent.action.u[:, : self.needed_action_size]
