"""Static dynamics (dynamics/static.py:8-15): no action input."""
from .common import Dynamics


class Static(Dynamics):
    @property
    def needed_action_size(self) -> int:
        return 0

    def process_action(self):
        pass
