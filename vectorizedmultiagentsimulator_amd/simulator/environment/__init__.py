from enum import Enum

from .environment import Environment


class Wrapper(Enum):
    """Wrapper selector of make_env (environment/__init__.py:9-33).  The RL-library wrappers are
    outside the MI355X engine's scope; selecting one raises."""

    RLLIB = 0
    GYM = 1
    GYMNASIUM = 2
    GYMNASIUM_VEC = 3

    def get_env(self, env: Environment, **kwargs):
        raise NotImplementedError(f"the {self.name} wrapper is not provided by the MI355X engine")
