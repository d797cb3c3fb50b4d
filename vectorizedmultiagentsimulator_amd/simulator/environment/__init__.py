from enum import Enum

from .environment import Environment


class Wrapper(Enum):
    """Wrapper selector of make_env (ref vmas/simulator/environment/__init__.py:9-33).  Each
    wrapper module imports its RL library at import time (gym; gymnasium + shimmy; ray), as the
    reference does, so selecting one without the library installed raises ImportError."""

    RLLIB = 0
    GYM = 1
    GYMNASIUM = 2
    GYMNASIUM_VEC = 3

    def get_env(self, env: Environment, **kwargs):
        if self is Wrapper.RLLIB:
            from .rllib import VectorEnvWrapper

            return VectorEnvWrapper(env, **kwargs)
        if self is Wrapper.GYM:
            from .gym import GymWrapper

            return GymWrapper(env, **kwargs)
        if self is Wrapper.GYMNASIUM:
            from .gym.gymnasium import GymnasiumWrapper

            return GymnasiumWrapper(env, **kwargs)
        if self is Wrapper.GYMNASIUM_VEC:
            from .gym.gymnasium_vec import GymnasiumVectorizedWrapper

            return GymnasiumVectorizedWrapper(env, **kwargs)
        raise ValueError(self)
