"""Gymnasium wrapper of a single-env Environment with terminated / truncated flags
(ref vmas/simulator/environment/gym/gymnasium.py:13-88).  Needs `gymnasium` and `shimmy` (their
space conversion), as the reference: an ImportError otherwise."""
from __future__ import annotations

import importlib.util
from typing import Optional

from ..environment import Environment
from .base import BaseGymWrapper

if importlib.util.find_spec("gymnasium") is None or importlib.util.find_spec("shimmy") is None:
    raise ImportError("Gymnasium or shimmy is not installed. Please install it with `pip install gymnasium shimmy`.")
import gymnasium as gym  # noqa: E402
from shimmy.openai_gym_compatibility import _convert_space  # noqa: E402


class GymnasiumWrapper(gym.Env, BaseGymWrapper):
    metadata = Environment.metadata

    def __init__(self, env: Environment, return_numpy: bool = True, render_mode: str = "human"):
        BaseGymWrapper.__init__(self, env, return_numpy=return_numpy, vectorized=False)
        assert env.num_envs == 1, (
            "GymnasiumEnv wrapper only supports singleton VMAS environment! For vectorized environments, use "
            "vectorized wrapper with `wrapper=gymnasium_vec`.")
        assert self._env.terminated_truncated, (
            "GymnasiumWrapper is only compatible with termination and truncation flags. Please set "
            "`terminated_truncated=True` in the VMAS environment.")
        self.observation_space = _convert_space(self._env.observation_space)
        self.action_space = _convert_space(self._env.action_space)
        self.render_mode = render_mode

    @property
    def unwrapped(self) -> Environment:
        return self._env

    def step(self, action):
        obs, rews, terminated, truncated, info = self._env.step(self._action_list_to_tensor(action))
        d = self._convert_env_data(obs=obs, rews=rews, info=info, terminated=terminated, truncated=truncated)
        return d.obs, d.rews, d.terminated, d.truncated, d.info

    def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None):
        if seed is not None:
            self._env.seed(seed)
        obs, info = self._env.reset_at(index=0, return_info=True)
        d = self._convert_env_data(obs=obs, info=info)
        return d.obs, d.info

    def render(self, agent_index_focus: Optional[int] = None, visualize_when_rgb: bool = False, **kwargs):
        return self._env.render(mode=self.render_mode, env_index=0, agent_index_focus=agent_index_focus,
                                visualize_when_rgb=visualize_when_rgb, **kwargs)
