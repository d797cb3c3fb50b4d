"""Gymnasium wrapper of a vectorised Environment: the whole batch per call, spaces batched over
num_envs (ref vmas/simulator/environment/gym/gymnasium_vec.py:28-97).  No auto-reset or partial
reset (the reference warns about it too).  Needs `gymnasium` and `shimmy`."""
from __future__ import annotations

import importlib.util
import warnings
from typing import Optional

from ..environment import Environment
from .base import BaseGymWrapper

if importlib.util.find_spec("gymnasium") is None or importlib.util.find_spec("shimmy") is None:
    raise ImportError("Gymnasium or shimmy is not installed. Please install it with `pip install gymnasium shimmy`.")
import gymnasium as gym  # noqa: E402
from gymnasium.vector.utils import batch_space  # noqa: E402
from shimmy.openai_gym_compatibility import _convert_space  # noqa: E402


class GymnasiumVectorizedWrapper(gym.Env, BaseGymWrapper):
    metadata = Environment.metadata

    def __init__(self, env: Environment, return_numpy: bool = True, render_mode: str = "human"):
        BaseGymWrapper.__init__(self, env, return_numpy=return_numpy, vectorized=True)
        self._num_envs = self._env.num_envs
        assert self._env.terminated_truncated, (
            "GymnasiumWrapper is only compatible with termination and truncation flags. Please set "
            "`terminated_truncated=True` in the VMAS environment.")
        self.single_observation_space = _convert_space(self._env.observation_space)
        self.single_action_space = _convert_space(self._env.action_space)
        self.observation_space = batch_space(self.single_observation_space, n=self._num_envs)
        self.action_space = batch_space(self.single_action_space, n=self._num_envs)
        self.render_mode = render_mode
        warnings.warn(
            "The Gymnasium Vector wrapper currently does not have auto-resets or support partial resets. "
            "Individual environments will not be reset when they are done: only global resets are available. "
            "Prefer the VMAS API unless the scenario does not implement `done` (all sub-environments are then "
            "done at the same time).")

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
        obs, info = self._env.reset(return_info=True)
        d = self._convert_env_data(obs=obs, info=info)
        return d.obs, d.info

    def render(self, agent_index_focus: Optional[int] = None, visualize_when_rgb: bool = False, **kwargs):
        return self._env.render(mode=self.render_mode, agent_index_focus=agent_index_focus,
                                visualize_when_rgb=visualize_when_rgb, **kwargs)
