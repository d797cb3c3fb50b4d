"""Shared conversion logic of the single-env and vectorised Gym-style wrappers
(ref vmas/simulator/environment/gym/base.py:15-131).

A wrapper holds one Environment and turns its per-agent lists / dicts of [num_envs, ...] tensors
into what the RL library expects: for a non-vectorised wrapper (num_envs == 1) the env index 0 is
taken out and rewards / dones become Python scalars; with ``return_numpy`` tensors become numpy
arrays; list infos become a dict keyed by agent name."""
from __future__ import annotations

from abc import ABC, abstractmethod
from collections import namedtuple
from typing import List, Optional

import torch

from ...utils import TorchUtils, extract_nested_with_index
from ..environment import Environment

EnvData = namedtuple("EnvData", ["obs", "rews", "terminated", "truncated", "done", "info"])


class BaseGymWrapper(ABC):
    def __init__(self, env: Environment, return_numpy: bool, vectorized: bool):
        self._env = env
        self.return_numpy = return_numpy
        self.dict_spaces = env.dict_spaces
        self.vectorized = vectorized

    @property
    def env(self):
        return self._env

    def _maybe_to_numpy(self, tensor):
        return TorchUtils.to_numpy(tensor) if self.return_numpy else tensor

    def _convert_output(self, data, item: bool = False):
        """One output: env 0 (and .item() for scalars) unless vectorised, then numpy if asked."""
        if not self.vectorized:
            data = extract_nested_with_index(data, index=0)
            if item:
                return data.item()
        return self._maybe_to_numpy(data)

    def _compress_infos(self, infos):
        if isinstance(infos, dict):
            return infos
        if isinstance(infos, list):
            return {self._env.agents[i].name: info for i, info in enumerate(infos)}
        raise ValueError(f"Expected list or dictionary for infos but got {type(infos)}")

    def _convert_env_data(self, obs=None, rews=None, info=None, terminated=None, truncated=None, done=None):
        keys = list(obs.keys()) if self.dict_spaces else range(self._env.n_agents)
        for k in keys:
            if obs is not None:
                obs[k] = self._convert_output(obs[k])
            if info is not None:
                info[k] = self._convert_output(info[k])
            if rews is not None:
                rews[k] = self._convert_output(rews[k], item=True)
        flags = [None if f is None else self._convert_output(f, item=True) for f in (terminated, truncated, done)]
        return EnvData(obs=obs, rews=rews, terminated=flags[0], truncated=flags[1], done=flags[2],
                       info=self._compress_infos(info) if info is not None else None)

    def _action_list_to_tensor(self, list_in: List) -> List:
        """Per-agent actions (tensors or array-likes) as [num_envs, action_size] tensors on the
        env's device: float32 for continuous actions, int64 for discrete ones."""
        env = self._env
        assert len(list_in) == env.n_agents, f"Expecting actions for {env.n_agents} agents, got {len(list_in)} actions"
        dtype = torch.float32 if env.continuous_actions else torch.long
        out = []
        for agent, act in zip(env.agents, list_in):
            shape = (env.num_envs, env.get_agent_action_size(agent))
            if isinstance(act, torch.Tensor):
                out.append(act.to(dtype=dtype, device=env.device).reshape(shape))
            else:
                out.append(torch.tensor(act, device=env.device, dtype=dtype).reshape(shape))
        return out

    @abstractmethod
    def step(self, action):
        raise NotImplementedError

    @abstractmethod
    def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None):
        raise NotImplementedError

    @abstractmethod
    def render(self, agent_index_focus: Optional[int] = None, visualize_when_rgb: bool = False, **kwargs):
        raise NotImplementedError
