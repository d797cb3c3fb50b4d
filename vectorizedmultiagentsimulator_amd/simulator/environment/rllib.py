"""RLlib VectorEnv wrapper of an Environment (ref vmas/simulator/environment/rllib.py:26-251).

RLlib's vector API is per sub-environment: actions come as a list over envs of per-agent
actions, observations / infos go back per env, and the reward of an env is the mean over agents
(every agent's reward is kept in its info under "rewards").  Needs `ray` (rllib), as the
reference: an ImportError otherwise."""
from __future__ import annotations

import importlib.util
from typing import Dict, List, Optional

import numpy as np
import torch
from torch import Tensor

from ..utils import TorchUtils
from .environment import Environment

if importlib.util.find_spec("ray") is None:
    raise ImportError("RLLib is not installed. Please install it with `pip install ray[rllib]<=2.2`.")
from ray import rllib  # noqa: E402


class VectorEnvWrapper(rllib.VectorEnv):
    """Vector environment wrapper for rllib."""

    def __init__(self, env: Environment):
        assert not env.terminated_truncated, (
            "Rllib wrapper is not compatible with termination and truncation flags. Please set "
            "`terminated_truncated=False` in the VMAS environment.")
        self._env = env
        super().__init__(observation_space=env.observation_space, action_space=env.action_space,
                         num_envs=env.num_envs)

    @property
    def env(self):
        return self._env

    def vector_reset(self):
        return self._read_data(TorchUtils.to_numpy(self._env.reset()))[0]

    def reset_at(self, index: Optional[int] = None):
        assert index is not None
        return self._read_data(self._env.reset_at(index), env_index=index)[0]

    def vector_step(self, actions):
        obs, rews, dones, infos = TorchUtils.to_numpy(self._env.step(self._action_list_to_tensor(actions)))
        obs, infos, rews = self._read_data(obs, infos, rews)
        return obs, rews, dones, infos

    def seed(self, seed=None):
        return self._env.seed(seed)

    def try_render_at(self, index: Optional[int] = None, mode="human", agent_index_focus: Optional[int] = None,
                      visualize_when_rgb: bool = False, **kwargs):
        return self._env.render(mode=mode, env_index=0 if index is None else index,
                                agent_index_focus=agent_index_focus, visualize_when_rgb=visualize_when_rgb, **kwargs)

    def get_sub_environments(self) -> List[Environment]:
        return [self._env]

    def _action_list_to_tensor(self, list_in: List) -> List:
        """[env][agent] actions -> per-agent [num_envs, action_size] float32 tensors."""
        env = self._env
        if len(list_in) != self.num_envs:
            raise TypeError("Input action is not in correct format")
        actions = [torch.zeros(self.num_envs, env.get_agent_action_size(a), device=env.device, dtype=torch.float32)
                   for a in env.agents]
        for j in range(self.num_envs):
            assert len(list_in[j]) == env.n_agents, (
                f"Expecting actions for {env.n_agents} agents, got {len(list_in[j])} actions")
            for i in range(env.n_agents):
                size = env.get_agent_action_size(env.agents[i])
                act = torch.tensor(list_in[j][i], dtype=torch.float32, device=env.device)
                if act.dim() == 0:
                    assert size == 1, f"Action of agent {i} in env {j} is supposed to be an scalar int"
                else:
                    assert act.dim() == 1 and act.shape[0] == size, (
                        f"Action of agent {i} in env {j} hase wrong shape: expected {size}, got {act.shape[0]}")
                actions[i][j] = act
        return actions

    def _read_data(self, obs, info=None, reward=None, env_index: Optional[int] = None):
        """Per-env (obs, info, mean reward); all envs as lists when env_index is None."""
        if env_index is not None:
            return self._get_data_at_env_index(env_index, obs, info, reward)
        per_env = [self._get_data_at_env_index(j, obs, info, reward) for j in range(self.num_envs)]
        return ([p[0] for p in per_env], [p[1] for p in per_env] if info else None,
                [p[2] for p in per_env] if reward else None)

    def _get_data_at_env_index(self, env_index: int, obs, info=None, reward=None):
        env = self._env
        assert len(obs) == env.n_agents
        if isinstance(obs, Dict):
            keys = [a.name for a in env.agents]
            new_obs = {}
        elif isinstance(obs, List):
            keys = list(range(env.n_agents))
            new_obs = []
        else:
            raise ValueError(f"Unsupported obs type {obs}")
        total_rew = 0.0
        new_info = {"rewards": {}} if info else None
        for agent_index, (agent, key) in enumerate(zip(env.agents, keys)):
            o = self._get_agent_data_at_env_index(env_index, obs[key])
            if isinstance(new_obs, dict):
                new_obs[agent.name] = o
            else:
                new_obs.append(o)
            if info:
                new_info[agent.name] = self._get_agent_data_at_env_index(env_index, info[key])
            if reward:
                r = self._get_agent_data_at_env_index(env_index, reward[key])
                new_info["rewards"].update({agent_index: r})
                total_rew += r
        return new_obs, new_info, (total_rew / env.n_agents if reward else None)

    def _get_agent_data_at_env_index(self, env_index: int, agent_data):
        if isinstance(agent_data, (np.ndarray, Tensor)):
            assert agent_data.shape[0] == self._env.num_envs
            if agent_data.ndim == 1 or (agent_data.ndim == 2 and agent_data.shape[1] == 1):
                return agent_data[env_index].item()
            if isinstance(agent_data, Tensor):
                return agent_data[env_index].cpu().detach().numpy()
            return agent_data[env_index]
        if isinstance(agent_data, Dict):
            return {k: self._get_agent_data_at_env_index(env_index, v) for k, v in agent_data.items()}
        raise ValueError(f"Unsupported data type {agent_data}")
