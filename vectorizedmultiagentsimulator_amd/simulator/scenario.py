# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""The Scenario plugin API (restates vmas/simulator/scenario.py:24-451).

Scenarios subclass ``BaseScenario`` and implement ``make_world``, ``reset_world_at``,
``observation`` and ``reward`` (optionally ``done``, ``info``, ``process_action``,
``pre_step``, ``post_step``), exactly as with the reference.
"""
import typing
from abc import ABC, abstractmethod
from typing import Optional

import torch
from torch import Tensor

from .core import Agent, World
from .utils import AGENT_INFO_TYPE, AGENT_OBS_TYPE, AGENT_REWARD_TYPE, INITIAL_VIEWER_SIZE, VIEWER_DEFAULT_ZOOM


class BaseScenario(ABC):
    def __init__(self):
        """Do not override."""
        self._world = None
        self.viewer_size = INITIAL_VIEWER_SIZE
        self.viewer_zoom = VIEWER_DEFAULT_ZOOM
        self.render_origin = (0.0, 0.0)
        self.plot_grid = False
        self.grid_spacing = 0.1
        self.visualize_semidims = True

    @property
    def world(self):
        assert self._world is not None, "You first need to set `self._world` in the `make_world` method"
        return self._world

    def to(self, device: torch.device):
        for attr, value in self.__dict__.items():
            if isinstance(value, Tensor):
                self.__dict__[attr] = value.to(device)
        self.world.to(device)

    def env_make_world(self, batch_dim: int, device: torch.device, **kwargs) -> World:
        # Do not override
        self._world = self.make_world(batch_dim, device, **kwargs)
        return self._world

    def env_reset_world_at(self, env_index: typing.Optional[int]):
        # Do not override
        self.world.reset(env_index)
        self.reset_world_at(env_index)

    def env_process_action(self, agent: Agent):
        # Do not override
        if agent.action_script is not None:
            agent.action_callback(self.world)
        self.process_action(agent)
        agent.dynamics.check_and_process_action()

    @abstractmethod
    def make_world(self, batch_dim: int, device: torch.device, **kwargs) -> World:
        raise NotImplementedError()

    @abstractmethod
    def reset_world_at(self, env_index: Optional[int] = None):
        raise NotImplementedError()

    @abstractmethod
    def observation(self, agent: Agent) -> AGENT_OBS_TYPE:
        raise NotImplementedError()

    @abstractmethod
    def reward(self, agent: Agent) -> AGENT_REWARD_TYPE:
        raise NotImplementedError()

    def done(self) -> Tensor:
        # ref scenario.py:300-328: a [batch_dim] all-False view expanded from one element.  The
        # element is made once per device and reused (the view is read-only, as the reference's
        # expanded tensor; a write through an earlier view bumps the version counter and a fresh
        # element is made): a captured step then holds no host-to-device copy of it per replay.
        w = self.world
        c = getattr(self, "_done_false", None)
        if c is None or c[0]._version != c[1] or c[0].device != torch.device(w.device):
            t = torch.tensor([False], device=w.device)
            c = self._done_false = (t, t._version)
        v = c[0].expand(w.batch_dim)
        v._vmas_constant = True  # (graph mode copies it from a contiguous copy made at capture)
        return v

    def info(self, agent: Agent) -> AGENT_INFO_TYPE:
        return {}

    def extra_render(self, env_index: int = 0):
        return []

    def top_layer_render(self, env_index: int = 0):
        return []

    def process_action(self, agent: Agent):
        return

    def pre_step(self):
        return

    def post_step(self):
        return
