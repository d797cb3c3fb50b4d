# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Sensors (restates vmas/simulator/sensors.py).  ``Lidar.measure`` runs one ray-cast kernel."""
from __future__ import annotations

import os

import typing
from abc import ABC, abstractmethod
from typing import Callable, Tuple, Union

import torch

from .utils import Color

if typing.TYPE_CHECKING:
    from .core import Agent, Entity, World


class Sensor(ABC):
    def __init__(self, world: "World"):
        super().__init__()
        self._world = world
        self._agent = None

    @property
    def agent(self):
        return self._agent

    @agent.setter
    def agent(self, agent: "Agent"):
        self._agent = agent

    @abstractmethod
    def measure(self):
        raise NotImplementedError

    def render(self, env_index: int = 0):
        raise NotImplementedError("rendering is not part of the MI355X engine")

    def to(self, device: torch.device):
        raise NotImplementedError


_EXPAND_ANGLES = os.environ.get("VMAS_LIDAR_EXPAND", "1") != "0"


class Lidar(Sensor):
    # graph mode (environment/_graph.py _write_only): measure() re-binds the measurement and nothing
    # of this class reads the previous one, so replays of a step do not carry it forward
    _vmas_graph_write_only = frozenset({"_last_measurement"})

    def __init__(
        self,
        world: "World",
        angle_start: float = 0.0,
        angle_end: float = 2 * torch.pi,
        n_rays: int = 8,
        max_range: float = 1.0,
        entity_filter: Callable[["Entity"], bool] = lambda _: True,
        render_color: Union[Color, Tuple[float, float, float]] = Color.GRAY,
        alpha: float = 1.0,
        render: bool = True,
    ):
        super().__init__(world)
        # sensors.py:60-69: n evenly spaced rays; a full turn drops the duplicated last angle
        if (angle_start - angle_end) % (torch.pi * 2) < 1e-5:
            angles = torch.linspace(angle_start, angle_end, n_rays + 1, device=self._world.device)[:n_rays]
        else:
            angles = torch.linspace(angle_start, angle_end, n_rays, device=self._world.device)
        # the reference repeats the row per env (sensors.py:69); the same values as a stride-0 view,
        # so the LIDAR kernels read one row (C4 / C5: 14 / 12.6 MB of angle reads per step less).
        # A per-env in-place edit of it now raises instead of writing; assigning a [B, n] tensor
        # to `_angles` still gives per-env angles.
        if _EXPAND_ANGLES:
            self._angles = angles.unsqueeze(0).expand(self._world.batch_dim, -1)
        else:  # (VMAS_LIDAR_EXPAND=0: the reference's repeated rows, an A/B knob)
            self._angles = angles.repeat(self._world.batch_dim, 1)
        self._max_range = max_range
        self._last_measurement = None
        self._render = render
        self._entity_filter = entity_filter
        self._render_color = render_color
        self._alpha = alpha

    def to(self, device: torch.device):
        self._angles = self._angles.to(device)

    @property
    def entity_filter(self):
        return self._entity_filter

    @entity_filter.setter
    def entity_filter(self, entity_filter):
        self._entity_filter = entity_filter

    @property
    def render_color(self):
        if isinstance(self._render_color, Color):
            return self._render_color.value
        return self._render_color

    @property
    def alpha(self):
        return self._alpha

    def measure(self, vectorized: bool = True):
        world = self._world
        from .core import World

        if not vectorized:
            dists = []
            for angle in self._angles.unbind(1):
                dists.append(
                    world.cast_ray(
                        self.agent, angle + self.agent.state.rot.squeeze(-1),
                        max_range=self._max_range, entity_filter=self.entity_filter,
                    )
                )
            measurement = torch.stack(dists, dim=1)
        elif type(world).cast_rays is World.cast_rays:
            # fused `self._angles + agent.state.rot` (sensors.py:115-120): one launch
            measurement = world.engine.cast_rays(
                self.agent, self._angles, self._max_range, self.entity_filter,
                rot_offset=self.agent.state.rot,
            )
        else:
            measurement = world.cast_rays(
                self.agent, self._angles + self.agent.state.rot,
                max_range=self._max_range, entity_filter=self.entity_filter,
            )
        self._last_measurement = measurement
        return measurement

    def set_render(self, render: bool):
        self._render = render
