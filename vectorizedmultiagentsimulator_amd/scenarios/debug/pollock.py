# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Pollock: many movable + rotatable spheres, lines and boxes -- every narrowphase class.

Parity fixture (restates vmas/scenarios/debug/pollock.py:15-97): all six pair classes with real
rotational dynamics, optional 16-ray LIDAR (vectorised or per-ray) as in tests/test_lidar.py.
"""
import torch

from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Box, Landmark, Line, Sphere, World
from vectorizedmultiagentsimulator_amd.simulator.scenario import BaseScenario
from vectorizedmultiagentsimulator_amd.simulator.sensors import Lidar
from vectorizedmultiagentsimulator_amd.simulator.utils import Color, ScenarioUtils


class Scenario(BaseScenario):
    def make_world(self, batch_dim: int, device: torch.device, **kwargs):
        self.n_agents = kwargs.pop("n_agents", 15)
        self.n_lines = kwargs.pop("n_lines", 15)
        self.n_boxes = kwargs.pop("n_boxes", 15)
        self.lidar = kwargs.pop("lidar", False)
        self.vectorized_lidar = kwargs.pop("vectorized_lidar", True)
        ScenarioUtils.check_kwargs_consumed(kwargs)

        self.agent_radius = 0.05
        self.line_length = 0.3
        self.box_length = 0.2
        self.box_width = 0.1
        self.world_semidim = 1
        self.min_dist_between_entities = 0.1

        world = World(batch_dim, device, dt=0.1, drag=0.25, substeps=5, collision_force=500,
                      x_semidim=self.world_semidim, y_semidim=self.world_semidim)
        for i in range(self.n_agents):
            world.add_agent(
                Agent(name=f"agent_{i}", shape=Sphere(radius=self.agent_radius), u_multiplier=0.7,
                      rotatable=True,
                      sensors=[Lidar(world, n_rays=16, max_range=0.5)] if self.lidar else [])
            )
        for i in range(self.n_lines):
            world.add_landmark(
                Landmark(name=f"line {i}", collide=True, movable=True, rotatable=True,
                         shape=Line(length=self.line_length), color=Color.BLACK)
            )
        for i in range(self.n_boxes):
            world.add_landmark(
                Landmark(name=f"box {i}", collide=True, movable=True, rotatable=True,
                         shape=Box(length=self.box_length, width=self.box_width), color=Color.RED)
            )
        return world

    def reset_world_at(self, env_index: int = None):
        bounds = (-self.world_semidim, self.world_semidim)
        ScenarioUtils.spawn_entities_randomly(
            self.world.agents + self.world.landmarks, self.world, env_index,
            self.min_dist_between_entities, bounds, bounds,
        )

    def reward(self, agent: Agent):
        return torch.zeros(self.world.batch_dim, device=self.world.device)

    def observation(self, agent: Agent):
        if not self.lidar:
            return torch.zeros(self.world.batch_dim, 1, device=self.world.device)
        return agent.sensors[0].measure(vectorized=self.vectorized_lidar)
