# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Waterfall: a chain of agents joined by collidable line joints, boxes and a floor.

Parity fixture for joints (restates vmas/scenarios/debug/waterfall.py).
"""
import torch

from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Box, Landmark, Line, Sphere, World
from vectorizedmultiagentsimulator_amd.simulator.joints import Joint
from vectorizedmultiagentsimulator_amd.simulator.scenario import BaseScenario
from vectorizedmultiagentsimulator_amd.simulator.utils import Color, ScenarioUtils


class Scenario(BaseScenario):
    def make_world(self, batch_dim: int, device: torch.device, **kwargs):
        self.n_agents = kwargs.pop("n_agents", 5)
        self.with_joints = kwargs.pop("joints", True)
        ScenarioUtils.check_kwargs_consumed(kwargs)
        self.agent_dist = 0.1
        self.agent_radius = 0.04

        world = World(batch_dim, device, dt=0.1, drag=0.25, substeps=5, collision_force=500)
        for i in range(self.n_agents):
            world.add_agent(Agent(name=f"agent_{i}", shape=Sphere(radius=self.agent_radius),
                                  u_multiplier=0.7, rotatable=True))
        if self.with_joints:
            for i in range(self.n_agents - 1):
                world.add_joint(
                    Joint(world.agents[i], world.agents[i + 1], anchor_a=(1, 0), anchor_b=(-1, 0),
                          dist=self.agent_dist, rotate_a=True, rotate_b=True, collidable=True, width=0, mass=1)
                )
            landmark = Landmark(name="joined landmark", collide=True, movable=True, rotatable=True,
                                shape=Box(length=self.agent_radius * 2, width=0.3), color=Color.GREEN)
            world.add_landmark(landmark)
            world.add_joint(
                Joint(world.agents[-1], landmark, anchor_a=(1, 0), anchor_b=(-1, 0), dist=self.agent_dist,
                      rotate_a=False, rotate_b=False, collidable=True, width=0, mass=1)
            )
        for i in range(5):
            world.add_landmark(
                Landmark(name=f"landmark {i}", collide=True, movable=True, rotatable=True,
                         shape=Box(length=0.3, width=0.1), color=Color.RED)
            )
        world.add_landmark(Landmark(name="floor", collide=True, movable=False, shape=Line(length=2),
                                    color=Color.BLACK))
        return world

    def reset_world_at(self, env_index: int = None):
        w = self.world
        chain = w.agents + [w.landmarks[self.n_agents - 1]]
        for i, entity in enumerate(chain):
            entity.set_pos(
                torch.tensor([-0.2 + (self.agent_dist + 2 * self.agent_radius) * i, 1.0],
                             dtype=torch.float32, device=w.device),
                batch_index=env_index,
            )
        boxes = w.landmarks[(self.n_agents + 1) if self.with_joints else 0: -1]
        for i, landmark in enumerate(boxes):
            landmark.set_pos(
                torch.tensor([0.2 if i % 2 else -0.2, 0.6 - 0.3 * i], dtype=torch.float32, device=w.device),
                batch_index=env_index,
            )
            landmark.set_rot(
                torch.tensor([torch.pi / 4 if i % 2 else -torch.pi / 4], dtype=torch.float32, device=w.device),
                batch_index=env_index,
            )
        w.landmarks[-1].set_pos(torch.tensor([0, -1], dtype=torch.float32, device=w.device), batch_index=env_index)

    def reward(self, agent: Agent):
        return -torch.linalg.vector_norm(agent.state.pos - self.world.landmarks[-1].state.pos, dim=1)

    def observation(self, agent: Agent):
        return torch.cat(
            [agent.state.pos, agent.state.vel]
            + [landmark.state.pos - agent.state.pos for landmark in self.world.landmarks],
            dim=-1,
        )
