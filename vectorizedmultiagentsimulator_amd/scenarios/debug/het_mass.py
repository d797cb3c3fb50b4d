# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Het mass: two agents whose masses are re-drawn on every reset.

Restates vmas/scenarios/debug/het_mass.py:18-113 -- the reference's case of a physical parameter
that changes while the world runs.  Here the world kernel takes masses as
kernel arguments, so a re-roll costs no recompilation (vmas_jit_world_set_params).
"""
import math

import numpy as np
import torch

from vectorizedmultiagentsimulator_amd.simulator.core import Agent, World
from vectorizedmultiagentsimulator_amd.simulator.scenario import BaseScenario
from vectorizedmultiagentsimulator_amd.simulator.utils import Color, ScenarioUtils, Y


class Scenario(BaseScenario):
    def make_world(self, batch_dim: int, device: torch.device, **kwargs):
        self.green_mass = kwargs.pop("green_mass", 4)
        self.blue_mass = kwargs.pop("blue_mass", 2)
        self.mass_noise = kwargs.pop("mass_noise", 1)
        ScenarioUtils.check_kwargs_consumed(kwargs)
        self.plot_grid = True

        world = World(batch_dim, device)
        self.green_agent = Agent(name="agent 0", collide=False, color=Color.GREEN, render_action=True,
                                 mass=self.green_mass, f_range=1)
        self.blue_agent = Agent(name="agent 1", collide=False, render_action=True, f_range=1)
        world.add_agent(self.green_agent)
        world.add_agent(self.blue_agent)
        self.max_speed = torch.zeros(batch_dim, device=device)
        self.energy_expenditure = self.max_speed.clone()
        return world

    def reset_world_at(self, env_index: int = None):
        # one draw per agent for the whole batch, from numpy's global generator (ref :50-55)
        self.blue_agent.mass = self.blue_mass + np.random.uniform(-self.mass_noise, self.mass_noise)
        self.green_agent.mass = self.green_mass + np.random.uniform(-self.mass_noise, self.mass_noise)
        shape = (1, self.world.dim_p) if env_index is not None else (self.world.batch_dim, self.world.dim_p)
        for agent in self.world.agents:
            agent.set_pos(torch.zeros(shape, device=self.world.device, dtype=torch.float32).uniform_(-1, 1),
                          batch_index=env_index)

    def process_action(self, agent: Agent):
        agent.action.u[:, Y] = 0

    def reward(self, agent: Agent):
        if agent == self.world.agents[0]:
            speeds = [torch.linalg.vector_norm(a.state.vel, dim=1) for a in self.world.agents]
            self.max_speed = torch.stack(speeds, dim=1).max(dim=1)[0]
            effort = [torch.linalg.vector_norm(a.action.u, dim=-1) / math.sqrt(self.world.dim_p * (a.f_range ** 2))
                      for a in self.world.agents]
            self.energy_expenditure = -torch.stack(effort, dim=1).sum(-1) * 0.17
        return self.max_speed + self.energy_expenditure

    def observation(self, agent: Agent):
        return torch.cat([agent.state.pos, agent.state.vel], dim=-1)

    def info(self, agent: Agent):
        return {"max_speed": self.max_speed, "energy_expenditure": self.energy_expenditure}
