# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Balance: agents carry a line with a package on it towards a goal, under gravity.

Workload of BASELINE configs C1/C2.  Restates vmas/scenarios/balance.py:15-262 (world layout,
reset distribution and RNG call order, reward, observation, done, heuristic policy).
Entities (in World.entities order): goal (sphere, no collide), package (sphere, movable),
line (movable + rotatable), floor (static box), agents (spheres).
"""
import torch

from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Box, Landmark, Line, Sphere, World
from vectorizedmultiagentsimulator_amd.simulator.heuristic_policy import BaseHeuristicPolicy
from vectorizedmultiagentsimulator_amd.simulator.scenario import BaseScenario
from vectorizedmultiagentsimulator_amd.simulator.utils import Color, ScenarioUtils, Y


class Scenario(BaseScenario):
    def make_world(self, batch_dim: int, device: torch.device, **kwargs):
        self.n_agents = kwargs.pop("n_agents", 3)
        self.package_mass = kwargs.pop("package_mass", 5)
        self.random_package_pos_on_line = kwargs.pop("random_package_pos_on_line", True)
        ScenarioUtils.check_kwargs_consumed(kwargs)
        assert self.n_agents > 1

        self.line_length = 0.8
        self.agent_radius = 0.03
        self.shaping_factor = 100
        self.fall_reward = -10
        self.visualize_semidims = False

        world = World(batch_dim, device, gravity=(0.0, -0.05), y_semidim=1)
        for i in range(self.n_agents):
            world.add_agent(Agent(name=f"agent_{i}", shape=Sphere(self.agent_radius), u_multiplier=0.7))

        goal = Landmark(name="goal", collide=False, shape=Sphere(), color=Color.LIGHT_GREEN)
        world.add_landmark(goal)
        self.package = Landmark(
            name="package", collide=True, movable=True, shape=Sphere(), mass=self.package_mass,
            color=Color.RED,
        )
        self.package.goal = goal
        world.add_landmark(self.package)
        self.line = Landmark(
            name="line", shape=Line(length=self.line_length), collide=True, movable=True,
            rotatable=True, mass=5, color=Color.BLACK,
        )
        world.add_landmark(self.line)
        self.floor = Landmark(name="floor", collide=True, shape=Box(length=10, width=1), color=Color.WHITE)
        world.add_landmark(self.floor)

        self.pos_rew = torch.zeros(batch_dim, device=device, dtype=torch.float32)
        self.ground_rew = self.pos_rew.clone()
        return world

    def _column(self, env_index, low, high):
        n = 1 if env_index is not None else self.world.batch_dim
        return torch.zeros((n, 1), device=self.world.device, dtype=torch.float32).uniform_(low, high)

    def _const(self, env_index, value):
        n = 1 if env_index is not None else self.world.batch_dim
        return torch.full((n, 1), value, device=self.world.device, dtype=torch.float32)

    def reset_world_at(self, env_index: int = None):
        w = self.world
        half = self.line_length / 2
        goal_pos = torch.cat([self._column(env_index, -1.0, 1.0), self._column(env_index, 0.0, w.y_semidim)], dim=1)
        line_pos = torch.cat(
            [self._column(env_index, -1.0 + half, 1.0 - half),
             self._const(env_index, -w.y_semidim + self.agent_radius * 2)],
            dim=1,
        )
        if self.random_package_pos_on_line:
            lo, hi = -half + self.package.shape.radius, half - self.package.shape.radius
        else:
            lo, hi = 0.0, 0.0
        package_rel_pos = torch.cat(
            [self._column(env_index, lo, hi), self._const(env_index, self.package.shape.radius)], dim=1
        )
        for i, agent in enumerate(w.agents):
            spacing = (self.line_length - agent.shape.radius) / (self.n_agents - 1)
            offset = torch.tensor(
                [-(self.line_length - agent.shape.radius) / 2 + i * spacing, -self.agent_radius * 2],
                device=w.device, dtype=torch.float32,
            )
            agent.set_pos(line_pos + offset, batch_index=env_index)
        self.line.set_pos(line_pos, batch_index=env_index)
        self.package.goal.set_pos(goal_pos, batch_index=env_index)
        self.line.set_rot(torch.zeros(1, device=w.device, dtype=torch.float32), batch_index=env_index)
        self.package.set_pos(line_pos + package_rel_pos, batch_index=env_index)
        self.floor.set_pos(
            torch.tensor([0, -w.y_semidim - self.floor.shape.width / 2 - self.agent_radius], device=w.device),
            batch_index=env_index,
        )
        self.compute_on_the_ground()
        dist = torch.linalg.vector_norm(self.package.state.pos - self.package.goal.state.pos, dim=1)
        if env_index is None:
            self.global_shaping = dist * self.shaping_factor
        else:
            self.global_shaping[env_index] = dist[env_index] * self.shaping_factor

    def compute_on_the_ground(self):
        self.on_the_ground = self.world.is_overlapping(self.line, self.floor) + self.world.is_overlapping(
            self.package, self.floor
        )

    def reward(self, agent: Agent):
        if agent == self.world.agents[0]:
            self.pos_rew[:] = 0
            self.ground_rew[:] = 0
            self.compute_on_the_ground()
            self.package_dist = torch.linalg.vector_norm(self.package.state.pos - self.package.goal.state.pos, dim=1)
            self.ground_rew.masked_fill_(self.on_the_ground, self.fall_reward)  # no host sync
            global_shaping = self.package_dist * self.shaping_factor
            self.pos_rew = self.global_shaping - global_shaping
            self.global_shaping = global_shaping
        return self.ground_rew + self.pos_rew

    def observation(self, agent: Agent):
        package, line = self.package, self.line
        return torch.cat(
            [
                agent.state.pos,
                agent.state.vel,
                agent.state.pos - package.state.pos,
                agent.state.pos - line.state.pos,
                package.state.pos - package.goal.state.pos,
                package.state.vel,
                line.state.vel,
                line.state.ang_vel,
                line.state.rot % torch.pi,
            ],
            dim=-1,
        )

    def done(self):
        return self.on_the_ground + self.world.is_overlapping(self.package, self.package.goal)

    def info(self, agent: Agent):
        return {"pos_rew": self.pos_rew, "ground_rew": self.ground_rew}


class HeuristicPolicy(BaseHeuristicPolicy):
    """Push the line up while the package is below its goal (balance.py:225-253)."""

    def compute_action(self, observation: torch.Tensor, u_range: float) -> torch.Tensor:
        batch_dim = observation.shape[0]
        dist_package_goal = observation[:, 8:10]
        y_distance_ge_0 = dist_package_goal[:, Y] >= 0
        if self.continuous_actions:
            action_agent = torch.clamp(
                torch.stack([torch.zeros(batch_dim, device=observation.device), -dist_package_goal[:, Y]], dim=1),
                min=-u_range, max=u_range,
            )
            action_agent[:, Y][y_distance_ge_0] = 0
        else:
            action_agent = torch.full((batch_dim,), 4, device=observation.device)
            action_agent[y_distance_ge_0] = 0
        return action_agent
