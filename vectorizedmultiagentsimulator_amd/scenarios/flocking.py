# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Flocking: agents flock around a scripted target agent among static obstacles.

Workload of BASELINE config C5.  Restates vmas/scenarios/flocking.py:18-206.  The target is an
Agent driven by an action script (a circle); each policy agent has a 12-ray LIDAR that sees the
non-agent entities (the obstacles).
"""
from typing import Dict

import torch
from torch import Tensor

from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Landmark, Sphere, World
from vectorizedmultiagentsimulator_amd.simulator.heuristic_policy import BaseHeuristicPolicy
from vectorizedmultiagentsimulator_amd.simulator.scenario import BaseScenario
from vectorizedmultiagentsimulator_amd.simulator.sensors import Lidar
from vectorizedmultiagentsimulator_amd.simulator.utils import Color, ScenarioUtils, X, Y


class Scenario(BaseScenario):
    def make_world(self, batch_dim: int, device: torch.device, **kwargs):
        n_agents = kwargs.pop("n_agents", 4)
        n_obstacles = kwargs.pop("n_obstacles", 5)
        self._min_dist_between_entities = kwargs.pop("min_dist_between_entities", 0.15)
        self.n_lidar_rays = kwargs.pop("n_lidar_rays", 12)
        self.collision_reward = kwargs.pop("collision_reward", -0.1)
        self.dist_shaping_factor = kwargs.pop("dist_shaping_factor", 1)
        ScenarioUtils.check_kwargs_consumed(kwargs)

        self.plot_grid = True
        self.desired_distance = 0.1
        self.min_collision_distance = 0.005
        self.x_dim = 1
        self.y_dim = 1

        world = World(batch_dim, device, collision_force=400, substeps=5)
        self._target = Agent(name="target", collide=True, color=Color.GREEN, render_action=True,
                             action_script=self.action_script_creator())
        world.add_agent(self._target)

        def not_an_agent(e):
            return not isinstance(e, Agent)

        for i in range(n_agents):
            agent = Agent(name=f"agent_{i}", collide=True,
                          sensors=[Lidar(world, n_rays=self.n_lidar_rays, max_range=0.2, entity_filter=not_an_agent)],
                          render_action=True)
            agent.collision_rew = torch.zeros(batch_dim, device=device)
            agent.dist_rew = agent.collision_rew.clone()
            world.add_agent(agent)

        self.obstacles = []
        for i in range(n_obstacles):
            obstacle = Landmark(name=f"obstacle_{i}", collide=True, movable=False,
                                shape=Sphere(radius=0.1), color=Color.RED)
            world.add_landmark(obstacle)
            self.obstacles.append(obstacle)
        return world

    def action_script_creator(self):
        def action_script(agent, world):
            t = self.t / 30
            agent.action.u = torch.stack([torch.cos(t), torch.sin(t)], dim=1)

        return action_script

    def _mean_sq_dist_error(self, agent, env_index=None):
        others = [a for a in self.world.agents if a != agent]
        if env_index is None:
            d = torch.stack([torch.linalg.vector_norm(agent.state.pos - a.state.pos, dim=-1) for a in others], dim=1)
        else:
            d = torch.stack(
                [torch.linalg.vector_norm(agent.state.pos[env_index] - a.state.pos[env_index]) for a in others], dim=0
            )
        return (d - self.desired_distance).pow(2).mean(-1) * self.dist_shaping_factor

    def reset_world_at(self, env_index: int = None):
        w = self.world
        n = 1 if env_index is not None else w.batch_dim
        target_pos = torch.zeros((n, w.dim_p), device=w.device, dtype=torch.float32)
        target_pos[:, Y] = -self.y_dim
        self._target.set_pos(target_pos, batch_index=env_index)
        ScenarioUtils.spawn_entities_randomly(
            self.obstacles + w.policy_agents, w, env_index, self._min_dist_between_entities,
            x_bounds=(-self.x_dim, self.x_dim), y_bounds=(-self.y_dim, self.y_dim),
            occupied_positions=target_pos.unsqueeze(1),
        )
        for agent in w.policy_agents:
            if env_index is None:
                agent.distance_shaping = self._mean_sq_dist_error(agent)
            else:
                agent.distance_shaping[env_index] = self._mean_sq_dist_error(agent, env_index)
        if env_index is None:
            self.t = torch.zeros(w.batch_dim, device=w.device)
        else:
            self.t[env_index] = 0

    def reward(self, agent: Agent):
        w = self.world
        if w.policy_agents.index(agent) == 0:
            self.t += 1
            if self.collision_reward != 0:
                for a in w.policy_agents:
                    a.collision_rew[:] = 0
                for i, a in enumerate(w.agents):
                    for j, b in enumerate(w.agents):
                        if j <= i:
                            continue
                        collision = w.get_distance(a, b) <= self.min_collision_distance
                        add = torch.where(collision, float(self.collision_reward), 0.0)
                        if a.action_script is None:
                            a.collision_rew += add
                        if b.action_script is None:
                            b.collision_rew += add
        agents_dist_shaping = self._mean_sq_dist_error(agent)
        agent.dist_rew = agent.distance_shaping - agents_dist_shaping
        agent.distance_shaping = agents_dist_shaping
        return agent.collision_rew + agent.dist_rew

    def observation(self, agent: Agent):
        return torch.cat(
            [agent.state.pos, agent.state.vel, agent.state.pos - self._target.state.pos,
             agent.sensors[0].measure()],
            dim=-1,
        )

    def info(self, agent: Agent) -> Dict[str, Tensor]:
        return {"agent_collision_rew": agent.collision_rew, "agent_distance_rew": agent.dist_rew}


class HeuristicPolicy(BaseHeuristicPolicy):
    """Circle at r=0.3 and steer away from obstacles seen by the LIDAR."""

    def compute_action(self, observation: torch.Tensor, u_range: float) -> torch.Tensor:
        assert self.continuous_actions
        circle_origin = torch.zeros(1, 2, device=observation.device)
        circle_radius = 0.3
        current_pos = observation[:, :2]
        v = current_pos - circle_origin
        on_circle = circle_origin + v / torch.linalg.norm(v, dim=1).unsqueeze(1) * circle_radius
        normal = torch.stack([on_circle[:, Y], -on_circle[:, X]], dim=1)
        normal /= torch.linalg.norm(normal, dim=1).unsqueeze(1)
        normal *= 0.1
        des_pos = on_circle + normal
        lidar = observation[:, 6:18]
        object_visible = torch.any(lidar < 0.1, dim=1)
        _, object_dir_index = torch.min(lidar, dim=1)
        object_dir = object_dir_index / lidar.shape[1] * 2 * torch.pi
        object_vec = torch.stack([torch.cos(object_dir), torch.sin(object_dir)], dim=1)
        des_pos_object = current_pos - object_vec * 0.1
        des_pos[object_visible] = des_pos_object[object_visible]
        return torch.clamp((des_pos - current_pos) * 10, min=-u_range, max=u_range)
