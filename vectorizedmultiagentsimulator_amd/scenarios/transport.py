# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Transport: agents push heavy box packages onto a goal.

Workload of BASELINE config C3.  Restates vmas/scenarios/transport.py:15-190 (layout, reset,
reward, observation, done) and its dribbling heuristic policy (transport.py:193-350).
Entities: goal (sphere r=0.15, no collide), packages (movable boxes), agents (spheres).
"""
import ctypes

import torch

from vectorizedmultiagentsimulator_amd import _native as N
from vectorizedmultiagentsimulator_amd.simulator import _fused
from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Box, Landmark, Sphere, World
from vectorizedmultiagentsimulator_amd.simulator.heuristic_policy import BaseHeuristicPolicy
from vectorizedmultiagentsimulator_amd.simulator.scenario import BaseScenario
from vectorizedmultiagentsimulator_amd.simulator.utils import Color, ScenarioUtils


class Scenario(BaseScenario):
    # re-bound by the first agent's reward before anything in the step reads it: graph replays
    # need not carry it (environment/_graph.py)
    _vmas_graph_write_only = frozenset({"rew"})

    def make_world(self, batch_dim: int, device: torch.device, **kwargs):
        n_agents = kwargs.pop("n_agents", 4)
        self.n_packages = kwargs.pop("n_packages", 1)
        self.package_width = kwargs.pop("package_width", 0.15)
        self.package_length = kwargs.pop("package_length", 0.15)
        self.package_mass = kwargs.pop("package_mass", 50)
        ScenarioUtils.check_kwargs_consumed(kwargs)

        self.shaping_factor = 100
        self.world_semidim = 1
        self.agent_radius = 0.03
        bound = self.world_semidim + 2 * self.agent_radius + max(self.package_length, self.package_width)
        world = World(batch_dim, device, x_semidim=bound, y_semidim=bound)
        for i in range(n_agents):
            world.add_agent(Agent(name=f"agent_{i}", shape=Sphere(self.agent_radius), u_multiplier=0.6))
        goal = Landmark(name="goal", collide=False, shape=Sphere(radius=0.15), color=Color.LIGHT_GREEN)
        world.add_landmark(goal)
        self.packages = []
        for i in range(self.n_packages):
            package = Landmark(
                name=f"package {i}", collide=True, movable=True, mass=self.package_mass,
                shape=Box(length=self.package_length, width=self.package_width), color=Color.RED,
            )
            package.goal = goal
            self.packages.append(package)
            world.add_landmark(package)
        # the fused program is also compiled into the world's specialised module (csrc/vmas_programs.hpp):
        # the eager step launches it from there, a replayed step runs it as k_world's epilogue
        world._jit_epilogue = N.EPILOGUE_TRANSPORT
        return world

    def reset_world_at(self, env_index: int = None):
        w = self.world
        bounds = (-self.world_semidim, self.world_semidim)
        ScenarioUtils.spawn_entities_randomly(
            w.agents, w, env_index, min_dist_between_entities=self.agent_radius * 2,
            x_bounds=bounds, y_bounds=bounds,
        )
        occupied = torch.stack([agent.state.pos for agent in w.agents], dim=1)
        if env_index is not None:
            occupied = occupied[env_index].unsqueeze(0)
        goal = w.landmarks[0]
        ScenarioUtils.spawn_entities_randomly(
            [goal] + self.packages, w, env_index,
            min_dist_between_entities=max(
                p.shape.circumscribed_radius() + goal.shape.radius + 0.01 for p in self.packages
            ),
            x_bounds=bounds, y_bounds=bounds, occupied_positions=occupied,
        )
        for package in self.packages:
            package.on_goal = w.is_overlapping(package, package.goal)
            dist = torch.linalg.vector_norm(package.state.pos - package.goal.state.pos, dim=1)
            if env_index is None:
                package.global_shaping = dist * self.shaping_factor
            else:
                package.global_shaping[env_index] = dist[env_index] * self.shaping_factor

    def reward(self, agent: Agent):
        if _fused.enabled(self.world) and self._fused_ok():
            return self._fused_reward(agent)
        w = self.world
        if agent == w.agents[0]:
            self.rew = torch.zeros(w.batch_dim, device=w.device, dtype=torch.float32)
            for package in self.packages:
                package.dist_to_goal = torch.linalg.vector_norm(package.state.pos - package.goal.state.pos, dim=1)
                package.on_goal = w.is_overlapping(package, package.goal)
                red = torch.tensor(Color.RED.value, device=w.device, dtype=torch.float32)
                green = torch.tensor(Color.GREEN.value, device=w.device, dtype=torch.float32)
                package.color = torch.where(package.on_goal.unsqueeze(-1), green, red.expand(w.batch_dim, 3))
                package_shaping = package.dist_to_goal * self.shaping_factor
                # rew[~on_goal] += shaping delta, without a boolean-mask host sync
                self.rew += torch.where(package.on_goal, 0.0, package.global_shaping - package_shaping)
                package.global_shaping = package_shaping
        return self.rew

    def observation(self, agent: Agent):
        if _fused.enabled(self.world) and self._fused_ok():
            return self._fused_observation(agent)
        package_obs = []
        for package in self.packages:
            package_obs.append(package.state.pos - package.goal.state.pos)
            package_obs.append(package.state.pos - agent.state.pos)
            package_obs.append(package.state.vel)
            package_obs.append(package.on_goal.unsqueeze(-1))
        return torch.cat([agent.state.pos, agent.state.vel, *package_obs], dim=-1)

    def done(self):
        if _fused.enabled(self.world) and self._fused_ok():
            return self._fused_done()
        return torch.all(torch.stack([package.on_goal for package in self.packages], dim=1), dim=-1)

    # ---- fused program (GPU worlds; csrc/vmas_scenarios.hip k_transport) -----------------------
    # The first agent's reward call runs ONE launch: the reward block above (every package's
    # dist_to_goal, on_goal, colour, re-bound global_shaping; the shared rew), every agent's
    # observation and done().  Reward calls return self.rew as the reference does; observation /
    # done calls hand out the precomputed tensors while their inputs are unchanged
    # (_fused.state_key), else recompute.

    def _fused_ok(self) -> bool:
        w = self.world
        return (len(self.packages) <= N.VMAS_TRANSPORT_MAX_PACKAGES and len(w.agents) <= N.VMAS_TRANSPORT_MAX_AGENTS
                and all(type(p.shape).__name__ == "Box" and type(p.goal.shape).__name__ == "Sphere"
                        for p in self.packages))

    def _obs_inputs(self):
        ts = []
        for p in self.packages:
            ts += [p.state.pos, p.state.rot, p.goal.state.pos, p.state.vel, p.on_goal]
        for a in self.world.agents:
            ts += [a.state.pos, a.state.vel]
        return ts

    def _run_fused(self, what: int):
        w = self.world
        dev = torch.device(w.device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        B = w.batch_dim
        keep = []
        io = N.VmasTransportIO()
        io.batch, io.n_agents, io.n_packages, io.what = B, len(w.agents), len(self.packages), what
        io.shaping_factor = float(self.shaping_factor)
        for k in range(3):
            io.red[k], io.green[k] = Color.RED.value[k], Color.GREEN.value[k]
        out = {"dist": [], "on_goal": [], "color": [], "gs": []}
        # (graph-mode capture: obs / rew / done written straight into each replay's fresh tensors)
        io.out_delta, direct = _fused.direct_outputs(w, (
            (torch.float32, (B, 4 + 7 * len(self.packages)), len(w.agents)) if what & N.VMAS_SCN_OBS else None,
            (torch.float32, (B,), 1) if what & N.VMAS_SCN_REWARD else None,
            (torch.bool, (B,), 1) if what & N.VMAS_SCN_DONE else None))
        for i, p in enumerate(self.packages):
            io.package[i] = _fused.ref(w, p, keep, 0)
            io.goal[i] = _fused.ref(w, p.goal, keep, 0)
            io.package_vel[i] = _fused.vec(_fused.f32(p.state.vel, dev), keep)
            if what & N.VMAS_SCN_REWARD:
                gs = _fused.f32(p.global_shaping, dev)
                keep.append(gs)
                io.global_shaping[i], io.gs_s0[i] = gs.data_ptr(), gs.stride(0)
                for k, shape, dt in (("dist", (B,), torch.float32), ("on_goal", (B,), torch.bool),
                                     ("color", (B, 3), torch.float32), ("gs", (B,), torch.float32)):
                    out[k].append(torch.empty(shape, device=dev, dtype=dt))
                io.dist_to_goal[i] = out["dist"][i].data_ptr()
                io.on_goal[i] = out["on_goal"][i].data_ptr()
                io.color[i] = out["color"][i].data_ptr()
                io.global_shaping_out[i] = out["gs"][i].data_ptr()
            else:
                og = p.on_goal
                if og.dtype is not torch.bool or og.device != dev or not og.is_contiguous():
                    og = og.to(device=dev, dtype=torch.bool).contiguous()
                keep.append(og)
                io.on_goal_in[i] = og.data_ptr()
        if what & N.VMAS_SCN_REWARD:
            out["rew"] = direct[1][0] if direct[1] else torch.empty(B, device=dev, dtype=torch.float32)
            io.rew = out["rew"].data_ptr()
        if what & N.VMAS_SCN_OBS:
            W = 4 + 7 * len(self.packages)
            out["obs"] = direct[0] or [torch.empty(B, W, device=dev, dtype=torch.float32) for _ in w.agents]
            for i, a in enumerate(w.agents):
                io.agent_pos[i] = _fused.vec(_fused.f32(a.state.pos, dev), keep)
                io.agent_vel[i] = _fused.vec(_fused.f32(a.state.vel, dev), keep)
                io.obs[i] = out["obs"][i].data_ptr()
        if what & N.VMAS_SCN_DONE:
            out["done"] = direct[2][0] if direct[2] else torch.empty(B, device=dev, dtype=torch.bool)
            io.done = out["done"].data_ptr()
        jit = w.engine.jit_program(N.EPILOGUE_TRANSPORT)
        if jit is not None:  # (the world module's k_program_jit: the code a replay runs as k_world's epilogue)
            N.check_jit(_fused.lib().vmas_jit_program_outputs(jit, N.EPILOGUE_TRANSPORT, ctypes.byref(io),
                                                              _fused.stream(w)), "vmas_jit_program_outputs")
        else:
            _fused.check(_fused.lib().vmas_transport_outputs(dev.index, ctypes.byref(io), _fused.stream(w)),
                         "vmas_transport_outputs")
        if what & N.VMAS_SCN_REWARD:
            self.rew = out["rew"]
            for i, p in enumerate(self.packages):
                p.dist_to_goal = out["dist"][i]
                p.on_goal = out["on_goal"][i]
                p.color = out["color"][i]
                p.global_shaping = out["gs"][i]
        return out

    def _fused_reward(self, agent: Agent):
        if agent == self.world.agents[0]:
            out = self._run_fused(N.VMAS_SCN_REWARD | N.VMAS_SCN_OBS | N.VMAS_SCN_DONE)
            self._fc = {"key": _fused.state_key(self._obs_inputs()), "obs": dict(enumerate(out["obs"])),
                        "done": out["done"]}
        return self.rew

    def _fused_observation(self, agent: Agent):
        i = self.world.agents.index(agent)
        c = getattr(self, "_fc", None)
        if c is None or i not in c["obs"] or c["key"] != _fused.state_key(self._obs_inputs()):
            out = self._run_fused(N.VMAS_SCN_OBS)
            c = self._fc = {"key": _fused.state_key(self._obs_inputs()), "obs": dict(enumerate(out["obs"])),
                            "done": None}
        return c["obs"].pop(i)

    def _fused_done(self):
        c = getattr(self, "_fc", None)
        if c is not None and c["done"] is not None and c["key"] == _fused.state_key(self._obs_inputs()):
            d, c["done"] = c["done"], None
            return d
        return self._run_fused(N.VMAS_SCN_DONE)["done"]

    def _vmas_tail_sources(self):
        """The tensors the fused program writes through (sc1, csrc/vmas_programs.hpp tr_reward_done):
        a graph replay may copy them inside the same launch (environment/_graph.py _tail_ok)."""
        return [t for p in self.packages for t in (p.dist_to_goal, p.on_goal, p.color, p.global_shaping)]


class HeuristicPolicy(BaseHeuristicPolicy):
    """Hermite-spline "dribbling" towards a hit point behind the package."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.lookahead = 0.0
        self.start_vel_dist_from_target_ratio = 0.5
        self.start_vel_behind_ratio = 0.5
        self.start_vel_mag = 1.0
        self.hit_vel_mag = 1.0
        self.package_radius = 0.15 / 2
        self.agent_radius = -0.02
        self.dribble_slowdown_dist = 0.0
        self.speed = 0.95

    def compute_action(self, observation: torch.Tensor, u_range: float) -> torch.Tensor:
        self.n_env = observation.shape[0]
        self.device = observation.device
        agent_pos = observation[:, :2]
        package_pos = observation[:, 6:8] + agent_pos
        goal_pos = -observation[:, 4:6] + package_pos
        control = self.dribble(agent_pos, package_pos, goal_pos)
        control *= self.speed * u_range
        return torch.clamp(control, -u_range, u_range)

    def dribble(self, agent_pos, package_pos, goal_pos, agent_vel=None):
        package_disp = goal_pos - package_pos
        ball_dist = package_disp.norm(dim=-1)
        direction = package_disp / ball_dist[:, None]
        hit_pos = package_pos - direction * (self.package_radius + self.agent_radius)
        hit_vel = direction * self.hit_vel_mag
        start_vel = self.get_start_vel(hit_pos, hit_vel, agent_pos, self.start_vel_mag * 2)
        slowdown_mask = ball_dist <= self.dribble_slowdown_dist
        hit_vel[slowdown_mask, :] *= ball_dist[slowdown_mask, None] / self.dribble_slowdown_dist
        return self.get_action(target_pos=hit_pos, target_vel=hit_vel, curr_pos=agent_pos,
                               curr_vel=agent_vel, start_vel=start_vel)

    @staticmethod
    def _npr(n, r):
        if r > n:
            return 0
        ans = 1
        for k in range(n, max(1, n - r), -1):
            ans = ans * k
        return ans

    def hermite(self, p0, p1, p0dot, p1dot, u=0.0, deriv=0):
        u = u.reshape((-1,))
        U = torch.stack(
            [self._npr(3 - i, deriv) * (u ** max(0, 3 - i - deriv)) for i in range(4)], dim=1
        ).float()
        A = torch.tensor(
            [[2.0, -2.0, 1.0, 1.0], [-3.0, 3.0, -2.0, -1.0], [0.0, 0.0, 1.0, 0.0], [1.0, 0.0, 0.0, 0.0]],
            device=U.device,
        )
        P = torch.stack([p0, p1, p0dot, p1dot], dim=1)
        return (U[:, None, :] @ A[None, :, :] @ P).squeeze(1)

    def get_start_vel(self, pos, vel, start_pos, start_vel_mag):
        start_vel_mag = torch.as_tensor(start_vel_mag, device=self.device).view(-1)
        goal_disp = pos - start_pos
        goal_dist = goal_disp.norm(dim=-1)
        vel_mag = vel.norm(dim=-1)
        vel_dir = vel.clone()
        vel_dir[vel_mag > 0] /= vel_mag[vel_mag > 0, None]
        goal_dir = goal_disp / goal_dist[:, None]
        vel_dir_normal = torch.stack([-vel_dir[:, 1], vel_dir[:, 0]], dim=1)
        dot_prod = (goal_dir * vel_dir_normal).sum(dim=1)
        vel_dir_normal[dot_prod > 0, :] *= -1
        dist_behind_target = self.start_vel_dist_from_target_ratio * goal_dist
        point_dir = -vel_dir * self.start_vel_behind_ratio + vel_dir_normal * (1 - self.start_vel_behind_ratio)
        target_pos = pos + point_dir * dist_behind_target[:, None]
        target_disp = target_pos - start_pos
        target_dist = target_disp.norm(dim=1)
        start_vel_aug_dir = target_disp
        start_vel_aug_dir[target_dist > 0] /= target_dist[target_dist > 0, None]
        return start_vel_aug_dir * start_vel_mag[:, None]

    def get_action(self, target_pos, target_vel=None, start_pos=None, start_vel=None, curr_pos=None,
                   curr_vel=None):
        if curr_pos is None:
            curr_pos = torch.zeros(target_pos.shape, device=self.device)
        if curr_vel is None:
            curr_vel = torch.zeros(target_pos.shape, device=self.device)
        if start_pos is None:
            start_pos = curr_pos
        if target_vel is None:
            target_vel = torch.zeros(target_pos.shape, device=self.device)
        if start_vel is None:
            start_vel = self.get_start_vel(target_pos, target_vel, start_pos, self.start_vel_mag * 2)
        u_start = torch.ones(curr_pos.shape[0], device=self.device) * self.lookahead
        des_curr_pos = self.hermite(start_pos, target_pos, start_vel, target_vel, u=u_start, deriv=0)
        des_curr_vel = self.hermite(start_pos, target_pos, start_vel, target_vel, u=u_start, deriv=1)
        return 0.5 * (des_curr_pos - curr_pos) + 0.5 * (des_curr_vel - curr_vel)
