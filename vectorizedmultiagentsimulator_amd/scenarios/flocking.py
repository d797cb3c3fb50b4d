# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Flocking: agents flock around a scripted target agent among static obstacles.

Workload of BASELINE config C5.  Restates vmas/scenarios/flocking.py:18-206.  The target is an
Agent driven by an action script (a circle); each policy agent has a 12-ray LIDAR that sees the
non-agent entities (the obstacles).
"""
import ctypes
from typing import Dict

import torch
from torch import Tensor

from vectorizedmultiagentsimulator_amd import _native as N
from vectorizedmultiagentsimulator_amd.simulator import _fused
from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Landmark, Sphere, World
from vectorizedmultiagentsimulator_amd.simulator.heuristic_policy import BaseHeuristicPolicy
from vectorizedmultiagentsimulator_amd.simulator.scenario import BaseScenario
from vectorizedmultiagentsimulator_amd.simulator.sensors import Lidar
from vectorizedmultiagentsimulator_amd.simulator.utils import Color, ScenarioUtils, X, Y


class Scenario(BaseScenario):
    # agent.dist_rew is re-bound by the agent's reward before anything in the step reads it (info
    # reads it after the reward; distance_shaping is read: carried): graph replays need not carry
    # it (environment/_graph.py _write_only)
    _vmas_graph_write_only_agents = frozenset({"dist_rew"})

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
            if _fused.enabled(world) and self.t.dtype is torch.float32 and self.t.is_contiguous():
                # one native launch for the same values (vmas_flocking_target_action)
                u = torch.empty(world.batch_dim, 2, device=self.t.device, dtype=torch.float32)
                _fused.check(_fused.lib().vmas_flocking_target_action(
                    _fused.device_index(world), self.t.data_ptr(), world.batch_dim, 30.0, u.data_ptr(),
                    _fused.stream(world)), "vmas_flocking_target_action")
            else:
                t = self.t / 30
                u = torch.stack([torch.cos(t), torch.sin(t)], dim=1)
            # cos / sin: |u| <= 1 by construction, so the scripted-action range check (core.py
            # _range_proven) needs no device work and graph replays need no rollback for it
            u._vmas_abs_bound = 1.0
            agent.action.u = u

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
        if _fused.enabled(self.world) and self._fused_plan() is not None:
            return self._fused_reward(agent)
        return self._torch_reward(agent)

    def _torch_reward(self, agent: Agent):
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
        if _fused.enabled(self.world) and self._fused_plan() is not None:
            return self._fused_observation(agent)
        return torch.cat(
            [agent.state.pos, agent.state.vel, agent.state.pos - self._target.state.pos,
             agent.sensors[0].measure()],
            dim=-1,
        )

    def info(self, agent: Agent) -> Dict[str, Tensor]:
        return {"agent_collision_rew": agent.collision_rew, "agent_distance_rew": agent.dist_rew}

    # ---- fused program (GPU worlds; csrc/vmas_scenarios.hip k_flocking) ------------------------
    # The first policy agent's reward call runs ONE launch, a thread per (env, policy agent): the
    # reward block above for every policy agent (t += 1, the pairwise collision rewards, the
    # separation term, dist_rew / distance_shaping, the reward) and every policy agent's
    # observation with its LIDAR.  Each agent's own reward call then re-binds its dist_rew /
    # distance_shaping and returns its reward, its observation call returns its observation and
    # sets its sensor's last measurement -- while the inputs are unchanged (_fused.state_key);
    # otherwise the call recomputes, as the reference does on every call.

    def _fused_plan(self):
        w = self.world
        agents, pol = w.agents, w.policy_agents
        sig = (tuple(id(a) for a in agents), tuple(id(e) for e in w.entities), w.batch_dim)
        plan = getattr(self, "_fplan", None)
        if plan is not None and plan[0] == sig:
            return plan[1]
        info = None
        dev = torch.device(w.device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        ok = (2 <= len(agents) <= N.VMAS_FLOCK_MAX_AGENTS and len(pol) >= 1 and self._target in agents
              and all(type(a.shape).__name__ == "Sphere" for a in agents))
        if ok:
            tgts, R = None, None
            for a in pol:
                if not a.sensors or type(a.sensors[0]).__name__ != "Lidar":
                    ok = False
                    break
                s = a.sensors[0]
                ts = [e for e in w.entities if e is not a and s.entity_filter(e)]
                if tgts is None:
                    tgts, R = ts, s._angles.shape[-1]
                if ([id(e) for e in ts] != [id(e) for e in tgts] or s._angles.shape != (w.batch_dim, R)
                        or len(ts) > N.VMAS_SCN_MAX_RAY_TARGETS
                        or any(type(e.shape).__name__ != "Sphere" for e in ts)):
                    ok = False
                    break
                for e in ts:
                    assert e.collides(a) and a.collides(e), "Rays are only casted among collidables"
        mode = _fused.reduce_order(dev, len(agents) - 1) if ok else None
        if ok and mode is not None:
            info = {"dev": dev, "targets": tgts, "R": R, "mode": mode,
                    "policy": [agents.index(a) for a in pol]}
        self._fplan = (sig, info)
        return info

    def _fused_inputs(self):
        w = self.world
        ts = [a.state.pos for a in w.agents]
        for a in w.policy_agents:
            s = a.sensors[0]
            ts += [a.state.vel, a.state.rot, s._angles]
        ts += [e.state.pos for e in self._fplan[1]["targets"]]
        ts += [e.state.rot for e in self._fplan[1]["targets"]]
        return ts

    def _run_fused(self, what: int):
        w = self.world
        plan = self._fused_plan()
        dev = plan["dev"]
        B = w.batch_dim
        agents, pol = w.agents, w.policy_agents
        keep = []
        io = N.VmasFlockingIO()
        io.batch, io.n_all, io.n_policy, io.what = B, len(agents), len(pol), what
        io.target, io.n_rays, io.n_ray_targets, io.sum_mode = agents.index(self._target), plan["R"], len(plan["targets"]), plan["mode"]
        io.min_collision_distance = float(self.min_collision_distance)
        io.collision_reward = float(self.collision_reward)
        io.desired_distance = float(self.desired_distance)
        io.dist_shaping_factor = float(self.dist_shaping_factor)
        io.collide_reward_on = 1 if self.collision_reward != 0 else 0
        io.fast_lidar = 0 if _fused.EXACT_LIDAR else 1
        io.max_range = float(pol[0].sensors[0]._max_range)
        for i, a in enumerate(agents):
            io.agents[i] = _fused.ref(w, a, keep, 0)
            io.scripted[i] = 0 if a.action_script is None else 1
        for i, e in enumerate(plan["targets"]):
            io.ray_targets[i] = _fused.ray_target(w, e, keep, dev)
        out = {}
        # (graph-mode capture: obs / rewards written straight into each replay's fresh tensors)
        io.out_delta, direct = _fused.direct_outputs(w, (
            (torch.float32, (B, 6 + plan["R"]), len(pol)) if what & N.VMAS_SCN_OBS else None,
            (torch.float32, (B,), len(pol)) if what & N.VMAS_SCN_REWARD else None, None))
        if what & N.VMAS_SCN_REWARD:
            t = self.t
            if t.dtype is not torch.float32 or not t.is_contiguous() or t.device != dev:
                raise _NotFusable
            io.t = t.data_ptr()
            for k in ("shaping", "dist_rew", "rewards"):
                out[k] = [torch.empty(B, device=dev, dtype=torch.float32) for _ in pol]
            if direct[1]:
                out["rewards"] = direct[1]
        if what & N.VMAS_SCN_OBS:
            R = plan["R"]
            out["obs"] = direct[0] or [torch.empty(B, 6 + R, device=dev, dtype=torch.float32) for _ in pol]
            out["lidar"] = [torch.empty(B, R, device=dev, dtype=torch.float32) for _ in pol]
        for p, a in enumerate(pol):
            io.policy[p] = plan["policy"][p]
            if what & N.VMAS_SCN_REWARD:
                sh, cr = a.distance_shaping, a.collision_rew
                for x in (sh, cr):
                    if x.dtype is not torch.float32 or not x.is_contiguous() or x.shape != (B,) or x.device != dev:
                        raise _NotFusable
                keep.append(sh)
                io.shaping_in[p], io.collision_rew[p] = sh.data_ptr(), cr.data_ptr()
                io.shaping_out[p] = out["shaping"][p].data_ptr()
                io.dist_rew[p] = out["dist_rew"][p].data_ptr()
                io.rewards[p] = out["rewards"][p].data_ptr()
            if what & N.VMAS_SCN_OBS:
                s = a.sensors[0]
                io.vel[p] = _fused.vec(_fused.f32(a.state.vel, dev), keep)
                io.rot[p] = _fused.vec(_fused.f32(a.state.rot, dev), keep)
                ang = _fused.f32(s._angles, dev)
                keep.append(ang)
                io.angles[p], io.ang_s0[p], io.ang_s1[p] = ang.data_ptr(), ang.stride(0), ang.stride(1)
                io.obs[p] = out["obs"][p].data_ptr()
                io.lidar[p] = out["lidar"][p].data_ptr()
        _fused.check(_fused.lib().vmas_flocking_outputs(dev.index, ctypes.byref(io), _fused.stream(w)),
                     "vmas_flocking_outputs")
        if what & N.VMAS_SCN_REWARD:
            _fused.bump_version(self.t)
            if io.collide_reward_on:
                for a in pol:
                    _fused.bump_version(a.collision_rew)
        return out

    def _fused_reward(self, agent: Agent):
        w = self.world
        pol = w.policy_agents
        p = pol.index(agent)
        if p == 0:
            try:
                out = self._run_fused(N.VMAS_SCN_REWARD | N.VMAS_SCN_OBS)
            except _NotFusable:
                self._fc = None
                return self._torch_reward(agent)
            self._fc = {
                "key": _fused.state_key(self._fused_inputs()),
                "rew": {i: (out["shaping"][i], out["dist_rew"][i], out["rewards"][i],
                            _fused.state_key([a.distance_shaping, a.collision_rew])) for i, a in enumerate(pol)},
                "obs": {i: (out["obs"][i], out["lidar"][i]) for i in range(len(pol))},
            }
        c = getattr(self, "_fc", None)
        if c is not None and p in c["rew"]:
            sh, dr, r, k = c["rew"][p]
            if k == _fused.state_key([agent.distance_shaping, agent.collision_rew]) and c["key"] == _fused.state_key(
                    self._fused_inputs()):
                del c["rew"][p]
                agent.dist_rew = dr
                agent.distance_shaping = sh
                return r
        c = self._fc = None if c is None else {**c, "rew": {}}
        return self._torch_reward(agent)

    def _fused_observation(self, agent: Agent):
        p = self.world.policy_agents.index(agent)
        c = getattr(self, "_fc", None)
        if c is None or p not in c["obs"] or c["key"] != _fused.state_key(self._fused_inputs()):
            try:
                out = self._run_fused(N.VMAS_SCN_OBS)
            except _NotFusable:
                return torch.cat([agent.state.pos, agent.state.vel, agent.state.pos - self._target.state.pos,
                                  agent.sensors[0].measure()], dim=-1)
            c = self._fc = {"key": _fused.state_key(self._fused_inputs()), "rew": {},
                            "obs": {i: (out["obs"][i], out["lidar"][i]) for i in range(len(out["obs"]))}}
        o, lid = c["obs"].pop(p)
        agent.sensors[0]._last_measurement = lid
        return o


class _NotFusable(Exception):
    """An operand the fused kernel does not take (dtype / layout / device): the torch program runs."""


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
