# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Discovery: agents must cover targets (``agents_per_target`` at a time); covered targets respawn.

Workload of BASELINE config C4 (LIDAR-heavy).  Restates vmas/scenarios/discovery.py:23-265.
Each agent carries a target LIDAR (``n_lidar_rays_entities`` rays) and, with
``use_agent_lidar=True``, a second LIDAR that sees agents (``n_lidar_rays_agents`` rays).
"""
import ctypes
import os
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
    # re-bound by the first agent's reward before anything in the step reads them (ref
    # discovery.py reward, is_first): graph replays need not carry them (environment/_graph.py)
    _vmas_graph_write_only = frozenset({"time_rew", "agents_pos", "targets_pos", "agents_targets_dists",
                                        "agents_per_target", "covered_targets"})

    def make_world(self, batch_dim: int, device: torch.device, **kwargs):
        self.n_agents = kwargs.pop("n_agents", 5)
        self.n_targets = kwargs.pop("n_targets", 7)
        self.x_semidim = kwargs.pop("x_semidim", 1)
        self.y_semidim = kwargs.pop("y_semidim", 1)
        self._min_dist_between_entities = kwargs.pop("min_dist_between_entities", 0.2)
        self._lidar_range = kwargs.pop("lidar_range", 0.35)
        self._covering_range = kwargs.pop("covering_range", 0.25)
        self.use_agent_lidar = kwargs.pop("use_agent_lidar", False)
        self.n_lidar_rays_entities = kwargs.pop("n_lidar_rays_entities", 15)
        self.n_lidar_rays_agents = kwargs.pop("n_lidar_rays_agents", 12)
        self._agents_per_target = kwargs.pop("agents_per_target", 2)
        self.targets_respawn = kwargs.pop("targets_respawn", True)
        self.shared_reward = kwargs.pop("shared_reward", False)
        self.agent_collision_penalty = kwargs.pop("agent_collision_penalty", 0)
        self.covering_rew_coeff = kwargs.pop("covering_rew_coeff", 1.0)
        self.time_penalty = kwargs.pop("time_penalty", 0)
        ScenarioUtils.check_kwargs_consumed(kwargs)

        self._comms_range = self._lidar_range
        self.min_collision_distance = 0.005
        self.agent_radius = 0.05
        self.target_radius = self.agent_radius
        self.viewer_zoom = 1
        self.target_color = Color.GREEN

        world = World(batch_dim, device, x_semidim=self.x_semidim, y_semidim=self.y_semidim,
                      collision_force=500, substeps=2, drag=0.25)

        def sees_agents(e):
            return e.name.startswith("agent")

        def sees_targets(e):
            return e.name.startswith("target")

        for i in range(self.n_agents):
            sensors = [
                Lidar(world, n_rays=self.n_lidar_rays_entities, max_range=self._lidar_range,
                      entity_filter=sees_targets, render_color=Color.GREEN)
            ]
            if self.use_agent_lidar:
                sensors.append(
                    Lidar(world, angle_start=0.05, angle_end=2 * torch.pi + 0.05,
                          n_rays=self.n_lidar_rays_agents, max_range=self._lidar_range,
                          entity_filter=sees_agents, render_color=Color.BLUE)
                )
            agent = Agent(name=f"agent_{i}", collide=True, shape=Sphere(radius=self.agent_radius),
                          sensors=sensors)
            agent.collision_rew = torch.zeros(batch_dim, device=device)
            agent.covering_reward = agent.collision_rew.clone()
            world.add_agent(agent)

        self._targets = []
        for i in range(self.n_targets):
            target = Landmark(name=f"target_{i}", collide=True, movable=False,
                              shape=Sphere(radius=self.target_radius), color=self.target_color)
            world.add_landmark(target)
            self._targets.append(target)

        self.covered_targets = torch.zeros(batch_dim, self.n_targets, device=device)
        self.shared_covering_rew = torch.zeros(batch_dim, device=device)
        return world

    def reset_world_at(self, env_index: int = None):
        w = self.world
        placable = self._targets[: self.n_targets] + w.agents
        if env_index is None:
            self.all_time_covered_targets = torch.full((w.batch_dim, self.n_targets), False, device=w.device)
        else:
            self.all_time_covered_targets[env_index] = False
        ScenarioUtils.spawn_entities_randomly(
            entities=placable, world=w, env_index=env_index,
            min_dist_between_entities=self._min_dist_between_entities,
            x_bounds=(-w.x_semidim, w.x_semidim), y_bounds=(-w.y_semidim, w.y_semidim),
        )
        for target in self._targets[self.n_targets:]:
            target.set_pos(self.get_outside_pos(env_index), batch_index=env_index)

    def reward(self, agent: Agent):
        if _fused.enabled(self.world) and self._fused_plan() is not None:
            return self._fused_reward(agent)
        w = self.world
        is_first = agent == w.agents[0]
        is_last = agent == w.agents[-1]
        if is_first:
            self.time_rew = torch.full((w.batch_dim,), self.time_penalty, device=w.device)
            self.agents_pos = torch.stack([a.state.pos for a in w.agents], dim=1)
            self.targets_pos = torch.stack([t.state.pos for t in self._targets], dim=1)
            self.agents_targets_dists = torch.cdist(self.agents_pos, self.targets_pos)
            self.agents_per_target = torch.sum(
                (self.agents_targets_dists < self._covering_range).type(torch.int), dim=1
            )
            self.covered_targets = self.agents_per_target >= self._agents_per_target
            self.shared_covering_rew[:] = 0
            for a in w.agents:
                self.shared_covering_rew += self.agent_reward(a)
            scr = self.shared_covering_rew
            scr.copy_(torch.where(scr != 0, scr / 2, scr))
        return self._reward_tail(agent, is_last)

    def _reward_tail(self, agent, is_last):
        w = self.world
        agent.collision_rew[:] = 0
        if self.agent_collision_penalty != 0:  # adding a zero penalty has no effect
            for a in w.agents:
                if a != agent:
                    hit = w.get_distance(a, agent) < self.min_collision_distance
                    agent.collision_rew += torch.where(hit, float(self.agent_collision_penalty), 0.0)
        if is_last:
            self._respawn()
        covering_rew = agent.covering_reward if not self.shared_reward else self.shared_covering_rew
        return agent.collision_rew + covering_rew + self.time_rew

    def _respawn(self):
        w = self.world
        if self.targets_respawn and self._respawn_native():
            return
        if self.targets_respawn:
            occupied_agents = [self.agents_pos]
            for i, target in enumerate(self._targets):
                occupied_targets = [o.state.pos.unsqueeze(1) for o in self._targets if o is not target]
                occupied = torch.cat(occupied_agents + occupied_targets, dim=1)
                pos = ScenarioUtils.find_random_pos_for_entity(
                    occupied, env_index=None, world=w,
                    min_dist_between_entities=self._min_dist_between_entities,
                    x_bounds=(-w.x_semidim, w.x_semidim), y_bounds=(-w.y_semidim, w.y_semidim),
                )
                # in-place update of the target's state (read by the next LIDAR scans)
                covered = self.covered_targets[:, i].unsqueeze(-1)
                target.state.pos.copy_(torch.where(covered, pos.squeeze(1), target.state.pos))
        else:
            self.all_time_covered_targets += self.covered_targets
            for i, target in enumerate(self._targets):
                covered = self.covered_targets[:, i].unsqueeze(-1)
                target.state.pos.copy_(torch.where(covered, self.get_outside_pos(None), target.state.pos))

    def _respawn_native(self) -> bool:
        """The respawn loop above in one stream-ordered native call (vmas_spawn_targets: a kernel
        per target, the tries drawn on the device with the reference's numbers, each target's
        generator offset chained on the device) and ONE host read of the tries consumed -- in a
        graph-mode step one host hole instead of one per target.  False (the loop above runs)
        off the GPU or where the device draws cannot reproduce torch's (_uniform.mode)."""
        w = self.world
        ap = self.agents_pos
        dev = torch.device(w.device)
        if (dev.type != "cuda" or not _fused.enabled(w) or len(self._targets) > N.VMAS_SPAWN_MAX_TARGETS
                or ap.dim() != 3 or ap.shape[1] > 32 or ap.dtype != torch.float32
                or self.covered_targets.dtype != torch.bool):
            return False
        from vectorizedmultiagentsimulator_amd.simulator.environment import _uniform

        if _uniform.mode(dev, w.batch_dim) is None:
            return False
        args = (ap, self.covered_targets, float(self._min_dist_between_entities), float(w.x_semidim),
                float(w.y_semidim), *[t.state.pos for t in self._targets])
        deferred = deferred_respawn()
        dsink = getattr(w, "_deferred_sink", None) if deferred else None
        sink = getattr(w, "_hole_sink", None)
        if deferred and not torch.cuda.is_current_stream_capturing() and \
                getattr(self, "_spawn_channel", None) is None:
            self._spawn_channel = SpawnChannel(dev, len(self._targets), w.batch_dim)  # (pinned memory: not in a capture)
        ch = getattr(self, "_spawn_channel", None)
        if ch is not None and (ch.backup.shape[0] != len(self._targets) or ch.backup.shape[1] != w.batch_dim):
            ch = None
        if dsink is not None and ch is not None:
            # a graph-mode capture: the launch stays inside the step's graph
            dsink(DeferredRespawn(args, self._spawn_channel))
        elif sink is not None:  # (the segmented form: the host read is a hole of the step)
            sink(respawn_targets_native, args)
        else:
            respawn_targets_native(*args)
        for t in self._targets:  # written in place, as the reference's copy_
            _fused.bump_version(t.state.pos)
        return True

    # ---- fused program (GPU worlds; csrc/vmas_scenarios.hip k_discovery_reward / _obs) ---------
    # The first agent's reward call runs ONE launch for the reward block above (the stacks, the
    # cdist distances, agents_per_target, covered_targets, every agent's covering_reward, the
    # shared reward, time_rew and every agent's reward); the last agent's call still respawns the
    # covered targets through the spawn sampler (host holes).  The first observation call -- after
    # the respawn, as in the reference -- runs ONE launch for every agent's observation and both
    # LIDARs.  The other calls hand out the precomputed tensors while their inputs are unchanged
    # (_fused.state_key), else fall back to the reference's per-call program.

    def _fused_plan(self):
        w = self.world
        sig = (tuple(id(e) for e in w.entities), w.batch_dim, self.agent_collision_penalty)
        plan = getattr(self, "_fplan", None)
        if plan is not None and plan[0] == sig:
            return plan[1]
        info = None
        ents, agents = w.entities, w.agents
        ok = (self.agent_collision_penalty == 0 and 1 <= len(agents) <= N.VMAS_DISC_MAX_AGENTS
              and len(self._targets) <= N.VMAS_DISC_MAX_TARGETS and len(ents) <= N.VMAS_DISC_MAX_ENTITIES
              and all(type(e.shape).__name__ == "Sphere" for e in ents))
        masks, n_rays = [], []
        if ok:
            nl = len(agents[0].sensors)
            ok = 1 <= nl <= N.VMAS_DISC_MAX_LIDARS
            for si in range(nl if ok else 0):
                m = None
                for a in agents:
                    if len(a.sensors) != nl or type(a.sensors[si]).__name__ != "Lidar":
                        ok = False
                        break
                    s = a.sensors[si]
                    am = sum(1 << k for k, e in enumerate(ents) if e is not a and s.entity_filter(e))
                    am |= (1 << ents.index(a)) if s.entity_filter(a) else 0
                    for e in ents:
                        if e is not a and s.entity_filter(e):
                            assert e.collides(a) and a.collides(e), "Rays are only casted among collidables"
                    if m is None:
                        m, R, mr = am, s._angles.shape[-1], s._max_range
                    if am != m or s._angles.shape != (w.batch_dim, R) or s._max_range != mr:
                        ok = False
                        break
                if not ok:
                    break
                masks.append(m)
                n_rays.append(R)
        if ok:
            info = {"masks": masks, "n_rays": n_rays, "agent_entity": [ents.index(a) for a in agents],
                    "target_entity": [ents.index(t) for t in self._targets]}
        self._fplan = (sig, info)
        return info

    def _fused_io(self, what: int, keep: list):
        w = self.world
        plan = self._fused_plan()
        dev = torch.device(w.device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        io = N.VmasDiscoveryIO()
        io.batch, io.n_agents, io.n_targets, io.what = w.batch_dim, len(w.agents), len(self._targets), what
        io.covering_range = float(self._covering_range)
        io.covering_rew_coeff = float(self.covering_rew_coeff)
        io.time_penalty = float(self.time_penalty)
        io.time_int = 1 if (isinstance(self.time_penalty, int) and not isinstance(self.time_penalty, bool)) else 0
        io.time_penalty_i = int(self.time_penalty) if io.time_int else 0
        io.fast_lidar = 0 if _fused.EXACT_LIDAR else 1
        io.agents_per_target = int(self._agents_per_target)
        io.shared_reward = 1 if self.shared_reward else 0
        io.n_entities, io.n_lidars = len(w.entities), len(plan["masks"])
        for i, e in enumerate(w.entities):
            io.pos[i] = _fused.vec(_fused.f32(e.state.pos, dev), keep)
            io.radius[i] = float(torch.tensor(e.shape.radius, dtype=torch.float32))
        for i, k in enumerate(plan["agent_entity"]):
            io.agent_entity[i] = k
        for j, k in enumerate(plan["target_entity"]):
            io.target_entity[j] = k
        return io, dev

    def _fused_reward(self, agent: Agent):
        w = self.world
        i = w.agents.index(agent)
        is_last = agent == w.agents[-1]
        if i == 0:
            keep = []
            io, dev = self._fused_io(N.VMAS_SCN_REWARD, keep)
            B, A, T = w.batch_dim, len(w.agents), len(self._targets)
            int_time = bool(io.time_int)
            at = self.all_time_covered_targets
            fuse_done = (at.dtype is torch.bool and at.is_contiguous() and at.shape == (B, T) and at.device == dev)
            # (graph-mode capture: rewards / done written straight into each replay's fresh tensors)
            io.out_delta, direct = _fused.direct_outputs(w, (
                None, (torch.float32, (B,), A), (torch.bool, (B,), 1) if fuse_done else None))
            out = {
                "agents_pos": torch.empty(B, A, 2, device=dev), "targets_pos": torch.empty(B, T, 2, device=dev),
                "dists": torch.empty(B, A, T, device=dev), "per_target": torch.empty(B, T, device=dev, dtype=torch.int64),
                "covered": torch.empty(B, T, device=dev, dtype=torch.bool),
                "time_rew": torch.empty(B, device=dev, dtype=torch.int64 if int_time else torch.float32),
                "rewards": direct[1] or [torch.empty(B, device=dev) for _ in w.agents],
            }
            for k in ("agents_pos", "targets_pos", "dists", "per_target", "covered", "time_rew"):
                setattr(io, k, out[k].data_ptr())
            # (a graph capture whose respawn goes through the spawn channel: this launch stages the
            # channel's armed words for it -- the respawn launch then runs no clear kernel)
            ch = getattr(self, "_spawn_channel", None)
            if (ch is not None and self.targets_respawn and deferred_respawn()
                    and getattr(w, "_deferred_sink", None) is not None
                    and ch.backup.shape[0] == T and ch.backup.shape[1] == B):
                io.stage_in, io.stage_out = ch.d_in, ch.mx.data_ptr() + 4 * N.VMAS_SPAWN_RNG_WORD
                ch.prestaged = True
            # the step's other reductions over the targets, in the same launch: info's count of
            # covered targets and done() (handed out by _targets_covered_count / done while their
            # inputs are the same tensors at the same versions)
            out["count"] = torch.empty(B, device=dev, dtype=torch.int64)
            io.covered_count = out["count"].data_ptr()
            if fuse_done:
                out["done"] = direct[2][0] if direct[2] else torch.empty(B, device=dev, dtype=torch.bool)
                io.all_time, io.done = at.data_ptr(), out["done"].data_ptr()
            inplace = [self.shared_covering_rew] + [a.covering_reward for a in w.agents] + [a.collision_rew for a in w.agents]
            if any(t.dtype is not torch.float32 or not t.is_contiguous() or t.shape != (B,) or t.device != dev
                   for t in inplace):
                self._fc = None
                return self._torch_reward_fallback(agent)
            io.shared = self.shared_covering_rew.data_ptr()
            for k, a in enumerate(w.agents):
                io.covering[k] = a.covering_reward.data_ptr()
                io.collision[k] = a.collision_rew.data_ptr()
                io.rewards[k] = out["rewards"][k].data_ptr()
            _fused.check(_fused.lib().vmas_discovery_outputs(dev.index, ctypes.byref(io), _fused.stream(w)),
                         "vmas_discovery_outputs")
            for t in inplace:
                _fused.bump_version(t)
            self.time_rew = out["time_rew"]
            self.agents_pos, self.targets_pos = out["agents_pos"], out["targets_pos"]
            self.agents_targets_dists = out["dists"]
            self.agents_per_target, self.covered_targets = out["per_target"], out["covered"]
            self._fc = {"rew": dict(enumerate(out["rewards"])), "rew_key": self._rew_key()}
            self._cov_count = (out["covered"], out["covered"]._version, out["count"])
            self._fdone = (at, at._version, out["done"]) if fuse_done else None
        c = getattr(self, "_fc", None)
        if c is not None and i in c.get("rew", {}) and c["rew_key"] == self._rew_key():
            r = c["rew"].pop(i)
            if is_last:
                self._respawn()
            return r
        return self._torch_reward_fallback(agent)

    def _rew_key(self):
        w = self.world
        return _fused.state_key([self.shared_covering_rew, self.time_rew]
                                + [a.covering_reward for a in w.agents] + [a.collision_rew for a in w.agents])

    def _torch_reward_fallback(self, agent):
        """The reference's per-call reward of a non-first agent (or of a first agent whose
        operands the kernel does not take: the whole torch program)."""
        if agent == self.world.agents[0]:
            with _fused.disabled():
                return self.reward(agent)
        return self._reward_tail(agent, agent == self.world.agents[-1])

    def _obs_inputs(self):
        w = self.world
        ts = [e.state.pos for e in w.entities]
        for a in w.agents:
            ts += [a.state.vel, a.state.rot] + [s._angles for s in a.sensors]
        return ts

    def _fused_observation(self, agent: Agent):
        w = self.world
        i = w.agents.index(agent)
        c = getattr(self, "_fo", None)
        if c is None or i not in c["obs"] or c["key"] != _fused.state_key(self._obs_inputs()):
            keep = []
            io, dev = self._fused_io(N.VMAS_SCN_OBS, keep)
            plan = self._fused_plan()
            B = w.batch_dim
            W = 4 + sum(plan["n_rays"])
            io.out_delta, direct = _fused.direct_outputs(w, ((torch.float32, (B, W), len(w.agents)), None, None))
            obs = direct[0] or [torch.empty(B, W, device=dev) for _ in w.agents]
            lid = [[torch.empty(B, R, device=dev) for _ in w.agents] for R in plan["n_rays"]]
            for s, (m, R) in enumerate(zip(plan["masks"], plan["n_rays"])):
                io.n_rays[s], io.mask[s] = R, m
                io.max_range[s] = float(w.agents[0].sensors[s]._max_range)
                for k, a in enumerate(w.agents):
                    ang = _fused.f32(a.sensors[s]._angles, dev)
                    keep.append(ang)
                    io.angles[s][k], io.ang_s0[s][k], io.ang_s1[s][k] = ang.data_ptr(), ang.stride(0), ang.stride(1)
                    io.lidar[s][k] = lid[s][k].data_ptr()
            for k, a in enumerate(w.agents):
                io.vel[k] = _fused.vec(_fused.f32(a.state.vel, dev), keep)
                io.rot[k] = _fused.vec(_fused.f32(a.state.rot, dev), keep)
                io.obs[k] = obs[k].data_ptr()
            _fused.check(_fused.lib().vmas_discovery_outputs(dev.index, ctypes.byref(io), _fused.stream(w)),
                         "vmas_discovery_outputs")
            c = self._fo = {"key": _fused.state_key(self._obs_inputs()),
                            "obs": {k: (obs[k], [lid[s][k] for s in range(len(lid))]) for k in range(len(obs))}}
        o, ls = c["obs"].pop(i)
        for s, m in enumerate(ls):
            agent.sensors[s]._last_measurement = m
        return o

    def get_outside_pos(self, env_index):
        w = self.world
        shape = (1, w.dim_p) if env_index is not None else (w.batch_dim, w.dim_p)
        return torch.empty(shape, device=w.device).uniform_(-1000 * w.x_semidim, -10 * w.x_semidim)

    def agent_reward(self, agent):
        agent_index = self.world.agents.index(agent)
        agent.covering_reward[:] = 0
        targets_covered_by_agent = self.agents_targets_dists[:, agent_index] < self._covering_range
        num_covered = (targets_covered_by_agent * self.covered_targets).sum(dim=-1)
        agent.covering_reward += num_covered * self.covering_rew_coeff
        return agent.covering_reward

    def observation(self, agent: Agent):
        if _fused.enabled(self.world) and self._fused_plan() is not None:
            return self._fused_observation(agent)
        parts = [agent.state.pos, agent.state.vel, agent.sensors[0].measure()]
        if self.use_agent_lidar:
            parts.append(agent.sensors[1].measure())
        return torch.cat(parts, dim=-1)

    def info(self, agent: Agent) -> Dict[str, Tensor]:
        return {
            "covering_reward": agent.covering_reward if not self.shared_reward else self.shared_covering_rew,
            "collision_rew": agent.collision_rew,
            "targets_covered": self._targets_covered_count(),
        }

    def _targets_covered_count(self) -> Tensor:
        """covered_targets.sum(-1) (ref discovery.py info), computed once per covered_targets
        tensor and version: every agent's info holds the same count.  The reference sums it once
        per agent; the environment returns each info value cloned (and a captured step copies
        each output separately), so every agent still gets a tensor of its own -- one reduction
        per step instead of one cast + reduction per agent."""
        ct = self.covered_targets
        c = getattr(self, "_cov_count", None)
        if c is None or c[0] is not ct or c[1] != ct._version:
            c = self._cov_count = (ct, ct._version, ct.sum(-1))
        return c[2]

    def done(self):
        c = getattr(self, "_fdone", None)  # (computed by the reward launch, see _fused_reward)
        self._fdone = None
        at = self.all_time_covered_targets
        if c is not None and c[0] is at and at._version == c[1]:
            return c[2]
        return at.all(dim=-1)


class HeuristicPolicy(BaseHeuristicPolicy):
    """Circle at r=0.75; steer towards visible targets and away from close agents."""

    def compute_action(self, observation: torch.Tensor, u_range: float) -> torch.Tensor:
        assert self.continuous_actions
        circle_origin = torch.zeros(1, 2, device=observation.device)
        circle_radius = 0.75
        current_pos = observation[:, :2]
        v = current_pos - circle_origin
        on_circle = circle_origin + v / torch.linalg.norm(v, dim=1).unsqueeze(1) * circle_radius
        normal = torch.stack([on_circle[:, Y], -on_circle[:, X]], dim=1)
        normal /= torch.linalg.norm(normal, dim=1).unsqueeze(1)
        normal *= 0.1
        des_pos = on_circle + normal

        lidar_targets = observation[:, 4:19]
        target_visible = torch.any(lidar_targets < 0.3, dim=1)
        _, target_dir_index = torch.min(lidar_targets, dim=1)
        target_dir = target_dir_index / lidar_targets.shape[1] * 2 * torch.pi
        target_vec = torch.stack([torch.cos(target_dir), torch.sin(target_dir)], dim=1)
        des_pos_target = current_pos + target_vec * 0.1
        des_pos[target_visible] = des_pos_target[target_visible]

        if observation.shape[-1] > 19:
            lidar_agents = observation[:, 19:31]
            agent_visible = torch.any(lidar_agents < 0.15, dim=1)
            _, agent_dir_index = torch.min(lidar_agents, dim=1)
            agent_dir = agent_dir_index / lidar_agents.shape[1] * 2 * torch.pi
            agent_vec = torch.stack([torch.cos(agent_dir), torch.sin(agent_dir)], dim=1)
            des_pos_agent = current_pos - agent_vec * 0.1
            des_pos[agent_visible] = des_pos_agent[agent_visible]

        return torch.clamp((des_pos - current_pos) * 10, min=-u_range, max=u_range)


def spawn_max_tries() -> int:
    """Tries per target before the one-launch respawn hands an env over to the reference's loop:
    0 = the kernel's compiled limit; only the test override VMAS_SPAWN_TEST_MAX_TRIES sets another
    (tests of that hand-over)."""
    return int(os.environ.get("VMAS_SPAWN_TEST_MAX_TRIES", "0") or 0)


def spawn_scratch(batch: int, n_targets: int, device) -> Tensor:
    """Device words of the windowed spawn kernel (vmas_spawn_scratch_words)."""
    n = int(N.load_library().vmas_spawn_scratch_words(batch, n_targets))
    if n <= 0:
        raise ValueError(f"vmas_spawn_scratch_words({batch}, {n_targets})")
    return torch.empty(n, dtype=torch.int32, device=device)


def _spawn_launch(agents_pos: Tensor, covered: Tensor, min_dist: float, x_semidim: float, y_semidim: float,
                  target_pos, mx: Tensor, channel=None, backup: Tensor = None, scratch: Tensor = None,
                  prestaged: bool = False):
    """One vmas_spawn_targets launch on the current stream; returns (io, philox increment)."""
    import numpy as np

    from vectorizedmultiagentsimulator_amd.simulator.environment import _uniform

    dev = agents_pos.device
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    B, A = agents_pos.shape[0], agents_pos.shape[1]
    T = len(target_pos)
    gen = torch.cuda.default_generators[idx]
    f32 = lambda v: float(np.float32(v))  # noqa: E731 -- torch casts the bounds to float
    io = N.VmasSpawnTargetsIO()
    io.batch, io.n_agents, io.n_targets, io.mode = B, A, T, _uniform.mode(dev, B)
    io.agents = agents_pos.data_ptr()
    io.ag_s0, io.ag_s1, io.ag_s2 = agents_pos.stride()
    for i, p in enumerate(target_pos):
        io.pos[i] = p.data_ptr()
        io.pos_s0[i], io.pos_s1[i] = p.stride()
    cov = covered.view(torch.uint8)
    io.covered = cov.data_ptr()
    io.cov_s0, io.cov_s1 = cov.stride()
    io.min_dist = float(torch.tensor(min_dist, dtype=torch.float32))
    io.x_lo, io.x_hi, io.y_lo, io.y_hi = f32(-x_semidim), f32(x_semidim), f32(-y_semidim), f32(y_semidim)
    if channel is None:  # (through a channel the launch reads them at run time)
        io.seed, io.offset = gen.initial_seed(), gen.get_offset()
    io.max_accepted = mx.data_ptr()
    io.channel = channel
    io.max_tries = spawn_max_tries()
    io.backup = backup.data_ptr() if backup is not None else None
    if scratch is not None:
        io.scratch, io.scratch_words = scratch.data_ptr(), scratch.numel()
    io.prestaged = 1 if prestaged else 0
    inc = ctypes.c_uint64(0)
    N.check_aux(N.load_library().vmas_spawn_targets(idx, ctypes.byref(io), ctypes.byref(inc),
                                                      ctypes.c_void_p(torch.cuda.current_stream(idx).cuda_stream)),
                "vmas_spawn_targets")
    return io, inc.value


def _spawn_consumed(h, T: int, offset: int, inc: int, gen) -> None:
    """Advance the generator by the tries the reference loop consumes (h: the launch's maxima)."""
    gen.set_offset(offset + sum(1 if m == 0 else m + 2 for m in h[:T]) * 2 * inc)


def respawn_reference_loop(agents_pos: Tensor, covered: Tensor, min_dist: float, x_semidim: float, y_semidim: float,
                           target_pos) -> None:
    """The reference's respawn loop (ref discovery.py:180-204): for each target in order,
    find_random_pos_for_entity over every env against the agents and the other targets, and the
    covered envs take the new position.  The sampler is the generic one (ScenarioUtils: the same
    numbers and generator use, unbounded, a warning past 50 000 tries, as ref utils.py:285-317)."""
    from types import SimpleNamespace

    world = SimpleNamespace(batch_dim=agents_pos.shape[0], device=agents_pos.device)
    for i, tp in enumerate(target_pos):
        occupied = torch.cat([agents_pos] + [o.unsqueeze(1) for j, o in enumerate(target_pos) if j != i], dim=1)
        pos = ScenarioUtils._find_random_pos_native(occupied, None, world, min_dist, (-x_semidim, x_semidim),
                                                    (-y_semidim, y_semidim))
        tp.copy_(torch.where(covered[:, i].unsqueeze(-1), pos.squeeze(1), tp))


HANDOVERS = [0]  # (one-launch respawns redone in this process: bench.py reports it)
REFERENCE_LOOP = [0]  # (of those, redone by the reference's host loop, not the per-target kernels)
HANDOVER_LOG = []  # why each was redone (the first 16): bench.py reports it


def _note_handover(where: str, timed_out: bool, h, T: int) -> None:
    if len(HANDOVER_LOG) < 16:
        HANDOVER_LOG.append({"where": where, "timed_out": bool(timed_out), "unresolved": int(h[T]),
                             "error_word": int(h[T + 1]) if len(h) > T + 1 else None})


def _respawn_redo(args, backup: Tensor, offset: int, gen) -> None:
    """Undo a one-launch respawn that left an env unresolved after max_tries tries, or whose
    bounded wait timed out (a workgroup never ran: the co-residency the resident kernel assumes did
    not hold), and redo it with the reference's loop: the targets back from the launch's backup,
    the generator back to the launch's offset."""
    HANDOVERS[0] += 1
    targets = args[5:]
    for i, tp in enumerate(targets):
        tp.copy_(backup[i])
    gen.set_offset(offset)
    if _redo_per_target(args, offset, gen):
        return
    REFERENCE_LOOP[0] += 1
    respawn_reference_loop(*args[:5], targets)


def _redo_per_target(args, offset: int, gen) -> bool:
    """The hand-over's first resort: the same respawn through the per-target kernels (no window,
    no list of envs with a covered target -- the windowed chain holds ~480 of them, and the first
    step after a full reset at C4 has ~650), exact as well (tests/test_spawn.py).  False, with the
    targets and the generator back where they were, when that one leaves an env unresolved too."""
    agents_pos, covered, min_dist, xs, ys = args[:5]
    targets = args[5:]
    T = len(targets)
    mx = torch.zeros(N.spawn_words(T), dtype=torch.int32, device=agents_pos.device)
    bk = torch.empty((T, agents_pos.shape[0], 2), dtype=torch.float32, device=agents_pos.device)
    io, inc = _spawn_launch(agents_pos, covered, min_dist, xs, ys, targets, mx, backup=bk)
    h = mx[:N.VMAS_SPAWN_ERR_WORD + 1].tolist()
    if h[N.VMAS_SPAWN_ERR_WORD] or h[T]:
        for i, tp in enumerate(targets):
            tp.copy_(bk[i])
        gen.set_offset(offset)
        return False
    _spawn_consumed(h, T, io.offset, inc, gen)
    HANDOVER_LOG.append({"redone_by": "per-target kernels"}) if len(HANDOVER_LOG) < 16 else None
    return True


def deferred_respawn() -> bool:
    """Graph mode: the respawn captured inside the step's graph through a spawn channel
    (DeferredRespawn) instead of a host hole splitting the step in two graphs
    (VMAS_GRAPH_DEFERRED_SPAWN=0: the hole; read per call -- make_env loads scenario modules afresh)."""
    return os.environ.get("VMAS_GRAPH_DEFERRED_SPAWN", "1") != "0"


class SpawnChannel:
    """Owner of a vmas_spawn_channel (mapped pinned host words), created outside any capture."""

    def __init__(self, dev: torch.device, n_targets: int, batch: int):
        self.idx = dev.index if dev.index is not None else torch.cuda.current_device()
        # the launch's device words, owned here (allocated outside any capture: a buffer from a
        # capture's private pool was found overwritten after a later replay)
        self.mx = torch.zeros(N.spawn_words(n_targets), dtype=torch.int32, device=dev)
        self.backup = torch.empty((n_targets, batch, 2), dtype=torch.float32, device=dev)  # (see _respawn_redo)
        self.scratch = spawn_scratch(batch, n_targets, dev)
        ch = ctypes.c_void_p()
        N.check_aux(N.load_library().vmas_spawn_channel_create(self.idx, ctypes.byref(ch)), "vmas_spawn_channel_create")
        self.ptr = ch
        d_in = ctypes.c_void_p()
        N.check_aux(N.load_library().vmas_spawn_channel_in(ch, ctypes.byref(d_in)), "vmas_spawn_channel_in")
        self.d_in = d_in.value
        self.prestaged = False  # (the step's reward launch staged the armed words: see Scenario._fused_reward)
        self.seq = 0
        self.busy = None  # the DeferredRespawn with a launch in flight

    def __del__(self):
        try:
            if self.busy is not None:
                torch.cuda.synchronize(self.idx)
            N.load_library().vmas_spawn_channel_destroy(self.ptr)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


class DeferredRespawn:
    """The respawn of a graph-mode step, kept inside the step's one graph.  At capture, one
    vmas_spawn_targets launch through a spawn channel (mapped host words): the launch reads the
    generator's seed and offset at run time and publishes its per-target maxima there.  Each replay:
    ``arm`` (before the launch) writes the generator state into the channel; ``finish`` (after the
    step's other host work is queued) waits for the maxima and advances the generator exactly as
    the eager call does -- the step's one host wait, with the rest of the step still running on the
    device, instead of a mid-step graph break and a second graph launch (StepGraph._deferred)."""

    def __init__(self, args, channel: SpawnChannel):
        self.args = args
        self.chan = channel
        self.ch = channel.ptr
        self.idx = channel.idx
        self.T = len(args) - 5
        self.pending = None
        self.inc = 0
        self.offset = 0
        self.mx = None

    def capture(self):
        a = self.args
        self.mx = self.chan.mx
        _, self.inc = _spawn_launch(a[0], a[1], a[2], a[3], a[4], a[5:], self.mx, channel=self.ch,
                                    backup=self.chan.backup, scratch=self.chan.scratch, prestaged=self.chan.prestaged)
        self.chan.prestaged = False

    def arm(self):
        if self.chan.busy is not None:  # (an earlier replay never finished: drain it first)
            self.chan.busy.finish(apply=False)
        gen = torch.cuda.default_generators[self.idx]
        self.chan.seq = self.chan.seq % 0xFFFFFFFF + 1
        self.offset = gen.get_offset()
        N.check_aux(N.load_library().vmas_spawn_channel_arm(self.ch, gen.initial_seed(), self.offset, self.chan.seq),
                    "vmas_spawn_channel_arm")
        self.pending = self.chan.seq
        self.chan.busy = self

    def finish(self, apply: bool = True) -> bool:
        """Waits for the replayed launch's words and advances the generator.  Returns True when the
        launch left an env unresolved or its bounded wait timed out: the respawn was then undone
        and redone with the reference's loop (_respawn_redo), and the step's observations, computed
        inside the graph after the respawn, must be recomputed (StepGraph._finish_deferred)."""
        if self.pending is None:
            return False
        seq, self.pending = self.pending, None
        if self.chan.busy is self:
            self.chan.busy = None
        words = (ctypes.c_int32 * (self.T + 2))()
        rc = N.load_library().vmas_spawn_channel_wait(self.ch, seq, words, self.T,
                                                      ctypes.c_void_p(torch.cuda.current_stream(self.idx).cuda_stream))
        timed_out = False
        if rc < 0:
            torch.cuda.synchronize(self.idx)
            timed_out = self.mx is not None and bool(int(self.mx[N.VMAS_SPAWN_ERR_WORD].item()))
            if not timed_out:
                N.check_aux(rc, "vmas_spawn_channel_wait")
        h = list(words)
        if not apply:
            return False
        gen = torch.cuda.default_generators[self.idx]
        if timed_out or h[self.T + 1] or h[self.T]:
            _note_handover("channel", timed_out, h, self.T)
            _respawn_redo(self.args, self.chan.backup, self.offset, gen)
            return True
        _spawn_consumed(h, self.T, self.offset, self.inc, gen)
        return False



def respawn_targets_native(agents_pos: Tensor, covered: Tensor, min_dist: float, x_semidim: float, y_semidim: float,
                           *target_pos: Tensor, out: Tensor = None) -> Tensor:
    """Discovery's target respawn loop (_respawn) through vmas_spawn_targets: target i moves to
    find_random_pos_for_entity(occupied = agents + the other targets) where covered[:, i].
    Returns the device int32 words of the call (N.spawn_words: per-target max accepted tries, the
    count of envs that found no position, the launch's counters) after reading them once and
    advancing the device generator by the tries the reference loop consumes.  ``out``: the
    tensor of a graph-mode hole's replay."""
    dev = agents_pos.device
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    T = len(target_pos)
    mx = out if out is not None else torch.zeros(N.spawn_words(T), dtype=torch.int32, device=dev)  # (zeros: see k_spawn_clear)
    backup = torch.empty((T, agents_pos.shape[0], 2), dtype=torch.float32, device=dev)
    scratch = spawn_scratch(agents_pos.shape[0], T, dev)
    io, inc = _spawn_launch(agents_pos, covered, min_dist, x_semidim, y_semidim, target_pos, mx, backup=backup,
                            scratch=scratch)
    h = mx[:N.VMAS_SPAWN_ERR_WORD + 1].tolist()  # the step's one host wait (maxima, unresolved, error)
    gen = torch.cuda.default_generators[idx]
    if h[N.VMAS_SPAWN_ERR_WORD] or h[T]:
        _note_handover("eager", bool(h[N.VMAS_SPAWN_ERR_WORD]), h[:T + 1] + [h[N.VMAS_SPAWN_ERR_WORD]], T)
        _respawn_redo((agents_pos, covered, min_dist, x_semidim, y_semidim, *target_pos), backup, io.offset, gen)
        return mx
    _spawn_consumed(h, T, io.offset, inc, gen)
    return mx
