# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""ORACLE -- test infrastructure only (never imported by the product package).

A PyTorch-CPU restatement, written from the reference's files, of what one
``env.step(actions)`` computes around ``World.step`` (oracle/vmas_oracle.py holds that part):

  * the action side:  ``Environment._set_action``'s continuous branch
                      (vmas/simulator/environment/environment.py:615-760), ``Holonomic.process_action``
                      (vmas/simulator/dynamics/holonomic.py:13-14), the scripted-action range check
                      (core.py:965-981) and the force clamps of ``_apply_action_force``
                      (core.py:2017-2027);
  * the four benchmark scenarios' per-step programs (reward, observation, done, info, and the
    carried shaping state set at reset):
      balance    vmas/scenarios/balance.py:200-266
      transport  vmas/scenarios/transport.py:112-190
      discovery  vmas/scenarios/discovery.py:146-265 (the target respawn is checked, not drawn)
      flocking   vmas/scenarios/flocking.py:83-206
  * ``Lidar``'s ray angles (vmas/simulator/sensors.py:60-69, 115-120).

Independence: nothing here reads the product's scenario objects or their attributes.  Inputs are
the entity list and shapes of a world (by the reference's entity names), state snapshots taken
with ``vmas_oracle.snapshot``, the actions the caller passed in, and the scenario's make_world
kwargs (defaults restated from the reference's ``kwargs.pop`` lines).  Geometry (is_overlapping,
get_distance, cast_rays) goes through ``vmas_oracle.OracleWorld``.

Discrete outcomes (overlap, coverage, collision flags) switch at a distance threshold; a last-bit
difference of that distance between CPU and GPU arithmetic can flip one.  Every program therefore
also returns ``margin`` per env: the smallest |distance - threshold| of every flag it evaluated,
so a checker can certify a mismatch as a threshold crossing (tests/_scenario_parity.py).

Parity status: as vmas_oracle.py -- the reference may not be run here, so these
programs are pinned by the reference's behavioural tests restated in tests/ and by agreement with
the product's own torch restatements on CPU worlds (tests/test_scenario_oracle.py); parity against
reference outputs is unpinned.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import torch
from torch import Tensor

from . import vmas_oracle as O

INF = float("inf")


# ------------------------------------------------------------------------------------------------
# the action side
def to_tensor(value, action_size: int) -> Tensor:
    """Action._to_tensor (core.py:510-515): a scalar range / multiplier becomes one per column."""
    return torch.tensor(value if isinstance(value, Sequence) else [value] * action_size, dtype=torch.float32)


def set_action(action: Tensor, *, action_size: int, u_range, u_multiplier, dim_p: int = 2, dim_c: int = 0,
               silent: bool = True, clamp_action: bool = False, noise: Optional[Tensor] = None,
               c_noise: Optional[Tensor] = None):
    """Environment._set_action, continuous actions (environment.py:615-760).  ``u_range`` /
    ``u_multiplier``: the agent's parameters (scalar or per column); ``noise``: the
    ``randn(...) * u_noise`` term the reference adds (drawn by the caller), None when u_noise is 0;
    ``c_noise`` likewise for the communication action.  Returns (u, c); raises AssertionError
    where the reference's asserts fire."""
    action = action.detach().to("cpu").clone()  # 616-620
    assert not action.isnan().any()  # 621-623
    u_range_t = to_tensor(u_range, action_size)
    u_mult_t = to_tensor(u_multiplier, action_size)
    comms = dim_c > 0 and not silent
    assert action.shape[1] == action_size + (dim_c if not silent else 0)  # 631-634 (get_agent_action_size)
    comm_action = None
    if clamp_action:  # 635-646
        physical_action = action[..., :action_size]
        a_range = u_range_t.unsqueeze(0).expand(physical_action.shape)
        physical_action = physical_action.clamp(-a_range, a_range)
        if comms:
            comm_action = action[..., action_size:]  # (the unclamped view: 643)
            action = torch.cat([physical_action, comm_action.clamp(0, 1)], dim=-1)
        else:
            action = physical_action
    action_index = 0
    physical_action = action[:, action_index:action_index + action_size]  # 651
    action_index += dim_p  # 652
    assert not torch.any(torch.abs(physical_action) > u_range_t), "out of its range"  # 653-655
    u = physical_action.to(torch.float32)  # 657
    u = u * u_mult_t  # 709 (u *= multiplier: u is a fresh slice copy's values, same numbers)
    if noise is not None:  # 711-720
        u = u + noise.to("cpu", torch.float32)
    c = None
    if comms:  # 721-760 (continuous branch)
        if comm_action is None:
            comm_action = action[:, action_index:]
        assert not torch.any(comm_action > 1) and not torch.any(comm_action < 0), "Comm actions are out of range"
        c = comm_action
        if c_noise is not None:
            c = c + c_noise.to("cpu", torch.float32)
    return u, c


def holonomic_process_action(u: Tensor) -> Tensor:
    """Holonomic.process_action (holonomic.py:13-14): state.force = u[:, :2]."""
    return u[:, :2]


def apply_action_force(force: Tensor, max_f=None, f_range=None) -> Tensor:
    """The clamps of World._apply_action_force (core.py:2017-2027), written back to state.force."""
    if max_f is not None:
        force = O.clamp_with_norm(force, max_f)
    if f_range is not None:
        force = torch.clamp(force, -f_range, f_range)
    return force


def check_scripted_action(u: Tensor, u_multiplier, u_range, action_size: int) -> None:
    """Agent.action_callback's range check (core.py:978-981)."""
    assert ((u / to_tensor(u_multiplier, action_size)).abs() <= to_tensor(u_range, action_size)).all(), \
        "Scripted physical action is out of range"


# ------------------------------------------------------------------------------------------------
# Lidar (sensors.py:47-69, 115-120)
def lidar_angles(batch_dim: int, n_rays: int, angle_start: float = 0.0, angle_end: float = 2 * math.pi) -> Tensor:
    if (angle_start - angle_end) % (math.pi * 2) < 1e-5:
        angles = torch.linspace(angle_start, angle_end, n_rays + 1)[:n_rays]
    else:
        angles = torch.linspace(angle_start, angle_end, n_rays)
    return angles.repeat(batch_dim, 1)


class LidarSpec:
    """One Lidar: its rays are ``angles + agent.state.rot`` cast at ``max_range`` against the
    entities ``entity_filter`` admits (World.cast_rays)."""

    def __init__(self, batch_dim, n_rays, max_range, entity_filter, angle_start=0.0, angle_end=2 * math.pi):
        self.angles = lidar_angles(batch_dim, n_rays, angle_start, angle_end)
        self.max_range = max_range
        self.entity_filter = entity_filter

    def measure(self, ow: "O.OracleWorld", agent_index: int):
        rays = self.angles + ow.ents[agent_index].state.rot
        return ow.cast_rays(agent_index, rays, self.max_range, self.entity_filter), rays


# ------------------------------------------------------------------------------------------------
# helpers
def _norm(v: Tensor) -> Tensor:
    return torch.linalg.vector_norm(v, dim=-1)


def _overlap_margin(ow, a, b) -> Tensor:
    """|quantity - threshold| of World.is_overlapping(a, b) (core.py:1944-1968): the box-sphere
    test compares two distance pairs, every other pair compares get_distance with 0."""
    ka, kb = O._kind(a.shape), O._kind(b.shape)
    if {ka, kb} == {"Box", "Sphere"}:
        box, sphere = (a, b) if kb == "Sphere" else (b, a)
        cp = O.get_closest_point_box(box.state.pos, box.state.rot, box.shape.width, box.shape.length, sphere.state.pos)
        d_sc = _norm(sphere.state.pos - cp)
        d_sb = _norm(sphere.state.pos - box.state.pos)
        d_cb = _norm(box.state.pos - cp)
        return torch.minimum((d_sb - d_cb).abs(), (d_sc - (sphere.shape.radius + O.LINE_MIN_DIST)).abs())
    return ow.get_distance(a, b).abs()


class _Program:
    """Common frame: the world's entity table by name and the policy / scripted agent lists."""

    def __init__(self, world):
        self.world = world
        self.B = world.batch_dim
        self.names = [e.name for e in world.entities]
        self.agent_names = [a.name for a in world.agents]
        self.agent_set = {id(a) for a in world.agents}
        self.policy_names = [a.name for a in world.agents if a.action_script is None]

    def idx(self, name: str) -> int:
        return self.names.index(name)

    def ow(self, snap) -> "O.OracleWorld":
        return O.OracleWorld(self.world, snap)

    @staticmethod
    def ent(ow, i):
        return ow.ents[i]


# ------------------------------------------------------------------------------------------------
class Balance(_Program):
    """vmas/scenarios/balance.py.  kwargs: n_agents (3), package_mass (5),
    random_package_pos_on_line (True) -- make_world (15-19) reads no other."""

    shaping_factor = 100  # balance.py:26
    fall_reward = -10  # balance.py:27

    def __init__(self, world, **kw):
        super().__init__(world)
        self.global_shaping = None

    def _ents(self, ow):
        return (ow.ents[self.idx("package")], ow.ents[self.idx("goal")], ow.ents[self.idx("line")],
                ow.ents[self.idx("floor")])

    def reset(self, snap) -> None:
        """reset_world_at(None)'s global shaping (balance.py:201-207)."""
        package, goal, _, _ = self._ents(self.ow(snap))
        self.global_shaping = _norm(package.state.pos - goal.state.pos) * self.shaping_factor

    def step(self, pre_snap, snap) -> Dict:
        ow = self.ow(snap)
        package, goal, line, floor = self._ents(ow)
        B = self.B
        # reward (balance.py:222-240), first agent's call
        on_the_ground = ow.is_overlapping(line, floor) + ow.is_overlapping(package, floor)  # 217-220
        package_dist = _norm(package.state.pos - goal.state.pos)
        ground_rew = torch.zeros(B)
        ground_rew[on_the_ground] = self.fall_reward
        global_shaping = package_dist * self.shaping_factor
        pos_rew = self.global_shaping - global_shaping
        self.global_shaping = global_shaping
        rew = ground_rew + pos_rew
        obs, rews, infos = [], [], []
        for name in self.policy_names:
            agent = ow.ents[self.idx(name)]
            rews.append(rew)
            obs.append(torch.cat([  # balance.py:242-257
                agent.state.pos, agent.state.vel, agent.state.pos - package.state.pos,
                agent.state.pos - line.state.pos, package.state.pos - goal.state.pos, package.state.vel,
                line.state.vel, line.state.ang_vel, line.state.rot % torch.pi], dim=-1))
            infos.append({"pos_rew": pos_rew, "ground_rew": ground_rew})  # 264-266
        done = on_the_ground + ow.is_overlapping(package, goal)  # 259-262
        margin = torch.minimum(torch.minimum(_overlap_margin(ow, line, floor), _overlap_margin(ow, package, floor)),
                               _overlap_margin(ow, package, goal))
        return {"obs": obs, "rew": rews, "done": done, "info": infos, "margin": margin, "lidar": []}


# ------------------------------------------------------------------------------------------------
class Transport(_Program):
    """vmas/scenarios/transport.py.  kwargs: n_agents (4), n_packages (1), package_width (0.15),
    package_length (0.15), package_mass (50)."""

    shaping_factor = 100  # transport.py:23

    def __init__(self, world, n_packages: int = 1, **kw):
        super().__init__(world)
        self.packages = [f"package {i}" for i in range(n_packages)]  # transport.py:55-66
        self.global_shaping = {}

    def reset(self, snap) -> None:
        """reset_world_at(None)'s global shaping per package (transport.py:112-121)."""
        ow = self.ow(snap)
        goal = ow.ents[self.idx("goal")]
        for p in self.packages:
            pk = ow.ents[self.idx(p)]
            self.global_shaping[p] = _norm(pk.state.pos - goal.state.pos) * self.shaping_factor

    def step(self, pre_snap, snap) -> Dict:
        ow = self.ow(snap)
        goal = ow.ents[self.idx("goal")]
        B = self.B
        rew = torch.zeros(B)  # transport.py:134-138
        on_goal, margin = {}, torch.full((B,), INF)
        for p in self.packages:  # 140-161
            pk = ow.ents[self.idx(p)]
            dist_to_goal = _norm(pk.state.pos - goal.state.pos)
            on_goal[p] = ow.is_overlapping(pk, goal)
            margin = torch.minimum(margin, _overlap_margin(ow, pk, goal))
            package_shaping = dist_to_goal * self.shaping_factor
            m = ~on_goal[p]
            rew[m] += self.global_shaping[p][m] - package_shaping[m]
            self.global_shaping[p] = package_shaping
        obs, rews, infos = [], [], []
        for name in self.policy_names:
            agent = ow.ents[self.idx(name)]
            rews.append(rew)
            package_obs = []
            for p in self.packages:  # 165-181
                pk = ow.ents[self.idx(p)]
                package_obs += [pk.state.pos - goal.state.pos, pk.state.pos - agent.state.pos, pk.state.vel,
                                on_goal[p].unsqueeze(-1)]
            obs.append(torch.cat([agent.state.pos, agent.state.vel, *package_obs], dim=-1))
            infos.append({})  # BaseScenario.info (scenario.py:330-349)
        done = torch.all(torch.stack([on_goal[p] for p in self.packages], dim=1), dim=-1)  # 183-190
        return {"obs": obs, "rew": rews, "done": done, "info": infos, "margin": margin, "lidar": []}


# ------------------------------------------------------------------------------------------------
class Discovery(_Program):
    """vmas/scenarios/discovery.py (make_world kwargs 23-43, reference defaults)."""

    min_collision_distance = 0.005  # discovery.py:46

    def __init__(self, world, n_targets: int = 7, min_dist_between_entities: float = 0.2, lidar_range: float = 0.35,
                 covering_range: float = 0.25, use_agent_lidar: bool = False, n_lidar_rays_entities: int = 15,
                 n_lidar_rays_agents: int = 12, agents_per_target: int = 2, targets_respawn: bool = True,
                 shared_reward: bool = False, agent_collision_penalty: float = 0, covering_rew_coeff: float = 1.0,
                 time_penalty: float = 0, **kw):
        super().__init__(world)
        self.n_targets = n_targets
        self.min_dist = min_dist_between_entities
        self.covering_range = covering_range
        self.agents_per_target = agents_per_target
        self.targets_respawn = targets_respawn
        self.shared_reward = shared_reward
        self.penalty = agent_collision_penalty
        self.coeff = covering_rew_coeff
        self.time_penalty = time_penalty
        self.use_agent_lidar = use_agent_lidar
        self.targets = [f"target_{i}" for i in range(n_targets)]
        self.x_semidim, self.y_semidim = float(world.x_semidim), float(world.y_semidim)
        B = world.batch_dim
        # discovery.py:77-101: a target LIDAR (15 rays) and, with use_agent_lidar, an agent LIDAR
        self.lidars = [LidarSpec(B, n_lidar_rays_entities, lidar_range, lambda e: e.name.startswith("target"))]
        if use_agent_lidar:
            self.lidars.append(LidarSpec(B, n_lidar_rays_agents, lidar_range, lambda e: e.name.startswith("agent"),
                                         angle_start=0.05, angle_end=2 * torch.pi + 0.05))
        self.all_time_covered_targets = None

    def reset(self, snap) -> None:
        self.all_time_covered_targets = torch.full((self.B, self.n_targets), False)  # discovery.py:127-132

    def step(self, pre_snap, snap) -> Dict:
        """``pre_snap``: the state before the step (the targets are static, so their positions
        there are what the reward reads before its respawn); ``snap``: after the step (agents moved,
        covered targets respawned).  Returns the programs' outputs plus ``covered`` for the
        respawn check."""
        B = self.B
        # the reward's view: agents after physics, targets before the respawn
        rsnap = dict(snap)
        for t in self.targets:
            rsnap[self.idx(t)] = pre_snap[self.idx(t)]
        ow = self.ow(rsnap)
        agents = [ow.ents[self.idx(n)] for n in self.agent_names]
        time_rew = torch.full((B,), self.time_penalty)  # discovery.py:151-155
        agents_pos = torch.stack([a.state.pos for a in agents], dim=1)
        targets_pos = torch.stack([ow.ents[self.idx(t)].state.pos for t in self.targets], dim=1)
        dists = torch.cdist(agents_pos, targets_pos)  # 160
        agents_per_target = torch.sum((dists < self.covering_range).type(torch.int), dim=1)
        covered_targets = agents_per_target >= self.agents_per_target  # 165
        margin = (dists - self.covering_range).abs().flatten(1).amin(-1)
        covering = []
        shared = torch.zeros(B)
        for i in range(len(agents)):  # agent_reward (229-242), summed into the shared reward
            targets_covered_by_agent = dists[:, i] < self.covering_range
            num = (targets_covered_by_agent * covered_targets).sum(dim=-1)
            cr = torch.zeros(B)
            cr += num * self.coeff
            covering.append(cr)
            shared += cr
        shared[shared != 0] /= 2  # 170
        rews, collision = [], []
        for i, agent in enumerate(agents):  # 173-178, 211-217
            col = torch.zeros(B)
            for j, a in enumerate(agents):
                if j != i:
                    d = ow.get_distance(a, agent)
                    col[d < self.min_collision_distance] += self.penalty
                    if self.penalty != 0:
                        margin = torch.minimum(margin, (d - self.min_collision_distance).abs())
            collision.append(col)
            cov = covering[i] if not self.shared_reward else shared
            rews.append(col + cov + time_rew)
        # observations (244-250) on the state after the respawn
        ow2 = self.ow(snap)
        obs, lidar = [], []
        for name in self.policy_names:
            ai = self.idx(name)
            agent = ow2.ents[ai]
            parts = [agent.state.pos, agent.state.vel]
            col0 = 4
            for spec in self.lidars:
                m, rays = spec.measure(ow2, ai)
                parts.append(m)
                lidar.append((len(obs), col0, col0 + m.shape[1], ai, rays, spec))
                col0 += m.shape[1]
            obs.append(torch.cat(parts, dim=-1))
        infos = []
        for i, name in enumerate(self.policy_names):  # 252-262
            k = self.agent_names.index(name)
            infos.append({"covering_reward": covering[k] if not self.shared_reward else shared,
                          "collision_rew": collision[k], "targets_covered": covered_targets.sum(-1)})
        if not self.targets_respawn:
            self.all_time_covered_targets += covered_targets  # 206
        done = self.all_time_covered_targets.all(dim=-1)  # 264-265
        rews = [rews[self.agent_names.index(n)] for n in self.policy_names]
        return {"obs": obs, "rew": rews, "done": done, "info": infos, "margin": margin, "lidar": lidar,
                "covered": covered_targets, "agents_pos": agents_pos}

    def check_respawn(self, pre_snap, snap, covered: Tensor, agents_pos: Tensor, skip: Optional[Tensor] = None,
                      tol: float = 1e-6) -> Dict:
        """The respawn of discovery.py:181-204 (targets_respawn=True), checked instead of redrawn
        (its sampler is pinned bit for bit by tests/test_spawn.py): a target keeps its position
        where it is not covered; where it is, its new position lies inside the bounds and at least
        ``min_dist`` (cdist, ``not (d < min_dist)``, utils.py:305-310) from every agent and from
        every other target as it stood when this target was drawn (the targets before it already
        respawned).  A distance within ``tol`` of the threshold counts as certified, not bad;
        ``skip``: envs not checked (certified flag crossings, where coverage itself may differ)."""
        if not self.targets_respawn:
            return {"bad_envs": 0, "respawned": 0, "threshold_envs": 0}
        bad = torch.zeros(self.B, dtype=torch.bool)
        near = torch.zeros(self.B, dtype=torch.bool)
        cur = [pre_snap[self.idx(t)]["pos"] for t in self.targets]
        for i, t in enumerate(self.targets):
            new = snap[self.idx(t)]["pos"]
            cov = covered[:, i]
            same = (new == cur[i]).all(-1)
            bad |= ~cov & ~same
            occ = torch.cat([agents_pos] + [cur[j].unsqueeze(1) for j in range(len(self.targets)) if j != i], dim=1)
            d = torch.cdist(occ, new.unsqueeze(1)).squeeze(-1)
            viol = (d < self.min_dist) & cov.unsqueeze(-1)
            close = (d - self.min_dist).abs() <= tol
            near |= (viol & close).any(-1)
            inside = ((new[:, 0].abs() <= self.x_semidim) & (new[:, 1].abs() <= self.y_semidim))
            bad |= (viol & ~close).any(-1) | (cov & ~inside)
            cur[i] = new
        if skip is not None:
            bad &= ~skip
            near &= ~skip
        return {"bad_envs": int(bad.sum()), "respawned": int(covered.sum()), "threshold_envs": int(near.sum())}


# ------------------------------------------------------------------------------------------------
class Flocking(_Program):
    """vmas/scenarios/flocking.py (make_world kwargs 19-27, reference defaults).  The scripted
    ``target`` agent moves on ``u = (cos t/30, sin t/30)`` with ``t`` the steps since reset."""

    desired_distance = 0.1  # flocking.py:30
    min_collision_distance = 0.005  # flocking.py:31

    def __init__(self, world, n_obstacles: int = 5, min_dist_between_entities: float = 0.15, n_lidar_rays: int = 12,
                 collision_reward: float = -0.1, dist_shaping_factor: float = 1, **kw):
        super().__init__(world)
        self.collision_reward = collision_reward
        self.dist_shaping_factor = dist_shaping_factor
        agents = self.agent_set
        # flocking.py:46-60: 12 rays at range 0.2 against every entity that is not an Agent
        self.lidar = LidarSpec(world.batch_dim, n_lidar_rays, 0.2, lambda e: id(e) not in agents)
        self.t = None
        self.distance_shaping = {}

    def _shaping(self, ow, name) -> Tensor:
        """(stack of |p - p_other| over the other agents - desired).pow(2).mean(-1) * factor
        (flocking.py:115-127, 173-183)."""
        agent = ow.ents[self.idx(name)]
        return (torch.stack([_norm(agent.state.pos - ow.ents[self.idx(a)].state.pos) for a in self.agent_names
                             if a != name], dim=1) - self.desired_distance).pow(2).mean(-1) * self.dist_shaping_factor

    def reset(self, snap) -> None:
        ow = self.ow(snap)
        for n in self.policy_names:  # flocking.py:113-127
            self.distance_shaping[n] = self._shaping(ow, n)
        self.t = torch.zeros(self.B)  # 144-145

    def scripted_u(self) -> Tensor:
        """action_script (flocking.py:84-86) at the step's t (before the reward advances it)."""
        t = self.t / 30
        return torch.stack([torch.cos(t), torch.sin(t)], dim=1)

    def step(self, pre_snap, snap) -> Dict:
        ow = self.ow(snap)
        B = self.B
        self.t += 1  # flocking.py:153
        collision_rew = {n: torch.zeros(B) for n in self.policy_names}
        margin = torch.full((B,), INF)
        if self.collision_reward != 0:  # 156-170
            names = self.agent_names
            for i, a in enumerate(names):
                for j, b in enumerate(names):
                    if j <= i:
                        continue
                    d = ow.get_distance(ow.ents[self.idx(a)], ow.ents[self.idx(b)])
                    collision = d <= self.min_collision_distance
                    margin = torch.minimum(margin, (d - self.min_collision_distance).abs())
                    if a in collision_rew:
                        collision_rew[a][collision] += self.collision_reward
                    if b in collision_rew:
                        collision_rew[b][collision] += self.collision_reward
        rews, dist_rews = [], {}
        for n in self.policy_names:  # 172-187
            s = self._shaping(ow, n)
            dist_rews[n] = self.distance_shaping[n] - s
            self.distance_shaping[n] = s
            rews.append(collision_rew[n] + dist_rews[n])
        obs, lidar, infos = [], [], []
        target = ow.ents[self.idx("target")]
        for n in self.policy_names:  # 189-198
            ai = self.idx(n)
            agent = ow.ents[ai]
            m, rays = self.lidar.measure(ow, ai)
            lidar.append((len(obs), 6, 6 + m.shape[1], ai, rays, self.lidar))
            obs.append(torch.cat([agent.state.pos, agent.state.vel, agent.state.pos - target.state.pos, m], dim=-1))
            infos.append({"agent_collision_rew": collision_rew[n], "agent_distance_rew": dist_rews[n]})  # 200-206
        done = torch.tensor([False]).expand(B)  # BaseScenario.done (scenario.py:326-328)
        return {"obs": obs, "rew": rews, "done": done, "info": infos, "margin": margin, "lidar": lidar}


# ------------------------------------------------------------------------------------------------
# What each benchmark scenario's make_world builds, restated from the reference's files (VERDICT r5
# "Next" #4): the teacher-forced checks above read mass, shapes, collision_force, substeps and the
# agents' u_range / u_multiplier from the product's world, so a constant misread by a product
# make_world would pass them; this table holds those constants independently.
#
# Defaults: World (core.py:1090-1106; DRAG / COLLISION_FORCE / JOINT_FORCE / TORQUE_CONSTRAINT_FORCE,
# utils.py:28-34), Entity / Landmark / Agent (core.py:538-556, 789-806, 830-868), the shapes
# (core.py:103, 141, 172), Lidar (sensors.py:47-56).
_WORLD_DEFAULTS = dict(dt=0.1, substeps=1, drag=0.25, linear_friction=0.0, angular_friction=0.0, x_semidim=None,
                       y_semidim=None, collision_force=100.0, joint_force=130.0, torque_constraint_force=1.0,
                       contact_margin=1e-3, gravity=(0.0, 0.0))


def _sphere(r=0.05):
    return ("sphere", r)


def _box(length=0.3, width=0.1, hollow=False):
    return ("box", length, width, hollow)


def _line(length=0.5):
    return ("line", length)


def _entity(shape, movable=False, rotatable=False, collide=True, mass=1.0, **extra):
    return dict(shape=shape, movable=movable, rotatable=rotatable, collide=collide, mass=mass, **extra)


def _agent(shape=None, u_multiplier=1.0, u_range=1.0, collide=True, mass=1.0, lidars=(), scripted=False):
    # an Agent is movable and rotatable by default (core.py:833-834); holonomic dynamics (action
    # size 2); sensors as (n_rays, max_range, angle_start, angle_end)
    return _entity(shape or _sphere(), movable=True, rotatable=True, collide=collide, mass=mass,
                   u_multiplier=u_multiplier, u_range=u_range, lidars=list(lidars), scripted=scripted)


def scenario_construction(name: str, **kw) -> Dict:
    """{"world": {...}, "entities": {entity name: {...}}} as the reference's make_world builds it
    for the given kwargs (their defaults restated from the reference's ``kwargs.pop`` lines)."""
    world = dict(_WORLD_DEFAULTS)
    ents: Dict[str, Dict] = {}
    if name == "balance":  # balance.py:15-78
        n_agents = kw.get("n_agents", 3)
        world.update(gravity=(0.0, -0.05), y_semidim=1.0)
        for i in range(n_agents):
            ents[f"agent_{i}"] = _agent(_sphere(0.03), u_multiplier=0.7)
        ents["goal"] = _entity(_sphere(), collide=False)
        ents["package"] = _entity(_sphere(), movable=True, mass=kw.get("package_mass", 5))
        ents["line"] = _entity(_line(0.8), movable=True, rotatable=True, mass=5)
        ents["floor"] = _entity(_box(10, 1))
    elif name == "transport":  # transport.py:15-66
        n_agents, n_packages = kw.get("n_agents", 4), kw.get("n_packages", 1)
        pl, pw = kw.get("package_length", 0.15), kw.get("package_width", 0.15)
        semi = 1 + 2 * 0.03 + max(pl, pw)
        world.update(x_semidim=semi, y_semidim=semi)
        for i in range(n_agents):
            ents[f"agent_{i}"] = _agent(_sphere(0.03), u_multiplier=0.6)
        ents["goal"] = _entity(_sphere(0.15), collide=False)
        for i in range(n_packages):
            ents[f"package {i}"] = _entity(_box(pl, pw), movable=True, mass=kw.get("package_mass", 50))
    elif name == "discovery":  # discovery.py:20-118
        n_agents, n_targets = kw.get("n_agents", 5), kw.get("n_targets", 7)
        lidar_range = kw.get("lidar_range", 0.35)
        world.update(x_semidim=kw.get("x_semidim", 1), y_semidim=kw.get("y_semidim", 1), collision_force=500,
                     substeps=2, drag=0.25)
        lidars = [(kw.get("n_lidar_rays_entities", 15), lidar_range, 0.0, 2 * math.pi)]
        if kw.get("use_agent_lidar", False):
            lidars.append((kw.get("n_lidar_rays_agents", 12), lidar_range, 0.05, 2 * math.pi + 0.05))
        for i in range(n_agents):
            ents[f"agent_{i}"] = _agent(_sphere(0.05), lidars=lidars)
        for i in range(n_targets):
            ents[f"target_{i}"] = _entity(_sphere(0.05))
    elif name == "flocking":  # flocking.py:18-75
        n_agents, n_obstacles = kw.get("n_agents", 4), kw.get("n_obstacles", 5)
        world.update(collision_force=400, substeps=5)
        ents["target"] = _agent(scripted=True)
        for i in range(n_agents):
            ents[f"agent_{i}"] = _agent(lidars=[(kw.get("n_lidar_rays", 12), 0.2, 0.0, 2 * math.pi)])
        for i in range(n_obstacles):
            ents[f"obstacle_{i}"] = _entity(_sphere(0.1))
    else:
        raise KeyError(name)
    return {"world": world, "entities": ents}


def _shape_of(shape) -> tuple:
    kind = type(shape).__name__.lower()
    if kind == "sphere":
        return ("sphere", shape.radius)
    if kind == "box":
        return ("box", shape.length, shape.width, shape.hollow)
    return ("line", shape.length)


def world_construction(world) -> Dict:
    """The same record read from a built world (the checked side: any World with the reference's
    attribute names).  A Lidar's angle span is recovered from its angle row."""
    gx, gy = (float(v) for v in world._gravity.reshape(-1)[:2].tolist())
    rec = {"world": dict(dt=world._dt, substeps=world._substeps, drag=world._drag,
                         linear_friction=world._linear_friction, angular_friction=world._angular_friction,
                         x_semidim=world._x_semidim, y_semidim=world._y_semidim,
                         collision_force=world._collision_force, joint_force=world._joint_force,
                         torque_constraint_force=world._torque_constraint_force,
                         contact_margin=world._contact_margin, gravity=(gx, gy)),
           "entities": {}}
    agents = {id(a) for a in world.agents}
    for e in world.entities:
        d = dict(shape=_shape_of(e.shape), movable=e.movable, rotatable=e.rotatable, collide=e.collide, mass=e.mass)
        if id(e) in agents:
            lidars = []
            for s in e.sensors or []:
                row = s._angles[0].detach().to("cpu", torch.float64)
                lidars.append((int(row.numel()), s._max_range, row))
            d.update(u_multiplier=e.u_multiplier, u_range=e.u_range, lidars=lidars,
                     scripted=e.action_script is not None)
        rec["entities"][e.name] = d
    return rec


def construction_mismatches(expected: Dict, got: Dict) -> List[str]:
    """Every field where a built world differs from the restated construction (empty: equal).
    Floats compare at fp32 (the product may hold a value as a float32 tensor)."""
    def feq(a, b):
        if a is None or b is None:
            return a is None and b is None
        return float(torch.tensor(float(a), dtype=torch.float32)) == float(torch.tensor(float(b), dtype=torch.float32))

    bad = []
    for k, v in expected["world"].items():
        g = got["world"][k]
        ok = all(feq(x, y) for x, y in zip(v, g)) if isinstance(v, tuple) else feq(v, g)
        if not ok:
            bad.append(f"world.{k}: expected {v}, got {g}")
    if sorted(expected["entities"]) != sorted(got["entities"]):
        bad.append(f"entities: expected {sorted(expected['entities'])}, got {sorted(got['entities'])}")
    for name, v in expected["entities"].items():
        g = got["entities"].get(name)
        if g is None:
            continue
        for k, x in v.items():
            if k == "lidars":
                if len(x) != len(g[k]):
                    bad.append(f"{name}.lidars: expected {len(x)}, got {len(g[k])}")
                    continue
                for j, ((n, rng, a0, a1), (gn, grng, grow)) in enumerate(zip(x, g[k])):
                    want = lidar_angles(1, n, a0, a1)[0].to(torch.float64)
                    if n != gn or not feq(rng, grng) or want.shape != grow.shape or not torch.allclose(
                            want, grow, rtol=0, atol=1e-6):
                        bad.append(f"{name}.lidar[{j}]: expected ({n} rays, range {rng}, angles {a0}..{a1}), "
                                   f"got ({gn} rays, range {grng})")
            elif k == "shape":
                gs = g[k]
                if x[0] != gs[0] or len(x) != len(gs) or not all(
                        (xa == ga) if isinstance(xa, bool) else feq(xa, ga) for xa, ga in zip(x[1:], gs[1:])):
                    bad.append(f"{name}.shape: expected {x}, got {gs}")
            elif isinstance(x, bool):
                if bool(g[k]) != x:
                    bad.append(f"{name}.{k}: expected {x}, got {g[k]}")
            elif not feq(x, g[k]):
                bad.append(f"{name}.{k}: expected {x}, got {g[k]}")
    return bad


PROGRAMS = {"balance": Balance, "transport": Transport, "discovery": Discovery, "flocking": Flocking}


def program(name: str, world, **kw) -> _Program:
    return PROGRAMS[name](world, **kw)
