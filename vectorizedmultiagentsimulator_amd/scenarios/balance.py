# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Balance: agents carry a line with a package on it towards a goal, under gravity.

Workload of BASELINE configs C1/C2.  Restates vmas/scenarios/balance.py:15-262 (world layout,
reset distribution and RNG call order, reward, observation, done, heuristic policy).
Entities (in World.entities order): goal (sphere, no collide), package (sphere, movable),
line (movable + rotatable), floor (static box), agents (spheres).
"""
import ctypes
import math

import torch

from vectorizedmultiagentsimulator_amd import _native as N
from vectorizedmultiagentsimulator_amd.simulator import _fused
from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Box, Landmark, Line, Sphere, World
from vectorizedmultiagentsimulator_amd.simulator.heuristic_policy import BaseHeuristicPolicy
from vectorizedmultiagentsimulator_amd.simulator.scenario import BaseScenario
from vectorizedmultiagentsimulator_amd.simulator.utils import Color, ScenarioUtils, Y


class Scenario(BaseScenario):
    # re-bound by the first agent's reward before anything in the step reads them (global_shaping
    # is read: carried): graph replays need not carry them (environment/_graph.py)
    _vmas_graph_write_only = frozenset({"on_the_ground", "package_dist", "pos_rew"})

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
        # the fused program below is also compiled into the world's specialised module: the eager
        # step launches it from there, and a replayed step runs it as k_world's epilogue
        # (csrc/vmas_programs.hpp; simulator/environment/_graph.py _KernelChain)
        world._jit_epilogue = N.EPILOGUE_BALANCE
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
        if _fused.enabled(self.world):
            return self._fused_reward(agent)
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
        if _fused.enabled(self.world):
            return self._fused_observation(agent)
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
        if _fused.enabled(self.world):
            return self._fused_done()
        return self.on_the_ground + self.world.is_overlapping(self.package, self.package.goal)

    # ---- fused program (GPU worlds; csrc/vmas_scenarios.hip k_balance) -------------------------
    # The first agent's reward call runs ONE launch for the whole step's program: the reward block
    # above (with every attribute it leaves: on_the_ground, package_dist, ground_rew in place, the
    # old pos_rew zeroed in place, pos_rew / global_shaping re-bound to fresh tensors), every
    # agent's reward, every agent's observation and done().  The other calls hand out the
    # precomputed tensors (popped, so the caller owns them) while their inputs are unchanged --
    # the same tensor objects at the same version counters (_fused.state_key); otherwise they
    # recompute, as the reference does on every call.

    def _obs_inputs(self):
        w, pk, ln = self.world, self.package, self.line
        ts = [pk.state.pos, pk.state.vel, pk.goal.state.pos, ln.state.pos, ln.state.vel, ln.state.ang_vel,
              ln.state.rot]
        for a in w.agents:
            ts += [a.state.pos, a.state.vel]
        return ts

    def _done_inputs(self):
        return [self.on_the_ground, self.package.state.pos, self.package.goal.state.pos]

    def _run_fused(self, what: int):
        w = self.world
        dev = torch.device(w.device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        B, A = w.batch_dim, len(w.agents)
        keep = []
        io = N.VmasBalanceIO()
        io.batch, io.n_agents, io.what = B, A, what
        io.shaping_factor = float(self.shaping_factor)
        io.fall_reward = float(self.fall_reward)
        io.pi = math.pi
        io.package = _fused.ref(w, self.package, keep, 0)
        io.goal = _fused.ref(w, self.package.goal, keep, 0)
        io.line = _fused.ref(w, self.line, keep, 0)
        io.floor = _fused.ref(w, self.floor, keep, 0)
        out = {}
        # (graph-mode capture: obs / rewards / done written straight into each replay's fresh tensors)
        io.out_delta, direct = _fused.direct_outputs(w, (
            (torch.float32, (B, 16), A) if what & N.VMAS_SCN_OBS else None,
            (torch.float32, (B,), A) if what & N.VMAS_SCN_REWARD else None,
            (torch.bool, (B,), 1) if what & N.VMAS_SCN_DONE else None))
        if what & N.VMAS_SCN_REWARD:
            gs = _fused.f32(self.global_shaping, dev)
            keep.append(gs)
            io.global_shaping, io.gs_s0 = gs.data_ptr(), gs.stride(0)
            for name in ("global_shaping", "package_dist", "pos_rew"):
                out[name] = torch.empty(B, device=dev, dtype=torch.float32)
            out["on_the_ground"] = torch.empty(B, device=dev, dtype=torch.bool)
            io.global_shaping_out = out["global_shaping"].data_ptr()
            io.package_dist = out["package_dist"].data_ptr()
            io.pos_rew = out["pos_rew"].data_ptr()
            io.on_the_ground = out["on_the_ground"].data_ptr()
            io.ground_rew = self.ground_rew.data_ptr()
            prev = self.pos_rew
            io.pos_rew_prev = prev.data_ptr() if prev.numel() else None
            out["rewards"] = direct[1] or [torch.empty(B, device=dev, dtype=torch.float32) for _ in range(A)]
            for i, r in enumerate(out["rewards"]):
                io.rewards[i] = r.data_ptr()
        if what & N.VMAS_SCN_OBS:
            io.package_vel = _fused.vec(_fused.f32(self.package.state.vel, dev), keep)
            io.line_vel = _fused.vec(_fused.f32(self.line.state.vel, dev), keep)
            io.line_ang_vel = _fused.vec(_fused.f32(self.line.state.ang_vel, dev), keep)
            for i, a in enumerate(w.agents):
                io.agent_pos[i] = _fused.vec(_fused.f32(a.state.pos, dev), keep)
                io.agent_vel[i] = _fused.vec(_fused.f32(a.state.vel, dev), keep)
            out["obs"] = direct[0] or [torch.empty(B, 16, device=dev, dtype=torch.float32) for _ in range(A)]
            for i, o in enumerate(out["obs"]):
                io.obs[i] = o.data_ptr()
        if what & N.VMAS_SCN_DONE:
            og = out.get("on_the_ground", self.on_the_ground)
            if og.device != dev or og.dtype is not torch.bool or not og.is_contiguous():
                og = og.to(device=dev, dtype=torch.bool).contiguous()
            keep.append(og)
            io.on_the_ground = og.data_ptr()
            out["done"] = direct[2][0] if direct[2] else torch.empty(B, device=dev, dtype=torch.bool)
            io.done = out["done"].data_ptr()
        jit = w.engine.jit_program(N.EPILOGUE_BALANCE)
        if jit is not None:  # (the world module's k_program_jit: the code a replay runs as k_world's epilogue)
            N.check_jit(_fused.lib().vmas_jit_program_outputs(jit, N.EPILOGUE_BALANCE, ctypes.byref(io), _fused.stream(w)),
                        "vmas_jit_program_outputs")
        else:
            _fused.check(_fused.lib().vmas_balance_outputs(dev.index, ctypes.byref(io), _fused.stream(w)),
                         "vmas_balance_outputs")
        if what & N.VMAS_SCN_REWARD:
            _fused.bump_version(self.ground_rew)
            if io.pos_rew_prev:
                _fused.bump_version(prev)
            self.on_the_ground = out["on_the_ground"]
            self.package_dist = out["package_dist"]
            self.pos_rew = out["pos_rew"]
            self.global_shaping = out["global_shaping"]
        return out

    def _fused_ok(self) -> bool:
        """The in-place / strided operands the kernel assumes (else the torch program runs)."""
        w = self.world
        B = w.batch_dim
        gr, pr = self.ground_rew, self.pos_rew
        return (len(w.agents) <= N.VMAS_SCN_MAX_AGENTS and gr.dtype is torch.float32 and gr.is_contiguous()
                and gr.shape == (B,) and gr.device == torch.device(w.device) and pr.dtype is torch.float32
                and pr.shape == (B,) and pr.is_contiguous() and pr.device == gr.device
                and pr.data_ptr() != gr.data_ptr() and self.global_shaping.shape == (B,))

    def _fused_reward(self, agent: Agent):
        w = self.world
        i = w.agents.index(agent)
        if i == 0:
            if not self._fused_ok():
                self._fused = None
                return self._torch_reward(agent)
            out = self._run_fused(N.VMAS_SCN_REWARD | N.VMAS_SCN_OBS | N.VMAS_SCN_DONE)
            self._fused = {
                "rew_key": _fused.state_key([self.ground_rew, self.pos_rew]),
                "rewards": dict(enumerate(out["rewards"])),
                "obs_key": _fused.state_key(self._obs_inputs()),
                "obs": dict(enumerate(out["obs"])),
                "done_key": _fused.state_key(self._done_inputs()),
                "done": out["done"],
            }
        c = getattr(self, "_fused", None)
        if c is not None and i in c["rewards"] and c["rew_key"] == _fused.state_key([self.ground_rew, self.pos_rew]):
            return c["rewards"].pop(i)
        return self.ground_rew + self.pos_rew

    def _torch_reward(self, agent: Agent):
        if agent == self.world.agents[0]:
            self.pos_rew[:] = 0
            self.ground_rew[:] = 0
            self.compute_on_the_ground()
            self.package_dist = torch.linalg.vector_norm(self.package.state.pos - self.package.goal.state.pos, dim=1)
            self.ground_rew.masked_fill_(self.on_the_ground, self.fall_reward)
            global_shaping = self.package_dist * self.shaping_factor
            self.pos_rew = self.global_shaping - global_shaping
            self.global_shaping = global_shaping
        return self.ground_rew + self.pos_rew

    def _fused_observation(self, agent: Agent):
        w = self.world
        i = w.agents.index(agent)
        c = getattr(self, "_fused", None)
        if c is None or i not in c["obs"] or c["obs_key"] != _fused.state_key(self._obs_inputs()):
            if len(w.agents) > N.VMAS_SCN_MAX_AGENTS:
                return self._torch_observation(agent)
            out = self._run_fused(N.VMAS_SCN_OBS)
            c = self._fused = {"rew_key": None, "rewards": {}, "obs_key": _fused.state_key(self._obs_inputs()),
                               "obs": dict(enumerate(out["obs"])), "done_key": None, "done": None}
        return c["obs"].pop(i)

    def _torch_observation(self, agent: Agent):
        package, line = self.package, self.line
        return torch.cat([agent.state.pos, agent.state.vel, agent.state.pos - package.state.pos,
                          agent.state.pos - line.state.pos, package.state.pos - package.goal.state.pos,
                          package.state.vel, line.state.vel, line.state.ang_vel, line.state.rot % torch.pi], dim=-1)

    def _fused_done(self):
        c = getattr(self, "_fused", None)
        if c is not None and c["done"] is not None and c["done_key"] == _fused.state_key(self._done_inputs()):
            d, c["done"] = c["done"], None
            return d
        return self._run_fused(N.VMAS_SCN_DONE)["done"]

    def info(self, agent: Agent):
        return {"pos_rew": self.pos_rew, "ground_rew": self.ground_rew}

    def _vmas_tail_sources(self):
        """The tensors the fused program writes through (sc1, csrc/vmas_programs.hpp bal_reward): a
        graph replay may copy them inside the same launch (environment/_graph.py _tail_ok)."""
        return [self.global_shaping, self.pos_rew, self.ground_rew]


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
