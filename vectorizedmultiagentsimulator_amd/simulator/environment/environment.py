# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""The vectorized Environment (restates vmas/simulator/environment/environment.py:49-1070).

Differences from the reference are limited to host-synchronisation placement (§8f row 1 of
SURVEY.md); results and exceptions are the same:
  * all agents' continuous actions are validated (NaN / range) with ONE device->host sync per
    step instead of two per agent (environment.py:621-623, 653-655);
  * random actions take their bounds from the python ``u_range`` values (the same fp32 numbers
    the reference reads back from ``u_range_tensor`` with a sync per call).
Rendering is outside the scope of the MI355X engine.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import os
import random
import sys
from typing import Dict, List, Optional, Sequence, Union, Any

import numpy as np
import torch
from torch import Tensor

from .. import core as _core
from ..core import Agent, TorchVectorizedObject
from ..scenario import BaseScenario
from ..utils import AGENT_OBS_TYPE, DEVICE_TYPING, TorchUtils, override
from . import spaces
from . import _uniform
from ._rng import numpy_global_rng, python_global_rng


@contextlib.contextmanager
def local_seed(vmas_random_state):
    """Swap in the simulator's RNG states for torch(CPU)/numpy/python (environment.py:30-46).

    The numpy and Python states are saved/restored by ``_rng.NumpyGlobalRng`` /
    ``PythonGlobalRng`` (the same states as get_state/set_state and getstate/setstate, without
    their element-wise key copies)."""
    npr, pyr = numpy_global_rng(), python_global_rng()
    torch_state = torch.random.get_rng_state()
    np_state = npr.snapshot()
    py_state = pyr.snapshot()
    torch.random.set_rng_state(vmas_random_state[0])
    npr.restore(vmas_random_state[1])
    pyr.restore(vmas_random_state[2])
    yield
    vmas_random_state[0] = torch.random.get_rng_state()
    vmas_random_state[1] = npr.snapshot()
    vmas_random_state[2] = pyr.snapshot()
    torch.random.set_rng_state(torch_state)
    npr.restore(np_state)
    pyr.restore(py_state)


def _f32(x) -> float:
    return float(np.float32(x))


_storage_use_count = getattr(torch._C, "_storage_Use_Count", None)


def _refs_of_fresh_argument(value) -> int:
    return sys.getrefcount(value)


# sys.getrefcount of a temporary passed straight into a function, measured on THIS interpreter
# (3.10 counts the caller's stack slot and the parameter; 3.11+ moves arguments into the callee
# frame, one reference fewer): a tensor that something else also holds counts more than this
_FRESH_REFS = _refs_of_fresh_argument(object())


def _owned_or_clone(value):
    """The reference clones every reward / observation / info it returns (environment.py:
    149-196) so that callers never alias tensors the scenario keeps.  A tensor that nothing else
    can reach -- the fresh result of torch.cat / an arithmetic op, referenced only by this call
    (Python refcount) and sharing its storage with no other tensor (storage use count: the tensor
    plus the temporary storage wrapper) -- is returned as is: identical values, no alias, one
    kernel less.  Anything else (scenario attributes, views, dicts) is cloned as the reference
    does."""
    if (isinstance(value, Tensor) and _storage_use_count is not None
            and sys.getrefcount(value) <= _FRESH_REFS  # no reference but the call's own
            and _storage_use_count(value.untyped_storage()._cdata) <= 2):
        return value
    return TorchUtils.recursive_clone(value)


class _ActionShadow:
    """Graph mode's random-action draw pre-applies the drawn actions into the persistent action
    buffer P that the captured step reads (_preapply_columns) -- the buffer agents' action.u, and a
    holonomic agent's state.force, view after a graph step.  The draw first copies P's current
    values into a fresh snapshot (vmas_uniform_columns_snap); while armed (from that draw to the
    step that consumes it) Action.u / AgentState.force return the matching view of the snapshot,
    so reading them between get_random_actions() and step() gives the last step's values, as in
    the reference."""

    __slots__ = ("active", "base", "end", "snap", "views")

    def __init__(self):
        self.active = False
        self.base = self.end = 0
        self.snap = None
        self.views = None

    def arm(self, P: Tensor, snap: Tensor) -> None:
        self.base, self.end = P.data_ptr(), P.data_ptr() + 4 * P.numel()
        self.snap = snap
        self.views = {}
        self.active = True

    def disarm(self) -> None:
        self.active = False
        self.snap = self.views = None

    def view(self, t):
        """The snapshot's view matching ``t`` (a view of P); ``t`` itself when it is elsewhere."""
        if t is None or t.dtype is not torch.float32 or not (self.base <= t.data_ptr() < self.end):
            return t
        v = self.views.get(id(t))
        if v is None or v[0] is not t:
            off = (t.data_ptr() - self.base) // 4
            v = self.views[id(t)] = (t, self.snap.as_strided(t.shape, t.stride(), off))
        return v[1]


def _plain_accessors(agent_cls, action_cls) -> bool:
    """The agent / action classes read `action`, `silent`, `batch_dim` and `u_range` through the
    core classes' own properties (which return `_action`, `_silent`, `_batch_dim`, `_u_range`) and
    keep `action_size` a plain attribute."""
    from ..core import Action

    bd = getattr(agent_cls, "batch_dim", None)
    return (getattr(agent_cls, "action", None) is Agent.action and getattr(agent_cls, "silent", None) is Agent.silent
            and isinstance(bd, property) and bd.fget is TorchVectorizedObject.batch_dim.fget
            and not hasattr(agent_cls, "action_size")
            and getattr(action_cls, "u_range", None) is Action.u_range)


class Environment(TorchVectorizedObject):
    metadata = {"render.modes": ["human", "rgb_array"], "runtime.vectorized": True}
    vmas_random_state = [torch.random.get_rng_state(), np.random.get_state(), random.getstate()]

    @local_seed(vmas_random_state)
    def __init__(
        self,
        scenario: BaseScenario,
        num_envs: int = 32,
        device: DEVICE_TYPING = "cpu",
        max_steps: Optional[int] = None,
        continuous_actions: bool = True,
        seed: Optional[int] = None,
        dict_spaces: bool = False,
        multidiscrete_actions: bool = False,
        clamp_actions: bool = False,
        grad_enabled: bool = False,
        terminated_truncated: bool = False,
        graph_step: Optional[bool] = None,
        **kwargs,
    ):
        if multidiscrete_actions:
            assert not continuous_actions, (
                "When asking for multidiscrete_actions, make sure continuous_actions=False"
            )
        self.scenario = scenario
        self.num_envs = num_envs
        TorchVectorizedObject.__init__(self, num_envs, torch.device(device))
        self.world = self.scenario.env_make_world(self.num_envs, self.device, **kwargs)
        self.agents = self.world.policy_agents
        self.n_agents = len(self.agents)
        self.max_steps = max_steps
        self.continuous_actions = continuous_actions
        self.dict_spaces = dict_spaces
        self.clamp_action = clamp_actions
        self.grad_enabled = grad_enabled
        # grad_enabled: the world step, ray casts and distance queries run through their native
        # backward (simulator/_engine.py _StepFn / _RaysFn / _DistFn); the fused scenario programs
        # (no backward) give way to the scenarios' torch programs
        self.world._grad_enabled = bool(grad_enabled)
        self._apply_cache = None  # see _apply_continuous_actions
        self._u_persist = None  # persistent action buffer of graph mode (see _apply_continuous_actions)
        self._spec_keep = None  # action tensors a speculative action launch reads
        self._draw_plans = {}  # agent -> cached column plan of its random actions
        self._uniform_cache = None  # see _fused_random_actions
        self._uniform_host = None  # (column plan, its csrc/vmas_host.cpp UniformDraw)
        self._ushadow = _ActionShadow()
        self._spec = None  # a draw made ahead by the post-replay launch (_draw_ahead_plan)
        self._spec_ok = False  # the last step consumed a draw applied by its own launch
        for ag in self.world.agents:
            ag._action._shadow = self._ushadow
            ag._state._shadow = self._ushadow
        self._preapply = None  # see _preapply_columns
        self._drawn = None  # the last draw whose applied values are in the persistent buffer
        self.preapplied_steps = 0  # graph steps whose actions were applied by their draw
        self._raw_outputs = False  # set while a step is captured (outputs are cloned after replay)
        self.terminated_truncated = terminated_truncated
        observations = self._reset(seed=seed)
        self.multidiscrete_actions = multidiscrete_actions
        self.action_space = self.get_action_space()
        self.observation_space = self.get_observation_space(observations)
        self._graph = None
        self.graph_auto = graph_step is None
        if graph_step is None:
            graph_step = self._auto_graph_step()
        if graph_step:
            if self.device.type != "cuda":
                raise ValueError("graph_step=True needs a ROCm device (HIP graphs)")
            if grad_enabled:
                raise ValueError("graph_step=True replays a captured step: it cannot carry autograd (grad_enabled=True)")
            from ._graph import StepGraph

            self._graph = StepGraph(self)
        self.viewer = None
        self.headless = None
        self.visible_display = None
        self.text_lines = None

    def _auto_graph_step(self) -> bool:
        """graph_step=None (the default; the reference's make_env has no such argument, so an
        unchanged caller -- torchrl's VmasEnv, the Gym wrappers -- lands here): replay the step as
        one HIP graph on a ROCm device with continuous actions and no autograd, for any scenario
        (VERDICT r5 "Next" #7).  The replay is captured only after a watched eager step proves the
        step free of host waits, host RNG draws and Python-side state changes (environment/_graph.py
        StepGraph; for a scenario outside the four benchmark ones also in-place changes of Python
        containers); otherwise, or if the capture fails, the env stays eager (``graph_status`` /
        ``graph_reason``).  Only the benchmark scenarios are trusted with write-only attributes and
        direct outputs.  VMAS_GRAPH_STEP=0 turns the automatic choice off; VMAS_GRAPH_STEP=own keeps
        it to this package's scenarios."""
        mode = os.environ.get("VMAS_GRAPH_STEP", "auto")
        if mode == "0":
            return False
        if self.device.type != "cuda" or self.grad_enabled or not self.continuous_actions:
            return False
        if mode == "own":
            from ._graph import _own_scenario

            return _own_scenario(self.scenario)
        return True

    @local_seed(vmas_random_state)
    def reset(self, seed: Optional[int] = None, return_observations: bool = True,
              return_info: bool = False, return_dones: bool = False):
        """Resets the environment in a vectorized way; returns observations for all envs/agents."""
        return self._reset(seed=seed, return_observations=return_observations,
                           return_info=return_info, return_dones=return_dones)

    @local_seed(vmas_random_state)
    def reset_at(self, index: int, return_observations: bool = True, return_info: bool = False,
                 return_dones: bool = False):
        """Resets the environment at ``index``."""
        return self._reset_at(index=index, return_observations=return_observations,
                              return_info=return_info, return_dones=return_dones)

    @local_seed(vmas_random_state)
    def get_from_scenario(self, get_observations: bool, get_rewards: bool, get_infos: bool,
                          get_dones: bool, dict_agent_names: Optional[bool] = None):
        return self._get_from_scenario(get_observations=get_observations, get_rewards=get_rewards,
                                       get_infos=get_infos, get_dones=get_dones,
                                       dict_agent_names=dict_agent_names)

    @local_seed(vmas_random_state)
    def seed(self, seed=None):
        return self._seed(seed=seed)

    @local_seed(vmas_random_state)
    def done(self):
        return self._done()

    def _reset(self, seed=None, return_observations=True, return_info=False, return_dones=False):
        if seed is not None:
            self._seed(seed)
        self.scenario.env_reset_world_at(env_index=None)
        self.steps = torch.zeros(self.num_envs, device=self.device)
        result = self._get_from_scenario(get_observations=return_observations, get_infos=return_info,
                                         get_rewards=False, get_dones=return_dones)
        return result[0] if result and len(result) == 1 else result

    def _reset_at(self, index, return_observations=True, return_info=False, return_dones=False):
        self._check_batch_index(index)
        self.scenario.env_reset_world_at(index)
        self.steps[index] = 0
        result = self._get_from_scenario(get_observations=return_observations, get_infos=return_info,
                                         get_rewards=False, get_dones=return_dones)
        return result[0] if result and len(result) == 1 else result

    def _get_from_scenario(self, get_observations, get_rewards, get_infos, get_dones,
                           dict_agent_names=None):
        if not get_infos and not get_dones and not get_rewards and not get_observations:
            return
        if dict_agent_names is None:
            dict_agent_names = self.dict_spaces
        obs = rewards = infos = terminated = truncated = dones = None
        if get_observations:
            obs = {} if dict_agent_names else []
        if get_rewards:
            rewards = {} if dict_agent_names else []
        if get_infos:
            infos = {} if dict_agent_names else []
        # order matters: rewards may mutate state that observations read (discovery.py:180-210)
        keep = (lambda v: v) if self._raw_outputs else _owned_or_clone
        if get_rewards:
            for agent in self.agents:
                reward = keep(self.scenario.reward(agent))
                if dict_agent_names:
                    rewards.update({agent.name: reward})
                else:
                    rewards.append(reward)
        if get_observations:
            for agent in self.agents:
                observation = keep(self.scenario.observation(agent))
                if dict_agent_names:
                    obs.update({agent.name: observation})
                else:
                    obs.append(observation)
        if get_infos:
            for agent in self.agents:
                info = self.scenario.info(agent)
                if not self._raw_outputs:
                    info = TorchUtils.recursive_clone(info)
                if dict_agent_names:
                    infos.update({agent.name: info})
                else:
                    infos.append(info)
        if self.terminated_truncated:
            if get_dones:
                terminated, truncated = self._done()
            result = [obs, rewards, terminated, truncated, infos]
        else:
            if get_dones:
                dones = self._done()
            result = [obs, rewards, dones, infos]
        return [data for data in result if data is not None]

    def _seed(self, seed=None):
        if seed is None:
            seed = 0
        torch.manual_seed(seed)
        np.random.seed(seed)
        random.seed(seed)
        return [seed]

    def step(self, actions: Union[List, Dict]):
        """Performs a vectorized step on all sub environments using ``actions``.

        Returns obs, rewards, dones, infos (or obs, rewards, terminated, truncated, infos).

        The reference swaps the simulator's host RNG states (torch CPU / numpy / python) in and
        out around the step (local_seed).  A replayed graph step runs no host RNG code -- its
        random numbers come from the device generator, and per-step host randomness is frozen at
        capture (graph mode's documented requirement) -- so the swap is a no-op there and is
        skipped; an exception raised there leaves the simulator's states swapped in, as the
        reference's swap does (its restore is not in a finally).
        """
        self._ushadow.disarm()  # (the step sets the agents' actions: no snapshot is shown any more)
        self._spec_ok = False
        # a draw made ahead is handed out only by the get_random_actions right after the step that
        # made it: one still pending here was never taken, and this step rewrites the buffer it
        # was applied into
        self._spec = None
        g = self._graph
        if g is not None and g.graph is not None and self.continuous_actions:
            try:
                # the last draw's own tensors, unmodified, pass every check of _check_action_list by
                # construction (a list of [B, action_size] fp32 device tensors, one per agent)
                drawn = self._drawn
                if not (drawn is not None and type(actions) is list and len(actions) == len(drawn[0])
                        and all(a is t and a._version == v for a, t, v in zip(actions, drawn[0], drawn[2]))):
                    actions = self._check_action_list(actions)
                g.before_actions()
                if g.graph is not None:
                    if self._can_speculate() and g.rollback_free() and self._take_preapplied(actions):
                        # drawn + applied by get_random_actions, and nothing in the step can roll it
                        # back: no backup, no generator snapshot
                        return g.replay_preapplied()
                    if self._can_speculate():
                        # the replay is launched before the action flags are known; a failed flag
                        # rolls the step back (StepGraph.replay_speculative) and the eager check
                        # below raises the reference's AssertionError
                        g.backup(self._u_persist[1])
                        if self._take_preapplied(actions):  # drawn + applied by get_random_actions
                            out = g.replay_speculative(lambda: True)
                            if out is not None:
                                return out
                            raise RuntimeError("a step of pre-applied random actions was rolled back")
                        seq = self._apply_continuous_actions(actions, persistent=True, speculative=True)
                        if seq:
                            out = g.replay_speculative(lambda: self._speculative_flags_ok(seq))
                            if out is not None:
                                return out
                            self._apply_continuous_actions(actions)
                            raise RuntimeError("action flags differ between two checks of the same actions")
                    if self._apply_continuous_actions(actions, persistent=True):
                        return g.step()
            except BaseException:
                self._swap_in_simulator_rng()
                raise
            return self._step_seeded(actions, prepared=True)
        return self._step_seeded(actions)

    def _swap_in_simulator_rng(self):
        s = Environment.vmas_random_state
        torch.random.set_rng_state(s[0])
        numpy_global_rng().restore(s[1])
        python_global_rng().restore(s[2])

    @local_seed(vmas_random_state)
    def _step_seeded(self, actions, prepared: bool = False):
        if not prepared:
            actions = self._check_action_list(actions)
            if self._graph is not None and self.continuous_actions:
                self._graph.before_actions()
        if self._graph is not None and self.continuous_actions:
            if self._apply_continuous_actions(actions, persistent=True):
                return self._graph.step()
            g, c = self._graph, self._apply_cache
            if g.graph is None and g.status == "warming" and c is not None and c[1] is None:
                # (the world's own configuration -- communication actions of non-silent agents -- keeps
                # the actions on the per-agent path: every step runs eagerly; report it)
                g.status = "eager"
                g.why = "communication actions (dim_c > 0, non-silent agents) take the per-agent action path"
        return self._step_eager(actions)

    def _check_action_list(self, actions):
        if isinstance(actions, Dict):
            actions_dict = actions
            actions = []
            for agent in self.agents:
                try:
                    actions.append(actions_dict[agent.name])
                except KeyError:
                    raise AssertionError(f"Agent '{agent.name}' not contained in action dict")
            assert len(actions_dict) == self.n_agents, (
                f"Expecting actions for {self.n_agents}, got {len(actions_dict)} actions"
            )
        assert len(actions) == self.n_agents, (
            f"Expecting actions for {self.n_agents}, got {len(actions)} actions"
        )
        for i in range(len(actions)):
            if not isinstance(actions[i], Tensor):
                actions[i] = torch.tensor(actions[i], dtype=torch.float32, device=self.device)
            if len(actions[i].shape) == 1:
                actions[i].unsqueeze_(-1)
            assert actions[i].shape[0] == self.num_envs, (
                f"Actions used in input of env must be of len {self.num_envs}, got {actions[i].shape[0]}"
            )
            assert actions[i].shape[1] == self.get_agent_action_size(self.agents[i]), (
                f"Action for agent {self.agents[i].name} has shape {actions[i].shape[1]},"
                f" but should have shape {self.get_agent_action_size(self.agents[i])}"
            )
        return actions

    def _step_eager(self, actions):
        if not (self.continuous_actions and self._apply_continuous_actions(actions)):
            if self.continuous_actions:
                self._validate_continuous_actions(actions)
            for i, agent in enumerate(self.agents):
                self._set_action(actions[i], agent, validated=self.continuous_actions)
        for agent in self.world.agents:
            self.scenario.env_process_action(agent)
        self.scenario.pre_step()
        self.world.step()
        self.scenario.post_step()
        self.steps += 1
        return self._get_from_scenario(get_observations=True, get_infos=True, get_rewards=True,
                                       get_dones=True)

    def _done(self):
        terminated = self.scenario.done()
        if not self._raw_outputs:  # (a captured step's outputs are cloned after every replay)
            terminated = terminated.clone()
        if self.max_steps is not None:
            truncated = self.steps >= self.max_steps
        else:
            truncated = None
        if self.terminated_truncated:
            if truncated is None:
                truncated = torch.zeros_like(terminated)
            return terminated, truncated
        if truncated is None:
            return terminated
        return terminated + truncated

    # ---- spaces -----------------------------------------------------------------------------------
    def get_action_space(self):
        if not self.dict_spaces:
            return spaces.Tuple([self.get_agent_action_space(agent) for agent in self.agents])
        return spaces.Dict({agent.name: self.get_agent_action_space(agent) for agent in self.agents})

    def get_observation_space(self, observations: Union[List, Dict]):
        if not self.dict_spaces:
            return spaces.Tuple(
                [self.get_agent_observation_space(agent, observations[i]) for i, agent in enumerate(self.agents)]
            )
        return spaces.Dict(
            {agent.name: self.get_agent_observation_space(agent, observations[agent.name]) for agent in self.agents}
        )

    def get_agent_action_size(self, agent: Agent):
        if self.continuous_actions:
            return agent.action.action_size + (self.world.dim_c if not agent.silent else 0)
        if self.multidiscrete_actions:
            return agent.action_size + (1 if not agent.silent and self.world.dim_c != 0 else 0)
        return 1

    def get_agent_action_space(self, agent: Agent):
        if self.continuous_actions:
            n_comm = self.world.dim_c if not agent.silent else 0
            return spaces.Box(
                low=np.array((-agent.action.u_range_tensor).tolist() + [0] * n_comm, dtype=np.float32),
                high=np.array(agent.action.u_range_tensor.tolist() + [1] * n_comm, dtype=np.float32),
                shape=(self.get_agent_action_size(agent),),
                dtype=np.float32,
            )
        if self.multidiscrete_actions:
            actions = agent.discrete_action_nvec + (
                [self.world.dim_c] if not agent.silent and self.world.dim_c != 0 else []
            )
            return spaces.MultiDiscrete(actions)
        return spaces.Discrete(
            math.prod(agent.discrete_action_nvec)
            * (self.world.dim_c if not agent.silent and self.world.dim_c != 0 else 1)
        )

    def get_agent_observation_space(self, agent: Agent, obs: AGENT_OBS_TYPE):
        if isinstance(obs, Tensor):
            return spaces.Box(low=-np.float32("inf"), high=np.float32("inf"), shape=obs.shape[1:],
                              dtype=np.float32)
        if isinstance(obs, Dict):
            return spaces.Dict({k: self.get_agent_observation_space(agent, v) for k, v in obs.items()})
        raise NotImplementedError(f"Invalid type of observation {obs} for agent {agent.name}")

    # ---- actions ----------------------------------------------------------------------------------
    @staticmethod
    def _u_range_value(agent: Agent, index: int) -> float:
        r = agent.action.u_range
        r = r[index] if isinstance(r, Sequence) else r
        return _f32(r)

    @local_seed(vmas_random_state)
    def get_random_action(self, agent: Agent) -> torch.Tensor:
        """Random action with shape ``(agent.batch_dim, agent.action_size)`` (environment.py:524-582)."""
        return self._random_action(agent)

    def _column_plan(self, agent: Agent):
        """(batch, device, columns, [(low, high)] per column) of an agent's continuous random
        action, cached per agent and u_range value (the per-call range lookups cost more host
        time than the draws' launches)."""
        ur = agent.action.u_range
        key = (ur if type(ur) in (float, int) else tuple(ur), self.world.dim_c, agent.silent, agent.action_size,
               agent.batch_dim, agent.device)
        c = self._draw_plans.get(agent)
        if c is None or c[0] != key:
            n_c = self.world.dim_c if (self.world.dim_c != 0 and not agent.silent) else 0
            bounds = []
            for action_index in range(agent.action_size):
                r = self._u_range_value(agent, action_index)
                bounds.append((-r, r))
            bounds += [(0, 1)] * n_c
            c = self._draw_plans[agent] = (key, (agent.batch_dim, agent.device, len(bounds), bounds))
        return c[1]

    def _random_action(self, agent: Agent) -> torch.Tensor:
        if self.continuous_actions and self._column_draws(agent.device):
            # each column drawn in place of the [B, n] result: the same uniform_ calls on the
            # same numbers of elements as the reference's per-column tensors + stack, without
            # the stack kernel (checked once per device: _column_draws)
            B, dev, n, bounds = self._column_plan(agent)
            out = torch.empty(B, n, device=dev, dtype=torch.float32)
            for col, (lo, hi) in zip(out.unbind(1), bounds):
                col.uniform_(lo, hi)
            return out
        if self.continuous_actions:
            actions = []
            # (uniform_ overwrites every element: empty() draws the same numbers as zeros())
            for action_index in range(agent.action_size):
                r = self._u_range_value(agent, action_index)
                actions.append(
                    torch.empty(agent.batch_dim, device=agent.device, dtype=torch.float32).uniform_(-r, r)
                )
            if self.world.dim_c != 0 and not agent.silent:
                for _ in range(self.world.dim_c):
                    actions.append(
                        torch.empty(agent.batch_dim, device=agent.device, dtype=torch.float32).uniform_(0, 1)
                    )
            return torch.stack(actions, dim=-1)
        action_space = self.get_agent_action_space(agent)
        if self.multidiscrete_actions:
            actions = [
                torch.randint(low=0, high=int(action_space.nvec[i]), size=(agent.batch_dim,), device=agent.device)
                for i in range(action_space.shape[0])
            ]
            return torch.stack(actions, dim=-1)
        return torch.randint(low=0, high=action_space.n, size=(agent.batch_dim,), device=agent.device)

    def get_random_actions(self) -> Sequence[torch.Tensor]:
        """Random actions for all agents.  The reference swaps the host RNG states once per
        agent (environment.py:584-606); swapping once around the loop draws the identical
        streams.  Continuous actions on a GPU are drawn from the device generator only, which
        local_seed does not swap: the swap of the host states is a no-op there and is skipped.
        (Drawing them on a side stream, overlapped with the previous step's graph, measured
        slower: 87-98 M vs 106-119 M env-steps/s, interleaved runs on one MI355X.)"""
        if self.continuous_actions and self.device.type == "cuda":
            fused = self._fused_random_actions()
            if fused is not None:
                return fused
            return [self._random_action(agent) for agent in self.agents]
        return self._random_actions_seeded()

    # ---- every agent's random action columns in one native launch (GPU) ---------------------------
    _UNIFORM_MODES = _uniform.MODES  # (device, batch) -> probed vmas_uniform_columns mode

    def _fused_random_actions(self):
        """get_random_actions for continuous actions on a GPU: every agent's [B, n] action, drawn
        column by column with the same numbers and generator advance as the reference's per-column
        uniform_ calls (checked by _uniform.mode), in one launch instead of one per column."""
        agents = self.agents
        if not agents:
            return None
        c = self._uniform_cache
        if c is not None and c[1] is not None and self._uniform_same(c[2]):
            sp, self._spec = self._spec, None
            if sp is not None and sp[0] is c[1]:
                outs = self._take_spec(sp)
                if outs is not None:
                    return outs
            return self._uniform_draw(c[1])
        plans = [self._column_plan(a) for a in agents]
        B, dev = plans[0][0], plans[0][1]
        if c is None or len(c[0]) != len(plans) or any(a is not b for a, b in zip(c[0], plans)):
            key = tuple(plans)
            n_cols = sum(p[2] for p in plans)
            ok = (n_cols <= 32 and all(p[0] == B and p[1] == dev for p in plans)
                  and self._column_draws(dev) and _uniform.mode(torch.device(dev), B) is not None)
            if not ok:
                self._uniform_cache = (key, None)
                return None
            from ... import _native as N

            cols = np.zeros(n_cols, dtype=N.UNIFORM_COLUMN_DTYPE)
            k = 0
            for p in plans:
                for j, (lo, hi) in enumerate(p[3]):
                    cols[k]["stride"], cols[k]["from_"], cols[k]["to"] = p[2], lo, hi
                    k += 1
            d = torch.device(dev)
            idx = d.index if d.index is not None else torch.cuda.current_device()
            widths = [p[2] for p in plans]
            # column k's byte offset in the [A, B, n] allocation of equal widths
            offs = (np.array([a * 4 * B * widths[0] + 4 * j for a in range(len(widths)) for j in range(widths[0])],
                             dtype=np.uint64) if len(set(widths)) == 1 else None)
            c = (key, (N, cols, widths, idx, _uniform.mode(d, B), torch.cuda.default_generators[idx],
                       cols.ctypes.data, B, dev, offs))
        if c[1] is None:
            self._uniform_cache = c
            return None
        self._uniform_cache = (c[0], c[1], self._uniform_sig())
        return self._uniform_draw(c[1])

    # ---- random actions drawn ahead, inside the post-replay launch (graph mode) ------------------
    # In the loop env.step(env.get_random_actions()) the draw of step t + 1 is the next device work
    # after step t's post-replay copies.  When step t consumed a draw applied by its own launch,
    # the post-replay launch also draws step t + 1's actions (vmas_copy_spans_draw: one launch
    # instead of two) at the generator's current state, without advancing it; the next
    # get_random_actions hands that draw out -- and advances the generator -- only if nothing
    # changed the generator (seed and offset), the column plan or its applied-column fields in
    # between, else it draws as usual.  The draw rewrote the persistent action buffer, so the
    # agents' action.u / state.force show its snapshot meanwhile (_ActionShadow).
    _SPEC_DRAW = os.environ.get("VMAS_GRAPH_DRAW_AHEAD", "1") != "0"

    def _draw_ahead_plan(self):
        """(column plan, its UniformDraw, P) when the next draw can be made ahead, else None."""
        if not (self._SPEC_DRAW and self._spec_ok) or self._ushadow.active:
            return None
        c = self._uniform_cache
        if c is None or c[1] is None or len(c) < 3 or not self._uniform_same(c[2]):
            return None
        st = c[1]
        if st[9] is None or len(st[1]) > 16:  # (equal widths; at most 16 columns in the merged launch)
            return None
        N = st[0]
        h = self._uniform_host
        if h is None or h[0] is not st:
            h = self._uniform_host = (st, N.load_host().UniformDraw(
                st[3], st[7], len(st[2]), st[2][0], st[1], st[6], len(st[1]), [int(o) for o in st[9]], st[4],
                N.fn_addr("vmas_uniform_columns_snap"), N.fn_addr("vmas_aux_last_error")))
        if not self._preapply_columns(st):
            return None
        return st, h[1], self._u_persist[1]

    def _drew_ahead(self, st, acts, snap, seed, offset, inc) -> None:
        self._ushadow.arm(self._u_persist[1], snap)
        self._spec = (st, acts, seed, offset, inc, self._preapply_tag)

    def _take_spec(self, sp):
        """The draw made ahead, if it is what a draw now would give: the same generator state, the
        same column plan and applied-column fields."""
        st, acts, seed, offset, inc, tag = sp
        gen = st[5]
        if gen.initial_seed() != seed or gen.get_offset() != offset or not self._preapply_columns(st) \
                or self._preapply_tag is not tag:
            return None
        gen.set_offset(offset + inc)
        self._drawn = (tuple(acts), tuple(o.data_ptr() for o in acts), tuple(o._version for o in acts),
                       self._u_persist[1])
        self.drawn_ahead = getattr(self, "drawn_ahead", 0) + 1
        return acts

    # ---- random actions drawn and applied in one launch (graph mode) -----------------------------
    def _preapply_columns(self, st):
        """When the next step will replay a captured graph with the speculative action path, the
        draw kernel also writes every column as the action kernel would apply it (clamp to
        u_range, times u_multiplier) into the persistent action buffer the graph reads.  A step
        given exactly these tensors, unmodified, then needs no action launch: uniform draws from
        [-u_range, u_range] pass the NaN / range checks by construction (environment.py:621-655).
        Sets (or clears) the columns' second outputs; returns whether they are set."""
        cols = st[1]
        g = self._graph
        ok = (g is not None and g.graph is not None and self._can_speculate())
        if ok:
            c = self._apply_cache
            refs, sizes = c[1][0], c[1][4]
            widths = st[2]
            ok = list(widths) == list(sizes)
        if ok:
            key = (id(c), self._u_persist[1].data_ptr())
            pre = self._preapply
            if pre is None or pre[0] != key:
                pre = None
                vals = []
                for ag in self.agents:  # host copies of u_range / u_multiplier (once per apply plan)
                    r = ag.action.u_range_tensor.detach().cpu().tolist()
                    m = ag.action.u_multiplier_tensor.detach().cpu().tolist()
                    vals.append((r, m))
                base = self._u_persist[1].data_ptr()
                u_out, u_rng, u_mul = [], [], []
                k = 0
                good = True
                for i, ag in enumerate(self.agents):
                    r, m = vals[i]
                    for j in range(sizes[i]):
                        lo, hi = float(cols[k]["from_"]), float(cols[k]["to"])
                        good &= (lo == -np.float32(r[j]) and hi == np.float32(r[j]))
                        u_out.append(base + 4 * (int(refs[i]["out_offset"]) + j))
                        u_rng.append(r[j])
                        u_mul.append(m[j])
                        k += 1
                if good:
                    pre = (key, np.array(u_out, dtype=np.uint64), np.array(u_rng, dtype=np.float32),
                           np.array(u_mul, dtype=np.float32), np.array(sizes, dtype=np.int64).repeat(sizes))
                self._preapply = pre if pre is not None else (key, None)
            ok = self._preapply[1] is not None
        if ok:
            # (the five column fields are written once per (column table, plan, clamp), not per draw)
            # (the table itself in the tag, compared by identity: kept alive, its id cannot be reused)
            tag = getattr(self, "_preapply_tag", None)
            if tag is None or tag[0] is not cols or tag[1] != self._preapply[0] or tag[2] != bool(self.clamp_action):
                tag = (cols, self._preapply[0], bool(self.clamp_action))
                _, u_out, u_rng, u_mul, strides = self._preapply
                cols["u_out"], cols["u_stride"], cols["u_range"], cols["u_mult"] = u_out, strides, u_rng, u_mul
                cols["u_clamp"] = int(bool(self.clamp_action))
                self._preapply_tag = tag
        elif cols["u_out"].any():
            cols["u_out"] = 0
            self._preapply_tag = None
        return ok

    def _take_preapplied(self, actions) -> bool:
        """The step's actions are the last draw's tensors, unmodified, and that draw also wrote
        their applied values into the persistent action buffer: bind every agent's u to it (the
        speculative path's state after its action launch) and return True."""
        d = self._drawn
        self._drawn = None
        if (d is None or len(actions) != len(d[0]) or self._u_persist is None or d[3] is not self._u_persist[1]
                or getattr(self._graph, "copied", True)):
            return False
        for a, t, ptr, ver in zip(actions, d[0], d[1], d[2]):
            if a is not t or a.data_ptr() != ptr or a._version != ver:
                return False
        us = self._u_persist[2]
        if us is None:
            return False
        for i, ag in enumerate(self.agents):
            act = ag.action
            if act._u is not us[i]:  # (bound by the previous step already: the setter's checks passed)
                act.u = us[i]
        self.preapplied_steps += 1
        self._spec_ok = True
        return True

    def _uniform_sig(self):
        """What _column_plan's keys depend on, compared by identity (None when a u_range is a
        mutable sequence: then the plans are rebuilt every call)."""
        sig = []
        for a in self.agents:
            act = a.action
            ur = act.u_range
            if type(ur) not in (float, int):
                return None
            sig.append((a, act, ur, a.silent, a.action_size, a.batch_dim))
        # plain: every agent and action of the core classes' accessors (the properties only return
        # the underscored fields), so _uniform_same may read the fields without a Python frame each
        plain = all(_plain_accessors(type(a), type(a.action)) for a in self.agents)
        # the device the plan draws on (env.to(...) moves the world and its agents); the static
        # version and the agent list: nothing this compares was assigned since (core.STATIC_VERSION)
        return (self.world.dim_c, sig, self.world.device, self.world.batch_dim, plain, _core.STATIC_VERSION[0],
                self.agents)

    def _uniform_same(self, sig) -> bool:
        # (the version fast path only for the core classes' plain accessors: a subclass whose
        # u_range / silent / action_size property computes its value from an attribute the
        # STATIC_VERSION hooks do not see goes through the property comparison below)
        if sig is not None and sig[4] and sig[5] == _core.STATIC_VERSION[0] and sig[6] is self.agents:
            return True
        if (sig is None or sig[0] != self.world.dim_c or len(sig[1]) != len(self.agents)
                or sig[2] != self.world.device or sig[3] != self.world.batch_dim):
            return False
        if sig[4]:  # (every draw and every post-replay launch asks: the fields directly)
            for a, (ag, act, ur, sil, asz, bd) in zip(self.agents, sig[1]):
                d = a.__dict__
                if (a is not ag or d.get("_action") is not act or act.__dict__.get("_u_range") is not ur
                        or d.get("_silent") is not sil or d.get("action_size") != asz or d.get("_batch_dim") != bd):
                    return False
            return True
        for a, (ag, act, ur, sil, asz, bd) in zip(self.agents, sig[1]):
            if (a is not ag or a.action is not act or act.u_range is not ur or a.silent is not sil
                    or a.action_size != asz or a.batch_dim != bd):
                return False
        return True

    def _uniform_draw(self, st):
        N, cols, widths, idx, mode, gen, cols_addr, B, dev, offs = st
        if offs is not None:
            # equal widths: one [A, B, n] allocation, the column table, the launch and the
            # generator advance in one C++ call (csrc/vmas_host.cpp UniformDraw)
            h = self._uniform_host
            if h is None or h[0] is not st:
                h = self._uniform_host = (st, N.load_host().UniformDraw(
                    idx, B, len(widths), widths[0], cols, cols_addr, len(cols), [int(o) for o in offs], mode,
                    N.fn_addr("vmas_uniform_columns_snap"), N.fn_addr("vmas_aux_last_error")))
            pre = self._preapply_columns(st)
            sh = self._ushadow
            if pre and not sh.active:
                # the draw rewrites the persistent action buffer that agents' action.u (and a
                # holonomic agent's state.force) view until the step consumes the draw: their
                # current values go to a snapshot first, which those attributes show meanwhile
                # (the reference's draw has no side effect on the agents, environment.py:524-582)
                P = self._u_persist[1]
                outs, snap = h[1].draw(P.data_ptr(), P.numel())
                sh.arm(P, snap)
            else:
                outs, _ = h[1].draw(0, 0)
            self._drawn = (tuple(outs), tuple(o.data_ptr() for o in outs), tuple(o._version for o in outs),
                           self._u_persist[1]) if pre else None
            return outs
        f_out = cols["out"]
        if offs is not None:  # one allocation, one [B, n] view per agent (disjoint rows)
            buf = torch.empty(len(widths), B, widths[0], device=dev, dtype=torch.float32)
            outs = list(buf.unbind(0))
            np.add(offs, buf.data_ptr(), out=f_out, casting="unsafe")
        else:
            outs = []
            k = 0
            for n in widths:
                out = torch.empty(B, n, device=dev, dtype=torch.float32)
                base = out.data_ptr()
                for j in range(n):
                    f_out[k] = base + 4 * j
                    k += 1
                outs.append(out)
        pre = self._preapply_columns(st)
        _uniform.launch(idx, B, cols, mode, gen, cols_addr)
        self._drawn = (tuple(outs), tuple(o.data_ptr() for o in outs), tuple(o._version for o in outs),
                       self._u_persist[1]) if pre else None
        return outs

    @local_seed(vmas_random_state)
    def _random_actions_seeded(self) -> Sequence[torch.Tensor]:
        return [self._random_action(agent) for agent in self.agents]

    _COLUMN_DRAWS: Dict[str, bool] = {}

    @classmethod
    def _column_draws(cls, device) -> bool:
        """Whether uniform_ on a column view of a [B, n] tensor draws exactly what uniform_ on a
        contiguous [B] tensor draws from the same generator state, and advances the generator
        by the same amount (the philox counter depends on the element index, not the layout).
        Probed once per device with the global generator saved and restored around it."""
        key = str(device)
        ok = cls._COLUMN_DRAWS.get(key)
        if ok is None:
            dev = torch.device(device)
            B = 1031  # not a multiple of any launch geometry
            if dev.type == "cuda":
                gen = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
            else:
                gen = torch.default_generator
            saved = gen.get_state()
            try:
                a = torch.empty(B, device=dev).uniform_(-0.7, 0.7)
                b = torch.empty(B, device=dev).uniform_(-0.3, 0.3)
                after_ref = gen.get_state()
                gen.set_state(saved)
                out = torch.empty(B, 2, device=dev)
                out[:, 0].uniform_(-0.7, 0.7)
                out[:, 1].uniform_(-0.3, 0.3)
                ok = (torch.equal(out[:, 0], a) and torch.equal(out[:, 1], b)
                      and torch.equal(gen.get_state(), after_ref))
            finally:
                gen.set_state(saved)
            cls._COLUMN_DRAWS[key] = ok
        return ok

    def _check_discrete_action(self, action: Tensor, low: int, high: int, type: str):
        assert torch.all(
            (action >= torch.tensor(low, device=self.device)) * (action < torch.tensor(high, device=self.device))
        ), f"Discrete {type} actions are out of bounds, allowed int range [{low},{high})"

    def _validate_continuous_actions(self, actions):
        """NaN + range checks of every agent with one host sync (environment.py:621-623, 653-655).

        fp32 actions (the normal case) are checked by one native kernel (vmas_check_actions);
        other dtypes keep the reference's torch comparisons in their own dtype."""
        if all(a.dtype == torch.float32 for a in actions):
            from ... import _native as N

            n = len(actions)
            refs = np.zeros(n, dtype=N.ACTION_REF_DTYPE)
            keep = []
            for i, (action, agent) in enumerate(zip(actions, self.agents)):
                a = action.detach()
                if a.device != self.device:
                    a = a.to(self.device)
                r = agent.action.u_range_tensor
                keep += [a, r]
                refs[i] = (a.data_ptr(), r.data_ptr(), a.stride(0), a.stride(1), a.shape[1],
                           agent.action_size, int(bool(self.clamp_action)), 0)
            flags = np.zeros(2 * max(n, 1), dtype=np.uint8)
            dev = self.device
            if dev.type == "cuda":
                idx = dev.index if dev.index is not None else torch.cuda.current_device()
                stream = ctypes.c_void_p(torch.cuda.current_stream(idx).cuda_stream)
            else:
                idx, stream = -1, None
            N.check(N.load_library().vmas_check_actions(idx, self.num_envs, refs.ctypes.data, n,
                                                        flags.ctypes.data, stream), "vmas_check_actions")
            del keep
        else:
            checks = []
            for action, agent in zip(actions, self.agents):
                action = action.detach()
                physical = action[..., : agent.action_size]
                if self.clamp_action:
                    r = agent.action.u_range_tensor.unsqueeze(0).expand(physical.shape)
                    physical = physical.clamp(-r, r)
                checks.append(action.isnan().any())
                checks.append(torch.any(torch.abs(physical) > agent.action.u_range_tensor))
            flags = torch.stack(checks).tolist()
        for i, agent in enumerate(self.agents):
            if flags[2 * i] or flags[2 * i + 1]:
                # the reference's loop has set the actions of the agents before this one
                for j in range(i):
                    self._set_action(actions[j], self.agents[j], validated=True)
                if flags[2 * i]:
                    print()  # as the reference (environment.py:621-622)
                assert not flags[2 * i]
                assert not flags[2 * i + 1], (
                    f"Physical actions of agent {agent.name} are out of its range {agent.u_range}"
                )

    @property
    def graph_status(self) -> str:
        """Graph mode (graph_step=True): "warming" (eager steps before the capture), "graph"
        (replaying), "eager" (the step could not be captured; see graph_reason), "dropped"
        (parameters changed: eager, capturing again); "off" without graph mode."""
        return "off" if self._graph is None else self._graph.status

    @property
    def graph_reason(self) -> str:
        return "" if self._graph is None else getattr(self._graph, "why", "")

    def _apply_continuous_actions(self, actions, persistent: bool = False, speculative: bool = False):
        """_set_action of every agent in one native call (vmas_apply_actions), for continuous fp32
        actions without communication and without autograd: the NaN / range checks, the clamp
        and u = physical * u_multiplier of environment.py:615-709, one launch and no stream
        synchronisation.  Agents are then processed in order exactly as the reference loop does
        (agent i raises before its u is assigned; the agents before it keep their new u and
        noise).  Returns False when the case does not apply (the per-agent path runs).

        speculative (graph mode, no action noise, at most 8 agents): the kernel is only launched
        and the agents' u are bound to the persistent buffer; returns the launch's sequence number
        (or False) and the caller checks the flags later with _finish_speculative_actions."""
        agents = self.agents
        n = len(agents)
        # the persistent buffer is rewritten: a draw's applied values are stale, and so is a draw
        # made ahead into it (_take_spec would hand out actions whose applied values are gone)
        self._drawn = None
        self._spec = None
        self._ushadow.disarm()
        if n == 0:
            return False
        for a in actions:
            if a.dtype is not torch.float32 or (self.grad_enabled and a.requires_grad):
                return False
        dev = self.device
        B = self.num_envs
        c = self._apply_cache
        key = (tuple(agents), bool(self.clamp_action), B, self.world.dim_c, str(dev))
        if c is None or c[0] != key:
            if self.world.dim_c > 0 and any(not ag.silent for ag in agents):
                self._apply_cache = (key, None)
                return False
            from ... import _native as N

            refs = np.zeros(n, dtype=N.ACTION_APPLY_REF_DTYPE)
            sizes = [ag.action_size for ag in agents]
            offs = np.cumsum([0] + sizes[:-1]) * B
            tensors = []
            for i, ag in enumerate(agents):
                r, m = ag.action.u_range_tensor, ag.action.u_multiplier_tensor
                if r.dtype is not torch.float32 or m.dtype is not torch.float32:
                    self._apply_cache = (key, None)
                    return False
                tensors.append((r, m))
                refs[i]["u_range"], refs[i]["u_mult"] = r.data_ptr(), m.data_ptr()
                refs[i]["out_offset"], refs[i]["n_phys"] = int(offs[i]), sizes[i]
                refs[i]["clamp"] = int(bool(self.clamp_action))
            if dev.type == "cuda":
                idx = dev.index if dev.index is not None else torch.cuda.current_device()
            else:
                idx = -1
            fields = (refs["u"], refs["s0"], refs["s1"], refs["n_cols"])
            flags = np.zeros(max(16, (2 * n + 7) // 8 * 8), dtype=np.uint8)  # (whole uint64 words)
            # the arrays' addresses once (ndarray.ctypes builds a helper object per access: ~1.6 us)
            c = self._apply_cache = (key, (refs, fields, flags, tensors, sizes, sum(sizes), idx, N,
                                           refs.ctypes.data, flags.ctypes.data, flags.view(np.uint64)))
        st = c[1]
        if st is None:
            return False
        refs, (f_u, f_s0, f_s1, f_nc), flags, tensors, sizes, total, idx, N, refs_addr, flags_addr, _ = st
        for i, ag in enumerate(agents):  # range / multiplier tensors are cached by the Action
            if ag.action._u_range_tensor is not tensors[i][0] or ag.action._u_multiplier_tensor is not tensors[i][1]:
                self._apply_cache = None
                return self._apply_continuous_actions(actions, persistent, speculative)
        if speculative and (idx < 0 or n > 8 or any(ag.action.u_noise > 0 for ag in agents)):
            return False
        keep = []
        for i, a in enumerate(actions):
            if a.device != dev:
                a = a.to(dev)
            keep.append(a)
            s = a.stride()
            f_u[i], f_s0[i], f_s1[i], f_nc[i] = a.data_ptr(), s[0], s[1], a.shape[1]
        if persistent:  # graph mode: every step writes the same buffer / the same u views
            pc = self._u_persist
            if pc is None or pc[0] is not c:
                if self._graph is not None and self._graph.graph is not None:
                    # the captured step reads the previous buffer's views
                    self._graph.drop("action parameters changed")
                    if speculative:
                        return False
                pc = self._u_persist = (c, torch.empty(B * total, device=dev, dtype=torch.float32), None)
            out = pc[1]
        else:
            out = torch.empty(B * total, device=dev, dtype=torch.float32)
        stream = N.stream_ptr(idx) if idx >= 0 else None
        lib = N.load_library()
        if speculative:
            seq = ctypes.c_uint32(0)
            N.check_aux(lib.vmas_apply_actions_launch(idx, B, refs_addr, n, out.data_ptr(), ctypes.byref(seq), stream),
                        "vmas_apply_actions_launch")
            self._spec_keep = keep  # the kernel reads them: alive until the flags are in
        else:
            N.check_aux(lib.vmas_apply_actions(idx, B, refs_addr, n, out.data_ptr(), flags_addr, stream),
                        "vmas_apply_actions")
        del keep
        k = sizes[0]
        if persistent and self._u_persist[2] is not None:
            us = self._u_persist[2]
        elif all(sz == k for sz in sizes):
            us = out.view(n, B, k).unbind(0)
        else:
            us = [out.narrow(0, int(o), B * sz).view(B, sz) for o, sz in zip(refs["out_offset"], sizes)]
        if persistent and self._u_persist[2] is None:
            self._u_persist = (self._u_persist[0], out, us)
        if speculative:
            for i, ag in enumerate(agents):
                ag.action.u = us[i]
            return seq.value
        for i, ag in enumerate(agents):
            if flags[2 * i]:
                print()  # the reference prints an empty line before this assert (environment.py:621-622)
                assert not flags[2 * i]
            assert not flags[2 * i + 1], (
                f"Physical actions of agent {ag.name} are out of its range {ag.u_range}"
            )
            ag.action.u = us[i]
            if ag.action.u_noise > 0:
                noise = torch.randn(*ag.action.u.shape, device=self.device, dtype=torch.float32) * ag.u_noise
                ag.action.u += noise
        return True

    # Speculative replay (default; VMAS_GRAPH_SPECULATIVE=0 turns it off): launch the replay
    # before the action flags are known and roll the step back on a failed flag.  Interleaved
    # A/B: 1.5 % slower while the host path was heavy (profiles/r01/run11_host_path), 2.9 % faster
    # once it was trimmed (run 14: 140.0-140.8 vs 136.3-136.9 M env-steps/s): the GPU no longer
    # idles between the action kernel and the replay.
    _SPECULATE = os.environ.get("VMAS_GRAPH_SPECULATIVE", "1") != "0"

    def _can_speculate(self) -> bool:
        c = self._apply_cache
        if not (self._SPECULATE and c is not None and c[1] is not None and c[1][6] >= 0 and len(self.agents) <= 8
                and self._u_persist is not None and self._u_persist[0] is c):
            return False
        for ag in self.agents:  # (the Action's own field: u_noise is a property per call)
            if ag._action._u_noise > 0:
                return False
        return True

    def _speculative_flags_ok(self, seq: int) -> bool:
        """Waits for the flags of a speculative launch; True when every agent's actions pass."""
        st = self._apply_cache[1]
        idx, N, flags_addr, words = st[6], st[7], st[9], st[10]
        N.check_aux(N.load_library().vmas_apply_actions_flags(idx, seq, len(self.agents), flags_addr, N.stream_ptr(idx)),
                    "vmas_apply_actions_flags")
        self._spec_keep = None
        return not (int(words[0]) | int(words[1]))  # (speculation: at most 8 agents, 16 flag bytes)

    def _set_action(self, action, agent, validated: bool = False):
        # The reference clones the action so that its in-place ops never touch the caller's
        # tensor.  The continuous path without communication has no in-place op on it: u is made
        # out of place below (u = action * multiplier, the same values as clone + *=).
        no_comm = not (self.world.dim_c > 0 and not agent.silent)
        scaled = False
        if not (self.continuous_actions and no_comm):
            action = action.clone()
        comm_action = None
        if not self.grad_enabled:
            action = action.detach()
        action = action.to(self.device)
        if not validated:
            assert not action.isnan().any()
        if not self.continuous_actions:  # (the continuous branch below replaces u outright)
            agent.action.u = torch.zeros(self.batch_dim, agent.action_size, device=self.device, dtype=torch.float32)
        assert action.shape[1] == self.get_agent_action_size(agent), (
            f"Agent {agent.name} has wrong action size, got {action.shape[1]}, "
            f"expected {self.get_agent_action_size(agent)}"
        )
        if self.clamp_action and self.continuous_actions:
            physical_action = action[..., : agent.action_size]
            a_range = agent.action.u_range_tensor.unsqueeze(0).expand(physical_action.shape)
            physical_action = physical_action.clamp(-a_range, a_range)
            if self.world.dim_c > 0 and not agent.silent:
                comm_action = action[..., agent.action_size:]
                action = torch.cat([physical_action, comm_action.clamp(0, 1)], dim=-1)
            else:
                action = physical_action
        action_index = 0
        if self.continuous_actions:
            physical_action = action[:, action_index: action_index + agent.action_size]
            action_index += self.world.dim_p
            if not validated:
                assert not torch.any(torch.abs(physical_action) > agent.action.u_range_tensor), (
                    f"Physical actions of agent {agent.name} are out of its range {agent.u_range}"
                )
            if no_comm:
                agent.action.u = physical_action.to(torch.float32) * agent.action.u_multiplier_tensor
                scaled = True
            else:
                agent.action.u = physical_action.to(torch.float32)
        else:
            if not self.multidiscrete_actions:
                # flat index of the cartesian product of the discrete spaces -> multi-discrete
                flat_action = action.squeeze(-1)
                actions = []
                nvec = list(agent.discrete_action_nvec) + (
                    [self.world.dim_c] if not agent.silent and self.world.dim_c != 0 else []
                )
                for i in range(len(nvec)):
                    n = math.prod(nvec[i + 1:])
                    actions.append(flat_action // n)
                    flat_action = flat_action % n
                action = torch.stack(actions, dim=-1)
            for n in agent.discrete_action_nvec:
                physical_action = action[:, action_index]
                self._check_discrete_action(physical_action.unsqueeze(-1), low=0, high=n, type="physical")
                u_max = agent.action.u_range_tensor[action_index]
                # odd n: action 0 maps to u = 0 (swap 0 with the middle value)
                if n % 2 != 0:
                    stay = physical_action == 0
                    decrement = (physical_action > 0) & (physical_action <= n // 2)
                    physical_action[stay] = n // 2
                    physical_action[decrement] -= 1
                agent.action.u[:, action_index] = (physical_action / (n - 1)) * (2 * u_max) - u_max
                action_index += 1
        if not scaled:
            agent.action.u *= agent.action.u_multiplier_tensor
        if agent.action.u_noise > 0:
            noise = torch.randn(*agent.action.u.shape, device=self.device, dtype=torch.float32) * agent.u_noise
            agent.action.u += noise
        if self.world.dim_c > 0 and not agent.silent:
            if not self.continuous_actions:
                comm_action = action[:, action_index:]
                self._check_discrete_action(comm_action, 0, self.world.dim_c, "communication")
                comm_action = comm_action.long()
                agent.action.c = torch.zeros(self.num_envs, self.world.dim_c, device=self.device, dtype=torch.float32)
                agent.action.c.scatter_(1, comm_action, 1)
            else:
                if comm_action is None:
                    comm_action = action[:, action_index:]
                assert not torch.any(comm_action > 1) and not torch.any(comm_action < 0), (
                    "Comm actions are out of range [0,1]"
                )
                agent.action.c = comm_action
            if agent.c_noise > 0:
                noise = torch.randn(*agent.action.c.shape, device=self.device, dtype=torch.float32) * agent.c_noise
                agent.action.c += noise

    def render(self, *args, **kwargs):
        raise NotImplementedError("rendering is not part of the MI355X engine")

    @override(TorchVectorizedObject)
    def to(self, device: DEVICE_TYPING):
        device = torch.device(device)
        self.scenario.to(device)
        super().to(device)
        self._uniform_cache = None  # (the fused random-action plan holds device buffers)
