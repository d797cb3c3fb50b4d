"""local_seed's numpy RNG swap (environment/_rng.py) must behave exactly like the reference's
get_state/set_state swap (environment.py:30-46): same draws inside and outside the simulator's
context, gaussian cache included (odd numbers of legacy normal draws on both sides)."""
import contextlib
import random

import numpy as np
import pytest
import torch

from vectorizedmultiagentsimulator_amd.simulator.environment import environment as envmod
from vectorizedmultiagentsimulator_amd.simulator.environment._rng import numpy_global_rng, python_global_rng


@contextlib.contextmanager
def reference_local_seed(state):  # the reference's swap, verbatim semantics
    t, n, p = torch.random.get_rng_state(), np.random.get_state(), random.getstate()
    torch.random.set_rng_state(state[0])
    np.random.set_state(state[1])
    random.setstate(state[2])
    yield
    state[0], state[1], state[2] = torch.random.get_rng_state(), np.random.get_state(), random.getstate()
    torch.random.set_rng_state(t)
    np.random.set_state(n)
    random.setstate(p)


def _script(ctx_factory):
    """Interleaved draws inside/outside the simulator context; returns every value drawn."""
    torch.manual_seed(11)
    np.random.seed(11)
    random.seed(11)
    np.random.normal()  # the user's side has a cached gaussian when the context is entered
    torch.manual_seed(5)
    np.random.seed(5)
    random.seed(5)
    inner = [torch.random.get_rng_state(), np.random.get_state(), random.getstate()]
    torch.manual_seed(11)
    np.random.seed(11)
    random.seed(11)
    np.random.normal()
    out = []
    for i in range(6):
        with ctx_factory(inner):
            out += list(np.random.normal(size=1 + i % 2))  # odd / even gaussian counts
            out += list(np.random.uniform(size=3))
            out += [torch.rand(2).tolist(), random.random()]
        out += list(np.random.normal(size=1 + (i + 1) % 2))
        out += [np.random.randint(1000), torch.rand(1).item(), random.random()]
    return out


def test_fast_swap_is_active_and_exact():
    assert numpy_global_rng().fast  # the offset probe validated on this numpy build
    assert python_global_rng().fast  # ... and on this CPython build
    saved = np.random.get_state()
    try:
        expected = _script(reference_local_seed)
        got = _script(envmod.local_seed)
    finally:
        np.random.set_state(saved)
    assert len(expected) == len(got)
    for a, b in zip(expected, got):
        assert a == b


def test_python_rng_swap_round_trips():
    r = python_global_rng()
    st = random.getstate()
    try:
        random.seed(9)
        random.gauss(0, 1)  # leaves gauss_next cached
        snap, want = r.snapshot(), random.getstate()
        a = [random.random(), random.gauss(0, 1), random.getrandbits(70)]
        random.seed(1234)
        r.restore(snap)
        assert random.getstate() == want
        assert [random.random(), random.gauss(0, 1), random.getrandbits(70)] == a
        r.restore(want)  # getstate() tuples are accepted too
        assert random.getstate() == want
    finally:
        random.setstate(st)


def test_restore_accepts_legacy_tuples():
    r = numpy_global_rng()
    st = np.random.get_state()
    np.random.seed(3)
    a = np.random.normal(size=3)
    r.restore(st)
    np.random.seed(3)
    assert np.array_equal(a, np.random.normal(size=3))
    np.random.set_state(st)


def _random_actions_both_ways(device):
    from vectorizedmultiagentsimulator_amd import make_env
    from vectorizedmultiagentsimulator_amd.simulator.environment import Environment

    env = make_env("balance", num_envs=777, device=device, seed=5, n_agents=3)
    cuda = env.device.type == "cuda"
    saved = [x.clone() if isinstance(x, torch.Tensor) else x for x in Environment.vmas_random_state]
    saved_cuda = torch.cuda.get_rng_state(env.device) if cuda else None
    key = str(env.device)
    Environment._COLUMN_DRAWS[key] = False  # the reference's per-column tensors + stack
    ref = env.get_random_actions()
    after_ref = [x.clone() if isinstance(x, torch.Tensor) else x for x in Environment.vmas_random_state]
    after_cuda = torch.cuda.get_rng_state(env.device) if cuda else None
    Environment.vmas_random_state[:] = saved
    if cuda:
        torch.cuda.set_rng_state(saved_cuda, env.device)
    Environment._COLUMN_DRAWS.pop(key)
    assert Environment._column_draws(env.device)
    fast = env.get_random_actions()
    for a, b in zip(ref, fast):
        assert a.shape == b.shape and torch.equal(a, b)
    assert torch.equal(Environment.vmas_random_state[0], after_ref[0])
    if cuda:
        assert torch.equal(torch.cuda.get_rng_state(env.device), after_cuda)


def test_random_actions_column_draws_match_reference_pattern():
    _random_actions_both_ways("cpu")


@pytest.mark.gpu
def test_random_actions_column_draws_match_reference_pattern_gpu(gpu_device):
    _random_actions_both_ways(gpu_device)


@pytest.mark.gpu
@pytest.mark.parametrize("name,n_agents,B", [("balance", 4, 32768), ("flocking", 8, 1031), ("transport", 3, 70001)])
def test_fused_random_actions_equal_per_column_uniform_gpu(gpu_device, name, n_agents, B):
    """get_random_actions on a GPU draws every agent's columns in one launch
    (vmas_uniform_columns); the numbers and the generator advance equal the reference's
    per-column torch uniform_ calls (environment.py:524-606) bit for bit."""
    from vectorizedmultiagentsimulator_amd import make_env
    from vectorizedmultiagentsimulator_amd.simulator.environment import Environment

    env = make_env(name, num_envs=B, device=gpu_device, seed=3, n_agents=n_agents)
    gen = torch.cuda.default_generators[env.device.index or 0]
    env.get_random_actions()  # probes the mode for this batch size
    assert Environment._UNIFORM_MODES[(str(env.device), B)] is not None
    for _ in range(3):
        saved = gen.get_state()
        ref = []
        for agent in env.agents:
            cols = []
            for i in range(agent.action_size):
                r = env._u_range_value(agent, i)
                cols.append(torch.empty(B, device=env.device).uniform_(-r, r))
            ref.append(torch.stack(cols, dim=-1))
        after = gen.get_state()
        gen.set_state(saved)
        got = env.get_random_actions()
        assert env._uniform_cache[1] is not None  # the fused path ran
        assert torch.equal(gen.get_state(), after)
        for a, b in zip(ref, got):
            assert a.shape == b.shape and torch.equal(a, b)
