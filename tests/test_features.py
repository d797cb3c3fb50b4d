"""The optional branches of the step (scenarios/debug/features.py) and the world attributes the
step reads, against the oracle: friction, force/torque clamps written back to the agent state,
max_speed / v_range, [B, 2] entity gravity, hollow boxes, communication state, and the
``_sub_dt`` attribute read as such (ref core.py:2068, 2870, 2879, 2905, 2907)."""
import pytest
import torch

from oracle import vmas_oracle as O
from tests._parity import assert_aggregate, make, step_parity, summarize


def _check_comm(env):
    """core.py:2909-2912: after the step a non-silent agent's state.c IS its action.c."""
    for a in env.world.agents:
        if a.silent:
            assert a.state.c is None
        else:
            assert a.state.c is a.action.c
            assert a.state.c.shape == (env.world.batch_dim, env.world.dim_c)


def _check_clamps(env):
    """core.py:2017-2040: the clamped force / torque is written back to the agent's state."""
    for a in env.world.agents:
        f, t = a.state.force, a.state.torque
        if a.max_f is not None:
            assert float(torch.linalg.vector_norm(f, dim=-1).max()) <= a.max_f * (1 + 1e-6)
        if a.f_range is not None:
            assert f.abs().max() <= torch.tensor(a.f_range, dtype=torch.float32)
        if a.max_t is not None:
            assert float(t.abs().max()) <= a.max_t * (1 + 1e-6)
        if a.t_range is not None:
            assert t.abs().max() <= torch.tensor(a.t_range, dtype=torch.float32)


def _sub_dt_parity(device, num_envs):
    env = make("features", dict(n_agents=4), None, device, num_envs=num_envs, seed=5)
    w = env.world
    env.step(env.get_random_actions())
    # _substeps changed without _sub_dt (and then the reverse): the reference reads both
    # attributes independently, so must the engine
    w._substeps = 6
    rep = O.compare_one_step(w)
    assert rep["ok"], rep
    assert abs(w._sub_dt - w._dt / 4) < 1e-12
    w._sub_dt = 0.013
    rep = O.compare_one_step(w)
    assert rep["ok"], rep


def test_features_branches_host():
    env = make("features", dict(n_agents=4), None, "cpu", num_envs=64, seed=3)
    for rep in step_parity(env, n_steps=3):
        assert rep["ok"], rep
    _check_comm(env)
    _check_clamps(env)


def test_sub_dt_attribute_host():
    _sub_dt_parity("cpu", 48)


@pytest.mark.gpu
@pytest.mark.parametrize("math", ["relaxed", "exact"])
def test_features_full_size_gpu(gpu_device, monkeypatch, math):
    """The same 16 384-env world and seed in both math modes: the relaxed / exact pair of PARITY
    lines separates what relaxed math costs from the world's own conditioning (band_max)."""
    if math == "exact":
        monkeypatch.setenv("VMAS_JIT_MATH", "exact")
    env = make("features", dict(n_agents=8), None, gpu_device, num_envs=16384, seed=0)
    reps = step_parity(env, n_steps=2)
    rec = summarize(f"features 16384 envs n_agents=8 {math}-math", env, reps)
    assert rec["math"] == math
    # ~10x the relaxed-math p99.9 / mean of round 4 (exact math measured 3-8x below them; the
    # max |diff| of both, 1e-4 rot / 1e-3 ang_vel, is the world's conditioning: DESIGN.md (c))
    assert_aggregate(rec, p999_bound={"pos": 2.4e-6, "vel": 3e-5, "rot": 2.2e-5, "ang_vel": 4.6e-4},
                     mean_bound={"pos": 8.5e-8, "vel": 8.7e-7, "rot": 1.1e-6, "ang_vel": 1.8e-5})
    for rep in reps:
        assert rep["ok"], rep
    assert env.world.engine.kernel_name == "k_world", env.world.engine.jit_error
    _check_comm(env)
    _check_clamps(env)


@pytest.mark.gpu
def test_sub_dt_attribute_gpu(gpu_device):
    _sub_dt_parity(gpu_device, 300)
