"""Fused continuous-action path (Environment._apply_continuous_actions -> vmas_apply_actions,
csrc/vmas_actions.hip) against the per-agent path (_validate_continuous_actions + _set_action,
the reference's environment.py:615-709 loop): identical u / force, clamp, noise draws, and the
reference's side effects when agent i raises (agents before it keep their new u)."""
import pytest
import torch

from vectorizedmultiagentsimulator_amd import make_env


def _pair(device, **kw):
    # (eager steps: the action paths themselves; graph mode's own use of them is tests/test_graph.py's)
    a = make_env("balance", num_envs=64, device=device, seed=3, n_agents=3, graph_step=False, **kw)
    b = make_env("balance", num_envs=64, device=device, seed=3, n_agents=3, graph_step=False, **kw)
    b._apply_continuous_actions = lambda actions, *args, **kw: False  # force the per-agent path
    return a, b


def _actions(env, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.rand(64, 2, generator=g) * 2 - 1).mul_(scale).to(env.device) for _ in env.agents]


def _check(device, clamp, scale):
    fused, ref = _pair(device, clamp_actions=clamp)
    for step in range(3):
        acts = _actions(fused, scale, seed=step)
        fused.step([x.clone() for x in acts])
        ref.step([x.clone() for x in acts])
        for x, y in zip(fused.agents, ref.agents):
            assert torch.equal(x.action.u, y.action.u)
            assert x.action.u.shape == y.action.u.shape and x.action.u.is_contiguous()
        for x, y in zip(fused.world.entities, ref.world.entities):
            assert torch.equal(x.state.pos, y.state.pos)
            assert torch.equal(x.state.vel, y.state.vel)


def test_fused_actions_match_per_agent_path():
    _check("cpu", clamp=False, scale=0.5)


def test_fused_actions_clamp_matches():
    _check("cpu", clamp=True, scale=3.0)


@pytest.mark.parametrize("bad", ["nan", "range"])
def test_fused_actions_failure_side_effects(bad):
    fused, ref = _pair("cpu")
    for env in (fused, ref):
        env.step(_actions(env, 0.5, seed=9))
    acts = _actions(fused, 0.5, seed=10)
    if bad == "nan":
        acts[1][7, 0] = float("nan")
    else:
        acts[1][7, 1] = 1.5
    before = [ag.action.u.clone() for ag in fused.agents]
    for env in (fused, ref):
        with pytest.raises(AssertionError) as ei:
            env.step([x.clone() for x in acts])
        if bad == "range":
            assert "out of its range" in str(ei.value)
    for i, (x, y) in enumerate(zip(fused.agents, ref.agents)):
        assert torch.equal(x.action.u, y.action.u), i
    # the reference's loop: agent 0 was processed, agent 1 raised before assigning its u
    assert torch.equal(fused.agents[0].action.u, acts[0] * fused.agents[0].action.u_multiplier_tensor)
    for i in (1, 2):
        assert torch.equal(fused.agents[i].action.u, before[i])


def test_fused_actions_noise_draws_match():
    fused, ref = _pair("cpu")
    for env in (fused, ref):
        for ag in env.agents:
            ag.action._u_noise = 0.1
    # the simulator's RNG state is shared by all environments (class attribute, as the
    # reference): give both steps the same one
    shared = type(fused).vmas_random_state
    saved = list(shared)
    for env in (fused, ref):
        shared[:] = saved
        env.step(_actions(env, 0.5, seed=4))
    for x, y in zip(fused.agents, ref.agents):
        assert torch.equal(x.action.u, y.action.u)


def test_fused_actions_skipped_for_other_dtypes():
    env = make_env("balance", num_envs=8, seed=0, n_agents=2)
    assert env._apply_continuous_actions([torch.zeros(8, 2, dtype=torch.float64)] * 2) is False


@pytest.mark.gpu
@pytest.mark.parametrize("clamp,scale", [(False, 0.5), (True, 3.0)])
def test_fused_actions_match_per_agent_path_gpu(gpu_device, clamp, scale):
    _check(gpu_device, clamp, scale)


@pytest.mark.gpu
def test_fused_actions_failure_gpu(gpu_device):
    env = make_env("balance", num_envs=32768, device=gpu_device, seed=0, n_agents=4)
    acts = env.get_random_actions()
    env.step(acts)
    bad = [a.clone() for a in acts]
    bad[3][32767, 1] = float("nan")
    with pytest.raises(AssertionError):
        env.step(bad)
    bad = [a.clone() for a in acts]
    bad[2][12345, 0] = 2.0
    with pytest.raises(AssertionError, match="out of its range"):
        env.step(bad)
    env.step(acts)  # the device flags were reset: a valid step passes again
