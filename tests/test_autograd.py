"""Autograd through the native path (csrc/vmas_grad.hip, simulator/_engine.py _StepFn / _DistFn /
_RaysFn): the reference's World is a plain torch program, so ``Environment(grad_enabled=True)``
lets a loss over several steps be differentiated w.r.t. actions and state
(ref vmas/simulator/environment/environment.py:55, tests/test_vmas.py:277-304).

Oracle: the CPU restatement of the reference's step / distance / ray programs (oracle/vmas_oracle.py)
differentiated by torch.autograd on the same inputs.  The native VJPs evaluate the same fp32 physics
on forward-mode dual numbers, so the gradients agree to fp32 rounding amplified by the contact
model's stiffness; the tolerance is relative to each field's gradient scale (see _close)."""

import pytest
import torch

from oracle import vmas_oracle as O
from vectorizedmultiagentsimulator_amd import make_env

from _parity import make

FIELDS = ("pos", "vel", "rot", "ang_vel")
AGENT_FIELDS = ("force", "torque")

# scenarios without scripted agents (World.step would call an action script between the leaves
# and the step): every narrowphase class, joints, friction / clamps / gravity
GRAD_SCENARIOS = [
    ("balance", dict(n_agents=4), 10),
    ("transport", dict(n_agents=4), None),
    ("waterfall", dict(n_agents=5), None),
    ("pollock", dict(n_agents=4, n_lines=3, n_boxes=3, lidar=False), None),
    ("features", dict(n_agents=4), None),
]


def _close(name, got, exp, rtol=2e-3, bad_frac=0.02):
    """Per-env comparison at ``rtol`` x the field's gradient scale (its largest |exp|, at least
    1).  A few envs may sit on a branch boundary of the contact model (a soft-contact cut-off, a
    tie between closest points), where one fp32 rounding picks the other side's derivative: at
    most ``bad_frac`` of the envs may differ."""
    assert got.shape == exp.shape, (name, got.shape, exp.shape)
    assert torch.isfinite(got).all(), name
    scale = max(float(exp.abs().max()), 1.0)
    bad = ((got - exp).abs() > rtol * scale).reshape(got.shape[0], -1).any(-1)
    assert int(bad.sum()) <= bad_frac * got.shape[0], (
        f"{name}: {int(bad.sum())}/{got.shape[0]} envs differ; max |d| = "
        f"{float((got - exp).abs().max()):.3g} at scale {scale:.3g}")


def _leaves(world, snap, device):
    """Fresh leaf tensors of one snapshot: set into the native world and into an oracle copy."""
    eng, ora = {}, {}
    for i, e in enumerate(world.entities):
        names = FIELDS + (AGENT_FIELDS if "force" in snap[i] else ())
        ora[i] = {}
        for k in names:
            v = snap[i][k]
            t = v.to(device).clone().requires_grad_(True)
            setattr(e.state, k, t)
            eng[(i, k)] = t
            ora[i][k] = v.clone().requires_grad_(True)
    return eng, ora


def _weights(snap, seed):
    g = torch.Generator().manual_seed(seed)
    return {i: {k: torch.randn(v.shape, generator=g) for k, v in d.items()} for i, d in snap.items()}


def step_grad_parity(env, seed=0):
    """d(sum of random weights x every output of one World.step) / d(every input): native vs oracle."""
    w = env.world
    snap = O.snapshot(w)
    eng, ora = _leaves(w, snap, w.device)
    W = _weights(snap, seed)
    w.step()
    loss = 0.0
    for i, e in enumerate(w.entities):
        for k in W[i]:
            loss = loss + (getattr(e.state, k).cpu() * W[i][k]).sum()
    loss.backward()

    ow = O.OracleWorld(w, ora)
    ow.step()
    res = ow.result()
    oloss = 0.0
    for i in res:
        for k in W[i]:
            oloss = oloss + (res[i][k] * W[i][k]).sum()
    oloss.backward()
    n_checked = 0
    for (i, k), t in eng.items():
        exp = ora[i][k].grad
        got = t.grad
        if exp is None:  # the input does not reach the loss in the reference either
            assert got is None or not got.any(), (w.entities[i].name, k)
            continue
        assert got is not None, (w.entities[i].name, k)
        _close(f"{w.entities[i].name}.{k}", got.cpu(), exp)
        n_checked += 1
    assert n_checked > 0


def _prepare(name, kw, substeps, device, n_envs=64, warm=3):
    env = make(name, kw, substeps, device, n_envs, seed=1)
    for _ in range(warm):  # into contact
        env.step(env.get_random_actions())
    return env


@pytest.mark.parametrize("name,kw,substeps", GRAD_SCENARIOS, ids=[s[0] for s in GRAD_SCENARIOS])
def test_step_vjp_matches_oracle_autograd_host(name, kw, substeps):
    step_grad_parity(_prepare(name, kw, substeps, "cpu"))


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps", GRAD_SCENARIOS, ids=[s[0] for s in GRAD_SCENARIOS])
def test_step_vjp_matches_oracle_autograd_gpu(gpu_device, name, kw, substeps):
    step_grad_parity(_prepare(name, kw, substeps, gpu_device, n_envs=256))


def query_grad_parity(env, seed=0):
    """get_distance for every entity pair, get_distance_from_point and every agent LIDAR:
    gradients w.r.t. positions / rotations / test points / ray angles, native vs oracle."""
    w = env.world
    snap = O.snapshot(w)
    g = torch.Generator().manual_seed(seed)
    n = len(w.entities)
    pairs = [(a, b) for a in range(n) for b in range(a + 1, n)]
    tp = torch.randn(w.batch_dim, 2, generator=g)
    for a, b in pairs[:40] + [(a, None) for a in range(n)]:
        eng, ora = _leaves(w, snap, w.device)
        ow = O.OracleWorld(w, ora)
        gw = torch.randn(w.batch_dim, generator=g)
        if b is None:
            tpe = tp.to(w.device).clone().requires_grad_(True)
            tpo = tp.clone().requires_grad_(True)
            got = w.get_distance_from_point(w.entities[a], tpe)
            exp = ow.get_distance_from_point(ow.ents[a], tpo)
        else:
            got = w.get_distance(w.entities[a], w.entities[b])
            exp = ow.get_distance(ow.ents[a], ow.ents[b])
        torch.testing.assert_close(got.detach().cpu(), exp.detach(), atol=2e-5, rtol=2e-5)
        (got.cpu() * gw).sum().backward()
        (exp * gw).sum().backward()
        for idx in (a, b):
            if idx is None:
                continue
            for k in ("pos", "rot"):
                ge, go = eng[(idx, k)].grad, ora[idx][k].grad
                if go is None:
                    assert ge is None or not ge.any()
                    continue
                _close(f"dist {a},{b} {w.entities[idx].name}.{k}", ge.cpu(), go)
        if b is None:
            _close(f"dist point {a}", tpe.grad.cpu(), tpo.grad)

    for ai, agent in enumerate(w.agents):
        idx = w.entities.index(agent)
        for sensor in agent.sensors:
            eng, ora = _leaves(w, snap, w.device)
            ow = O.OracleWorld(w, ora, grad_safe=True)
            angles = sensor._angles.detach().cpu()  # [B, n_rays]
            ae = angles.to(w.device).clone().requires_grad_(True)
            ao = angles.clone().requires_grad_(True)
            got = w.cast_rays(agent, ae + eng[(idx, "rot")], sensor._max_range, sensor.entity_filter)
            exp = ow.cast_rays(idx, ao + ora[idx]["rot"], sensor._max_range, sensor.entity_filter)
            gw = torch.randn(exp.shape, generator=g)
            (got.cpu() * gw).sum().backward()
            (exp * gw).sum().backward()
            _close(f"rays {agent.name} angles", ae.grad.cpu(), ao.grad)
            for i in range(len(w.entities)):
                for k in ("pos", "rot"):
                    ge, go = eng[(i, k)].grad, ora[i][k].grad
                    if go is None:
                        assert ge is None or not ge.any(), (agent.name, w.entities[i].name, k)
                        continue
                    _close(f"rays {agent.name} {w.entities[i].name}.{k}", ge.cpu(), go)


QUERY_SCENARIOS = [
    ("pollock", dict(n_agents=3, n_lines=3, n_boxes=3, lidar=True), None),
    ("discovery", dict(n_agents=3, use_agent_lidar=True), None),
]


@pytest.mark.parametrize("name,kw,substeps", QUERY_SCENARIOS, ids=[s[0] for s in QUERY_SCENARIOS])
def test_query_vjps_match_oracle_autograd_host(name, kw, substeps):
    query_grad_parity(_prepare(name, kw, substeps, "cpu", n_envs=32, warm=2))


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps", QUERY_SCENARIOS, ids=[s[0] for s in QUERY_SCENARIOS])
def test_query_vjps_match_oracle_autograd_gpu(gpu_device, name, kw, substeps):
    query_grad_parity(_prepare(name, kw, substeps, gpu_device, n_envs=128, warm=2))


# ---- restated reference test (tests/test_vmas.py:277-304) --------------------------------------
# the reference's list is vmas.scenarios + mpe_scenarios minus football / simple_crypto /
# road_traffic; of those this package has the four benchmark scenarios; waterfall
# (debug) adds joints
DIFF_SCENARIOS = ["balance", "discovery", "flocking", "transport", "waterfall"]


def differentiable(scenario, device, n_steps=10, n_envs=10):
    env = make_env(scenario, num_envs=n_envs, device=device, continuous_actions=True, seed=0, grad_enabled=True)
    for step in range(n_steps):
        actions = []
        for agent in env.agents:
            action = env.get_random_action(agent)
            action.requires_grad_(True)
            if step == 0:
                first_action = action
            actions.append(action)
        obs, rews, dones, info = env.step(actions)
    loss = obs[-1].mean() + rews[-1].mean()
    (grad,) = torch.autograd.grad(loss, first_action)  # connected through all 10 steps
    assert torch.isfinite(grad).all()
    return grad


@pytest.mark.parametrize("scenario", DIFF_SCENARIOS)
def test_vmas_differentiable_host(scenario):
    differentiable(scenario, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", DIFF_SCENARIOS)
def test_vmas_differentiable_gpu(gpu_device, scenario):
    g = differentiable(scenario, gpu_device)
    assert g.is_cuda


def _chain_loss(device, n_steps, u0):
    env = make_env("balance", num_envs=4, device=device, seed=0, grad_enabled=True, n_agents=3)
    u = u0.to(device).requires_grad_(True)
    for _ in range(n_steps):
        env.step([u[i] for i in range(len(env.agents))])
    loss = sum((a.state.pos ** 2).sum() for a in env.agents) + env.scenario.package.state.pos.sum()
    (g,) = torch.autograd.grad(loss, u)
    return loss.detach().cpu(), g.cpu()


def test_multi_step_chain_matches_finite_difference_host():
    """A loss after 4 steps w.r.t. the actions (one leaf, used by every step): the chained
    VJPs against a central finite difference (fp32 forward, so a loose tolerance)."""
    u0 = torch.rand(3, 4, 2, generator=torch.Generator().manual_seed(0)) * 0.2 - 0.1
    _, g = _chain_loss("cpu", 4, u0)
    assert g.abs().sum() > 0
    d = torch.zeros_like(u0)
    d[1, 2, 0] = 1.0
    h = 1e-2
    lp, _ = _chain_loss("cpu", 4, u0 + h * d)
    lm, _ = _chain_loss("cpu", 4, u0 - h * d)
    fd = float(lp - lm) / (2 * h)
    assert abs(fd - float(g[1, 2, 0])) <= 0.05 * max(abs(fd), 1e-2), (fd, float(g[1, 2, 0]))
