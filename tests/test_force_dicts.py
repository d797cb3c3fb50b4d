"""World.forces_dict / torques_dict (ref core.py:1975-2198): with ``world.export_forces = True`` the
step leaves each entity's force and torque totals of the LAST substep, as the reference's
accumulators hold them after World.step.  Checked against the oracle's accumulators on the same
state, on the host backend (CPU) and on gfx950 through k_world and the generic k_step.

Tolerance: the state parity's velocity tolerance (1e-4, oracle.vmas_oracle.compare) carried to
the force that produces it in one substep: 1e-4 * mass / sub_dt for a force, 1e-4 * moment of
inertia / sub_dt for a torque (k_world's relaxed math in jointless worlds, and joint gains that
amplify last-bit differences of earlier substeps, move the last substep's totals by that much), plus
1e-4 of the field's largest magnitude over the batch, plus 4x the oracle's own 1-ulp sensitivity
band of the totals (as the state parity adds O.sensitivity_band).  An env whose step passed within a few ulps of a contact cut-off (the oracle's
certified cut-off margin) may differ by any amount, as the state parity allows."""
import pytest
import torch

from oracle import vmas_oracle as O
from tests._parity import make

CUTOFF_TOL = 4e-6


def _force_band(world, snap, ow, n=2, eps=1.2e-7, seed=1234):
    """The oracle's own conditioning of the totals (as O.sensitivity_band for the state): max
    change of each entity's last-substep force / torque under ~1-ulp relative input perturbations."""
    g = torch.Generator().manual_seed(seed)
    band = {}
    for _ in range(n):
        pert = {i: {k: v * (1 + eps * torch.randn(v.shape, generator=g)) for k, v in d.items()}
                for i, d in snap.items()}
        _, pw = O.oracle_step(world, pert, "batch")
        for i, (oe, pe) in enumerate(zip(ow.ents, pw.ents)):
            for key, a, b in (("f", ow.forces_dict[oe], pw.forces_dict[pe]), ("t", ow.torques_dict[oe], pw.torques_dict[pe])):
                d = (a - b).abs().nan_to_num(0.0)
                band[i, key] = torch.maximum(band[i, key], d) if (i, key) in band else d
    return band


def _check(world, rtol=1e-4, steps=3):
    for _ in range(steps):
        snap = O.snapshot(world)
        _, ow = O.oracle_step(world, snap, "batch")
        band = _force_band(world, snap, ow)
        world.export_forces = True
        world.step()
        certified = ow.cutoff_margin <= CUTOFF_TOL
        n = 0
        for i, e in enumerate(world.entities):
            oe = ow.ents[i]
            tol_f, tol_t = (1e-4 * e.mass / world._sub_dt, 1e-4 * e.moment_of_inertia / world._sub_dt)
            for got, exp, atol, key in ((world.forces_dict[e], ow.forces_dict[oe], tol_f, "f"),
                                        (world.torques_dict[e], ow.torques_dict[oe], tol_t, "t")):
                assert got.shape == exp.shape
                got = got.detach().cpu()
                # rtol against the field's largest magnitude over the batch: a total is a sum of
                # terms (contacts, joints) that cancel, so its error scales with the terms, not the sum
                lim = atol + rtol * exp.abs().max() + 4 * band[i, key]
                bad = ((got - exp).abs() > lim).any(-1) & ~certified
                if bad.any():
                    j = int(bad.nonzero()[0, 0])
                    raise AssertionError(f"{e.name} {key}: {int(bad.sum())} envs, env {j}: got {got[j].tolist()} "
                                         f"expected {exp[j].tolist()} limit {lim[j].tolist()}")
                n += int((exp != 0).any(-1).sum())
        assert n > 0  # some entity received a non-zero force


def _features(device, num_envs):
    env = make("features", dict(n_agents=4), None, device, num_envs=num_envs, seed=11)
    env.step(env.get_random_actions())
    return env


def test_force_dicts_by_default():
    """Like the reference (core.py:1975-1992), every step leaves forces_dict / torques_dict; a
    world with export_forces = False has none."""
    env = make("balance", dict(n_agents=2), None, "cpu", num_envs=4, seed=0)
    env.step(env.get_random_actions())
    fd = env.world.forces_dict
    assert set(fd) == set(env.world.entities)
    assert all(v.shape == (4, 2) for v in fd.values())
    assert all(v.shape == (4, 1) for v in env.world.torques_dict.values())
    env.world.export_forces = False
    env.step(env.get_random_actions())
    with pytest.raises(AttributeError, match="export_forces"):
        env.world.forces_dict


@pytest.mark.parametrize("name,kw", [("features", dict(n_agents=4)), ("waterfall", dict(n_agents=5))])
def test_export_kernel_compiles(name, kw):
    env = make(name, kw, None, "cpu", num_envs=8, seed=0)
    env.world.export_forces = True
    src = env.world.engine.jit_compile_check()
    assert "float* out[8]" in src and "lfx" in src


def test_force_dicts_host():
    _check(_features("cpu", 64).world)


def test_force_dicts_host_joints():
    env = make("waterfall", dict(n_agents=5), None, "cpu", num_envs=32, seed=2)
    env.step(env.get_random_actions())
    _check(env.world)


@pytest.mark.gpu
def test_force_dicts_k_world_gpu(gpu_device):
    env = _features(gpu_device, 256)
    assert env.world.engine.kernel_name == "k_world"
    _check(env.world)


@pytest.mark.gpu
def test_force_dicts_k_world_joints_gpu(gpu_device):
    env = make("waterfall", dict(n_agents=5), None, gpu_device, num_envs=200, seed=2)
    env.step(env.get_random_actions())
    assert env.world.engine.kernel_name == "k_world"
    _check(env.world)


@pytest.mark.gpu
def test_force_dicts_k_step_gpu(gpu_device, monkeypatch):
    monkeypatch.setenv("VMAS_JIT", "0")
    env = _features(gpu_device, 256)
    assert env.world.engine.kernel_name == "k_step"
    _check(env.world)


@pytest.mark.gpu
def test_export_leaves_the_step_unchanged_gpu(gpu_device):
    """The export only adds stores: the integrated state is bit-identical with and without it."""
    env = _features(gpu_device, 512)
    w = env.world
    snap = O.snapshot(w)
    w.export_forces = False
    w.step()
    off = O.snapshot(w)
    O.load_snapshot(w, snap)
    w.export_forces = True
    w.step()
    on = O.snapshot(w)
    for i in off:
        for k in off[i]:
            assert torch.equal(off[i][k], on[i][k]), (i, k)


@pytest.mark.gpu
def test_force_dicts_graph_mode_gpu(gpu_device):
    """A replayed step exports the same totals as the eager step (bit-identical), through the
    graph's own buffer (graph mode: views of the graph's tensors)."""
    from vectorizedmultiagentsimulator_amd import make_env

    envs = [make_env("balance", num_envs=256, device=gpu_device, seed=0, graph_step=g, n_agents=4)
            for g in (True, False)]
    for env in envs:
        env.world.export_forces = True
    for _ in range(6):
        acts = envs[0].get_random_actions()
        for env in envs:
            env.step([a.clone() for a in acts])
        ga, ea = envs[0].world, envs[1].world
        for x, y in zip(ga.entities, ea.entities):
            assert torch.equal(ga.forces_dict[x], ea.forces_dict[y]), x.name
            assert torch.equal(ga.torques_dict[x], ea.torques_dict[y]), x.name
    assert envs[0].graph_status == "graph"


def test_static_rows_are_the_steps_values_host():
    """Rows of entities that neither move nor rotate: zeros, or the friction of their
    constant velocity as it was AT THE STEP (ref core.py:2053-2101) -- a later set_vel or friction
    change before the dict is read does not change them."""
    env = make("balance", dict(n_agents=4), 2, "cpu", num_envs=16, seed=0)
    w = env.world
    static = [e for e in w.entities if not (e.movable or e.rotatable)]
    assert static
    e = static[0]
    e.linear_friction = 0.3
    vel = torch.linspace(-0.5, 0.5, 32).view(16, 2)
    e.set_vel(vel, batch_index=None)
    env.step(env.get_random_actions())
    e.set_vel(torch.zeros(16, 2), batch_index=None)  # changed after the step, before the read
    e.linear_friction = 0.9
    expect = torch.zeros(16, 2)
    w.engine._static_forces(type("E", (), {"state": type("S", (), {"vel": vel, "ang_vel": None})(),
                                            "linear_friction": 0.3, "angular_friction": None, "mass": e.mass,
                                            "moment_of_inertia": e.moment_of_inertia})(),
                            expect, torch.zeros(16, 1), w)
    got = w.forces_dict[e]
    assert torch.equal(got, expect) and float(got.abs().max()) > 0
    for other in static[1:]:
        assert float(w.forces_dict[other].abs().max()) == 0.0 and float(w.torques_dict[other].abs().max()) == 0.0
