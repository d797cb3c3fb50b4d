"""World-specialised step kernels (csrc/vmas_jit.hip, hipRTC): every benchmark/parity world's
kernel is generated and compiles for gfx950 (CPU check); on the GPU it runs (kernel_name
'k_world'), matches the oracle, and is bit-identical to the generic k_step on the same state."""
import ctypes

import pytest
import torch

from oracle import vmas_oracle as O
from tests._parity import SCENARIOS, make, step_parity

SPECIALISED = SCENARIOS  # every parity world fits (waterfall: one workgroup per CU)


@pytest.mark.parametrize("name,kw,substeps", SPECIALISED, ids=[s[0] for s in SPECIALISED])
def test_jit_kernel_compiles(name, kw, substeps):
    env = make(name, kw, substeps, "cpu", num_envs=8, seed=0)
    src = env.world.engine.jit_compile_check()
    assert "k_world" in src


def test_jit_oversized_world_keeps_its_rows_in_global_memory():
    """8 agents + 10 lines + 10 boxes: hundreds of box pairs, beyond one workgroup's LDS.  The
    world-specialised kernel still compiles, with its rows in a per-workgroup slab of global
    memory (Gen::global_rows) instead of LDS (ref core.py:2103-2188 handles any entity count)."""
    env = make("pollock", dict(n_agents=8, n_lines=10, n_boxes=10), None, "cpu", num_envs=8, seed=0)
    src = env.world.engine.jit_compile_check()
    assert "float* L = a.rows + " in src and "float* rows;" in src


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps", SPECIALISED, ids=[s[0] for s in SPECIALISED])
def test_jit_parity_and_bit_identity_gpu(gpu_device, monkeypatch, name, kw, substeps):
    env = make(name, kw, substeps, gpu_device, num_envs=300, seed=4)
    for rep in step_parity(env, n_steps=3):
        assert rep["ok"], rep
    assert env.world.engine.kernel_name == "k_world", env.world.engine.jit_error
    # same state through the generic kernel: bit-identical with exact math (the default relaxed
    # math of jointless worlds is checked against the oracle above, at its tolerance)
    monkeypatch.setenv("VMAS_JIT_MATH", "exact")
    env = make(name, kw, substeps, gpu_device, num_envs=300, seed=4)
    for _ in range(2):
        env.step(env.get_random_actions())
    assert env.world.engine.kernel_name == "k_world", env.world.engine.jit_error
    monkeypatch.setenv("VMAS_JIT", "0")
    ref = make(name, kw, substeps, gpu_device, num_envs=300, seed=4)
    snap = O.snapshot(env.world)
    O.load_snapshot(ref.world, snap)
    for a, ra in zip(env.world.agents, ref.world.agents):  # (dim_c > 0: the comm update reads it)
        if a.action.c is not None:
            ra.action.c = a.action.c.clone()
    for bp in ("batch", "env"):
        O.load_snapshot(env.world, snap)
        O.load_snapshot(ref.world, snap)
        env.world.broadphase = ref.world.broadphase = bp
        env.world.step()
        ref.world.step()
        assert ref.world.engine.kernel_name == "k_step"
        a, b = O.snapshot(env.world), O.snapshot(ref.world)
        for i in a:
            for k in a[i]:
                assert torch.equal(a[i][k], b[i][k]), (bp, env.world.entities[i].name, k)


@pytest.mark.gpu
def test_jit_balance_full_size_gpu(gpu_device):
    env = make("balance", dict(n_agents=4), 10, gpu_device, num_envs=32768, seed=0)
    for rep in step_parity(env, n_steps=2):
        assert rep["ok"], rep
    assert env.world.engine.kernel_name == "k_world"


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps,num_envs", [
    ("balance", dict(n_agents=4), 10, 100_000),  # more 64-env groups than resident workgroups
    ("flocking", dict(n_agents=6), None, 3000),
    ("waterfall", dict(), None, 700),
], ids=["balance100k", "flocking", "waterfall"])
def test_device_fixed_point_matches_host_loop_gpu(gpu_device, monkeypatch, name, kw, substeps, num_envs):
    """The persistent fixed point (every pass in one launch, groups claimed per pass; also with
    a grid far below the group count, where workgroups claim several groups and steal) is
    bit-identical to the host-driven pass loop and runs the same number of passes."""
    envs = {}
    for mode, cap in (("host", None), ("persistent", None), ("persistent37", "37")):
        monkeypatch.setenv("VMAS_JIT_GRID", mode.rstrip("0123456789"))
        if cap:
            monkeypatch.setenv("VMAS_JIT_GRID_CAP", cap)
        else:
            monkeypatch.delenv("VMAS_JIT_GRID_CAP", raising=False)
        envs[mode] = make(name, kw, substeps, gpu_device, num_envs=num_envs, seed=2)
        envs[mode].world.engine._ensure()  # the mode is read when the kernel is built
    snap = O.snapshot(envs["host"].world)
    for mode, env in envs.items():
        O.load_snapshot(env.world, snap)
    for _ in range(3):
        for env in envs.values():
            env.world.step()
        eng = {m: e.world.engine for m, e in envs.items()}
        assert eng["host"].kernel_name == "k_world" and eng["host"].jit_grid == 0
        assert eng["persistent"].jit_grid < 0
        # (work items: 64-env groups, or 128 with two groups per workgroup -- VMAS_JIT_NG=2)
        item = 128 if "/ 128;" in eng["persistent37"].jit_source() else 64
        assert eng["persistent37"].jit_grid == -min(37, (num_envs + item - 1) // item)
        passes = {m: e.last_iterations for m, e in eng.items()}
        assert passes["persistent"] == passes["persistent37"] == passes["host"] >= 1, passes
        a = O.snapshot(envs["host"].world)
        for mode in ("persistent", "persistent37"):
            b = O.snapshot(envs[mode].world)
            for i in a:
                for k in a[i]:
                    assert torch.equal(a[i][k], b[i][k]), (mode, i, k)


def _violating_pollock(device):
    """A 2-env world whose all-active first pass violates the batch broadphase: a line/sphere
    pair just outside the circumscribed radius in both envs, inside the thin contact shell."""
    env = make("pollock", dict(n_agents=1, n_lines=1, n_boxes=0), None, device, num_envs=2, seed=0)
    w = env.world
    line, agent = w.landmarks[0], w.agents[0]
    d = line.shape.length / 2 + agent.shape.radius + 0.002
    agent.set_pos(torch.tensor([[d, 0.0], [d, 0.0]], device=w.device), batch_index=None)
    agent.set_vel(torch.zeros(2, 2, device=w.device), batch_index=None)
    line.set_pos(torch.zeros(2, 2, device=w.device), batch_index=None)
    line.set_rot(torch.zeros(2, 1, device=w.device), batch_index=None)
    return env


@pytest.mark.gpu
def test_fixed_point_second_pass_gpu(gpu_device):
    """The violating world needs a second pass (inside the one launch) and then equals the oracle."""
    env = _violating_pollock(gpu_device)
    rep = O.compare_one_step(env.world)
    assert env.world.engine.kernel_name == "k_world"
    assert rep["ok"], rep
    assert rep["iterations"] == 2, rep


@pytest.mark.gpu
def test_fixed_point_no_convergence_poisons_outputs_gpu(gpu_device, monkeypatch):
    """A fixed point capped at one pass cannot converge on the violating world: the step's outputs
    are NaN (visible in the step itself) and the sticky error is raised by the next check."""
    monkeypatch.setenv("VMAS_JIT_MAX_PASSES", "1")
    env = _violating_pollock(gpu_device)
    env.world.engine._ensure()
    env.world.step()
    torch.cuda.synchronize()
    agent = env.world.agents[0]
    assert torch.isnan(agent.state.pos).all() and torch.isnan(agent.state.vel).all()
    with pytest.raises(Exception, match="fixed point"):
        env.world.engine.check_device_errors()


@pytest.mark.gpu
@pytest.mark.parametrize("envs,cap,held", [(32768, None, 224), (2048, None, 250), (32768, "16", 250)],
                         ids=["32768envs-224cus", "2048envs-250cus", "grid16-250cus"])
def test_fixed_point_with_cus_held_by_another_stream_gpu(gpu_device, monkeypatch, envs, cap, held):
    """A kernel on a second stream holds most of the chip's wave slots for 0.5 s while the step
    launches: part of the step's grid cannot become resident until it ends.  Workgroups only wait
    for groups that running workgroups have claimed, so the step completes exactly (oracle parity,
    no error bit; the resident workgroups steal the groups of the absent ones).  Small grids
    (<= 32 workgroups: one workgroup per start shard) and a capped grid are included: the final
    decider must wait for the late workgroups' starts before advancing the epoch, or a late
    workgroup would run the NEXT step's pass on stale inputs -- so the step after the held one is
    checked too."""
    from vectorizedmultiagentsimulator_amd import _native as N

    if cap is not None:
        monkeypatch.setenv("VMAS_JIT_GRID_CAP", cap)
    env = make("balance", dict(n_agents=4), 10, gpu_device, num_envs=envs, seed=0)
    env.step(env.get_random_actions())
    w = env.world
    for held_step in (True, False):
        snap = O.snapshot(w)
        expected, ow = O.oracle_step(w, snap)
        band = O.sensitivity_band(w, snap, expected)
        if held_step:
            side = torch.cuda.Stream()
            torch.cuda.synchronize()
            N.check_aux(N.load_library().vmas_test_hold(0, held, 500_000, ctypes.c_void_p(side.cuda_stream)),
                        "vmas_test_hold")
        w.step()
        torch.cuda.synchronize()
        w.engine.check_device_errors()
        rep = O.compare(O.snapshot(w), expected, w, band=band, cutoff=ow.cutoff_margin)
        assert rep["ok"], (held_step, rep)
    assert w.engine.kernel_name == "k_world"


@pytest.mark.gpu
def test_oversized_world_runs_specialised_kernel_gpu(gpu_device):
    """The oversized world on k_world with global-memory rows and its persistent (sync-free) fixed
    point, at oracle parity; the generic k_step (VMAS_JIT=0) on the same world too."""
    env = make("pollock", dict(n_agents=8, n_lines=10, n_boxes=10), None, gpu_device, num_envs=128, seed=0)
    for rep in step_parity(env, n_steps=2):
        assert rep["ok"], rep
    assert env.world.engine.kernel_name == "k_world", env.world.engine.jit_error
    assert "float* L = a.rows + " in env.world.engine.jit_source()


@pytest.mark.gpu
def test_oversized_world_runs_generic_kernel_gpu(gpu_device, monkeypatch):
    monkeypatch.setenv("VMAS_JIT", "0")
    env = make("pollock", dict(n_agents=8, n_lines=10, n_boxes=10), None, gpu_device, num_envs=128, seed=0)
    for rep in step_parity(env, n_steps=2):
        assert rep["ok"], rep
    assert env.world.engine.kernel_name == "k_step"


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps", [s for s in SPECIALISED if s[0] in ("balance", "flocking")],
                         ids=["balance", "flocking"])
def test_jit_nan_state_matches_oracle_gpu(gpu_device, name, kw, substeps):
    """A NaN agent position in one env: NaN envs are never in broadphase range but get NaN
    forces from pairs that other envs keep active -- the fixed point's Z bits (an out-of-range env
    got a nonzero force) must still see them (k_world reduces a sphere pair's Z test to a NaN
    test).  The step must match the oracle's, NaN pattern included."""
    env = make(name, kw, substeps, gpu_device, num_envs=300, seed=6)
    for _ in range(2):
        env.step(env.get_random_actions())
    assert env.world.engine.kernel_name == "k_world"
    a = env.world.agents[1]
    with torch.no_grad():
        a.state.pos[5, 0] = float("nan")
        a.state.pos[17, 1] = float("nan")
    report = O.compare_one_step(env.world)
    assert report["ok"], report


def _reroll(world, gen):
    """New values for every mutable entity parameter (structure unchanged): masses (ref
    het_mass.py:50-55), drags, and the world drag."""
    for e in world.entities:
        if e.movable:
            e.mass = float(e.mass) * (0.5 + gen.random())
            e._drag = 0.1 + 0.3 * gen.random()
    world._drag = 0.2 + 0.1 * gen.random()


def test_jit_source_is_independent_of_parameter_values():
    """The generated kernel source (hence the code object) does not depend on mass / drag values:
    only on the world's structure (CPU: generated + hipRTC-compiled without a device)."""
    import random

    env = make("balance", dict(n_agents=4), 10, "cpu", num_envs=64, seed=0)
    src0 = env.world.engine.jit_compile_check()
    _reroll(env.world, random.Random(0))
    src1 = env.world.engine.jit_compile_check()
    assert src0 == src1


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_mutable_params_one_compile_gpu(gpu_device, graph):
    """het_mass (ref scenarios/debug/het_mass.py:48-54) re-rolls the agents' masses on every
    reset, and balance here re-rolls every movable entity's mass and drag (plus the world drag)
    before each step: exactly one hipRTC compile per world structure, and every step at oracle
    parity with the new values."""
    import random

    from vectorizedmultiagentsimulator_amd import _native as N
    from vectorizedmultiagentsimulator_amd import make_env

    gen = random.Random(1)
    for name, kw, resets in (("het_mass", {}, 6), ("balance", dict(n_agents=4), 6)):
        env = make_env(name, num_envs=256, device=gpu_device, seed=0, graph_step=graph, **kw)
        env.step(env.get_random_actions())
        c0, _ = N.jit_stats()
        jit0 = env.world.engine._jit.value
        for _ in range(resets):
            env.reset()
            if name == "balance":
                _reroll(env.world, gen)
            for _ in range(3):
                env.step(env.get_random_actions())
            rep = O.compare_one_step(env.world)
            assert rep["ok"], (name, rep)
        c1, cached = N.jit_stats()
        assert c1 == c0, f"{name}: {c1 - c0} recompiles for parameter changes"
        assert env.world.engine._jit.value == jit0  # the same world kernel object throughout
        assert cached <= 32
