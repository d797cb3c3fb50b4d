"""World-specialised step kernels (csrc/vmas_jit.hip, hipRTC): every benchmark/parity world's
kernel is generated and compiles for gfx950 (CPU check); on the GPU it runs (kernel_name
'k_world'), matches the oracle, and is bit-identical to the generic k_step on the same state."""
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


def test_jit_falls_back_for_oversized_world():
    # 8 agents + 10 lines + 10 boxes: hundreds of box pairs, beyond one workgroup's LDS
    env = make("pollock", dict(n_agents=8, n_lines=10, n_boxes=10), None, "cpu", num_envs=8, seed=0)
    with pytest.raises(Exception, match="LDS budget"):
        env.world.engine.jit_compile_check()


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps", SPECIALISED, ids=[s[0] for s in SPECIALISED])
def test_jit_parity_and_bit_identity_gpu(gpu_device, monkeypatch, name, kw, substeps):
    env = make(name, kw, substeps, gpu_device, num_envs=300, seed=4)
    for rep in step_parity(env, n_steps=3):
        assert rep["ok"], rep
    assert env.world.engine.kernel_name == "k_world", env.world.engine.jit_error
    # same state through the generic kernel: bit-identical
    monkeypatch.setenv("VMAS_JIT", "0")
    ref = make(name, kw, substeps, gpu_device, num_envs=300, seed=4)
    snap = O.snapshot(env.world)
    O.load_snapshot(ref.world, snap)
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
    """The persistent launch (fixed-point passes on the device, cooperative or plain launch)
    is bit-identical to the host-driven pass loop and runs the same number of passes."""
    envs = {}
    for mode in ("host", "coop", "plain"):
        monkeypatch.setenv("VMAS_JIT_GRID", mode)
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
        assert eng["coop"].jit_grid > 0 and eng["plain"].jit_grid < 0
        passes = {m: e.last_iterations for m, e in eng.items()}
        assert passes["coop"] == passes["plain"] == passes["host"] >= 1, passes
        a = O.snapshot(envs["host"].world)
        for mode in ("coop", "plain"):
            b = O.snapshot(envs[mode].world)
            for i in a:
                for k in a[i]:
                    assert torch.equal(a[i][k], b[i][k]), (mode, i, k)


@pytest.mark.gpu
def test_oversized_world_runs_generic_kernel_gpu(gpu_device):
    env = make("pollock", dict(n_agents=8, n_lines=10, n_boxes=10), None, gpu_device, num_envs=128, seed=0)
    for rep in step_parity(env, n_steps=2):
        assert rep["ok"], rep
    assert env.world.engine.kernel_name == "k_step"
    assert "LDS budget" in env.world.engine.jit_error


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
