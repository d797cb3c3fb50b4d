"""Fused scenario programs (csrc/vmas_scenarios.hip, simulator/_fused.py):
on a GPU world a benchmark scenario's per-step reward / observation / done tensor program runs as
one native launch.  Its oracle is the scenario's own torch program (the reference's, restated in
scenarios/): the same env stepped with the program forced to torch must give bit-identical
outputs, scenario attributes and world state, eagerly and replayed from a HIP graph, across
reset_at / reset."""

import math
import pytest
import torch

from vectorizedmultiagentsimulator_amd import make_env
from vectorizedmultiagentsimulator_amd.simulator import _fused
from vectorizedmultiagentsimulator_amd.simulator.environment import Environment

from test_graph import _assert_same, _flat, _rng_load, _rng_save, _state


def test_fused_programs_off_on_cpu_worlds():
    env = make_env("balance", num_envs=4, device="cpu", seed=0, n_agents=3)
    assert not _fused.enabled(env.world)


# (scenario, kwargs, substeps, scenario attributes the program leaves behind)
FUSED = [
    ("balance", dict(n_agents=4), 10, ["on_the_ground", "package_dist", "ground_rew", "pos_rew", "global_shaping"]),
    ("transport", dict(n_agents=4), None, ["rew", "package.dist_to_goal", "package.on_goal", "package.color",
                                           "package.global_shaping"]),
    ("discovery", dict(n_agents=5, use_agent_lidar=True), None,
     ["time_rew", "agents_pos", "targets_pos", "agents_targets_dists", "agents_per_target", "covered_targets",
      "shared_covering_rew", "agent.covering_reward", "agent.collision_rew", "agent.sensors.0._last_measurement",
      "agent.sensors.1._last_measurement", "target_pos"]),
    ("flocking", dict(n_agents=5), None, ["t", "agent.dist_rew", "agent.distance_shaping", "agent.collision_rew",
                                          "agent.sensors.0._last_measurement"]),
]


class _Torch:
    """Context: the scenario programs run as torch ops (the reference's program)."""

    def __enter__(self):
        self.prev = _fused._ON
        _fused._ON = False

    def __exit__(self, *exc):
        _fused._ON = self.prev


def _attrs(env, names):
    out = []
    for n in names:
        if n == "target_pos":
            out += [t.state.pos for t in env.scenario._targets]
        elif n.startswith("package."):
            out += [getattr(p, n.split(".", 1)[1]) for p in env.scenario.packages]
        elif n.startswith("agent."):  # per (policy) agent; dotted path, integer parts index lists
            for a in env.world.policy_agents:
                v = a
                for part in n.split(".")[1:]:
                    v = v[int(part)] if part.isdigit() else getattr(v, part)
                out.append(v)
        else:
            out.append(getattr(env.scenario, n))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps,attrs", FUSED, ids=[c[0] for c in FUSED])
def test_fused_program_matches_torch_program_gpu(gpu_device, monkeypatch, name, kw, substeps, attrs):
    monkeypatch.setattr(_fused, "EXACT_LIDAR", True)  # (LIDAR bit-identical to World.cast_rays)
    envs = {}
    for mode in ("torch", "fused", "graph"):
        saved = _rng_save()
        with _Torch() if mode == "torch" else _NullCtx():
            env = make_env(name, num_envs=777, device=gpu_device, seed=3, graph_step=mode == "graph", **kw)
        if substeps:
            env.world._substeps = substeps
            env.world._sub_dt = env.world._dt / substeps
        envs[mode] = env
        if mode != "graph":
            _rng_load(saved)
    ref = envs["torch"]
    for t in range(12):
        actions = ref.get_random_actions()
        outs = {}
        for mode, env in envs.items():
            s = _rng_save()
            with _Torch() if mode == "torch" else _NullCtx():
                if t == 5:
                    env.reset_at(7)
                if t == 9:
                    env.reset()
                outs[mode] = env.step([a.clone() for a in actions])
            if mode != "graph":
                _rng_load(s)
        for mode in ("fused", "graph"):
            _assert_same(outs["torch"], outs[mode], f"{name} {mode} outputs step {t}")
            _assert_same(_state(ref), _state(envs[mode]), f"{name} {mode} state step {t}")
            _assert_same(_attrs(ref, attrs), _attrs(envs[mode], attrs), f"{name} {mode} attributes step {t}")
    assert envs["graph"].graph_status == "graph", envs["graph"].graph_reason


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


@pytest.mark.gpu
def test_fused_balance_cache_follows_state_changes_gpu(gpu_device):
    """A call whose inputs changed since the launch recomputes (the reference recomputes on every
    call): an observation after an in-place position edit, and a second reward call."""
    env = make_env("balance", num_envs=64, device=gpu_device, seed=0, n_agents=3)
    env.step(env.get_random_actions())
    sc, w = env.scenario, env.world
    r0 = sc.reward(w.agents[0])
    with torch.no_grad():
        w.agents[1].state.pos[3, 0] += 0.25
    obs1 = sc.observation(w.agents[1])
    with _Torch():
        expect = sc.observation(w.agents[1])
    assert torch.equal(obs1, expect)
    r0b = sc.reward(w.agents[2])
    assert torch.equal(r0, r0b) and r0.data_ptr() != r0b.data_ptr()
    assert torch.equal(sc.done(), sc.on_the_ground + w.is_overlapping(sc.package, sc.package.goal))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [3, 4, 7, 8, 12])
def test_reduce_order_probe_finds_torch_mean_order_gpu(gpu_device, n):
    """The fused kernels' mean over n contiguous values reproduces torch's .mean(-1) on the device
    bit for bit in one of the ordered_sum modes (else the scenario would keep its torch program)."""
    assert _fused.reduce_order(torch.device(gpu_device), n) is not None


# (scenario, kwargs, observation columns that are LIDAR rays, per policy agent)
FAST_LIDAR = [
    ("flocking", dict(n_agents=5), lambda env, a: slice(6, None)),
    ("discovery", dict(n_agents=5), lambda env, a: slice(4, None)),
    ("discovery", dict(n_agents=8, n_targets=7, use_agent_lidar=True), lambda env, a: slice(4, None)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,lidar_cols", FAST_LIDAR, ids=[f"{c[0]}{i}" for i, c in enumerate(FAST_LIDAR)])
def test_fast_lidar_program_gpu(gpu_device, name, kw, lidar_cols):
    """The default fused programs (fast LIDAR): every output but the LIDAR rays is bit-identical to
    the scenario's torch program; the rays match the CPU oracle's World.cast_rays on the same state
    within the LIDAR tolerance, a ray outside it only at a hit / miss boundary (certified,
    tests/_parity.py lidar_parity)."""
    from tests._parity import lidar_parity

    envs = {}
    for mode in ("torch", "fused"):
        saved = _rng_save()
        with _Torch() if mode == "torch" else _NullCtx():
            envs[mode] = make_env(name, num_envs=4096, device=gpu_device, seed=3, **kw)
        if mode == "torch":
            _rng_load(saved)
    ref, fus = envs["torch"], envs["fused"]
    worst = 0.0
    for t in range(8):
        actions = ref.get_random_actions()
        outs = {}
        for mode, env in envs.items():
            s = _rng_save()
            with _Torch() if mode == "torch" else _NullCtx():
                outs[mode] = env.step([a.clone() for a in actions])
            if mode == "torch":
                _rng_load(s)
        obs_t, obs_f = outs["torch"][0], outs["fused"][0]
        for a, ot, of in zip(fus.world.policy_agents, obs_t, obs_f):
            keep = torch.ones(ot.shape[-1], dtype=torch.bool)
            keep[lidar_cols(fus, a)] = False
            assert torch.equal(ot[:, keep], of[:, keep]), (t, a.name)
        _assert_same(outs["torch"][1:], outs["fused"][1:], f"{name} rewards / dones / infos step {t}")
        _assert_same(_state(ref), _state(fus), f"{name} state step {t}")
        rep = lidar_parity(fus, measured=True)
        assert rep["ok"], (t, rep)
        worst = max(worst, rep["bad_rows"] / max(rep["rows"], 1))
    assert worst < 1e-3  # boundary rays are rare


@pytest.mark.gpu
def test_fast_lidar_rotated_agents_gpu(gpu_device):
    """Agents turned by up to +-300 rad: the fast LIDAR's hardware sin / cos take the
    angle in revolutions and lose |angle| * 2^-24 rad, so angles beyond 16 rad go through the
    range-reduced sincosf; the measured rays stay within the oracle's LIDAR tolerance."""
    from tests._parity import lidar_parity

    env = make_env("flocking", num_envs=4096, device=gpu_device, seed=7, n_agents=5)
    g = torch.Generator(device="cpu").manual_seed(0)
    for a in env.world.agents:
        rot = (torch.rand(4096, 1, generator=g) * 600.0 - 300.0).to(gpu_device)
        a.set_rot(rot, batch_index=None)
    for _ in range(2):
        env.step(env.get_random_actions())
        rep = lidar_parity(env, measured=True)
        assert rep["ok"], rep
        assert rep["bad_rows"] <= 4, rep


@pytest.mark.gpu
@pytest.mark.parametrize("max_turns", [60, 16_000, 160_000], ids=["4e2rad", "1e5rad", "1e6rad"])
def test_relaxed_trig_large_rotation_gpu(gpu_device, max_turns):
    """Relaxed math (the GPU default of jointless worlds) with rotatable boxes and lines turned by
    up to 4e2 / 1e5 / 1e6 radians (the reference never wraps rot, core.py:2907): one teacher-forced
    step against the oracle (the entity trig's branch-free 2 pi reduction, vmas_physics.hpp red2pi:
    accurate to ~2e-7 well past these magnitudes)."""
    from oracle import vmas_oracle as O
    from tests._parity import make

    env = make("features", dict(n_agents=4), None, gpu_device, num_envs=2048, seed=2)
    env.step(env.get_random_actions())
    g = torch.Generator(device="cpu").manual_seed(1)
    for e in env.world.entities:
        if e.rotatable:
            turns = torch.randint(-max_turns, max_turns + 1, (2048, 1), generator=g).float() * (2 * math.pi)
            e.set_rot(e.state.rot + turns.to(gpu_device), batch_index=None)
    rep = O.compare_one_step(env.world)
    assert "VMAS_PHYS_RELAXED" in env.world.engine.jit_source()
    assert rep["ok"], rep


@pytest.mark.gpu
def test_exact_math_gpu(gpu_device):
    """The scenario programs' flag-independent division and square root (csrc/vmas_programs.hpp
    xdiv / xsqrt, compiled into the relaxed world modules) equal IEEE `/` and sqrtf bit for bit:
    random bit patterns (normals, denormals, infinities, NaNs) plus edge values."""
    import ctypes

    from vectorizedmultiagentsimulator_amd import _native as N

    g = torch.Generator(device="cpu").manual_seed(11)
    n = 1 << 22
    bits = torch.randint(-(1 << 31), (1 << 31) - 1, (2, n), generator=g, dtype=torch.int64).to(torch.int32)
    ab = bits.view(torch.float32).clone()
    edge = torch.tensor([0.0, -0.0, 1.0, -1.0, float("inf"), -float("inf"), float("nan"), 1e-45, -1e-45, 1e-38,
                         3.4e38, float.fromhex("0x1.0p-96"), float.fromhex("0x1.0p-97"), 2.0, 0.5, 1e-30], dtype=torch.float32)
    k = edge.numel()
    ab[0, :k * k] = edge.repeat_interleave(k)
    ab[1, :k * k] = edge.repeat(k)
    ab[1, k * k:2 * k * k] = 3.0  # (ordinary denominators too)
    ab[0, 2 * k * k:] = ab[0, 2 * k * k:].abs()  # half the square roots of non-negative values
    a, b = ab[0].to(gpu_device), ab[1].to(gpu_device)
    out = torch.empty(4 * n, device=gpu_device, dtype=torch.float32)
    idx = torch.device(gpu_device).index or 0
    N.check(N.load_library().vmas_test_exact_math(idx, a.data_ptr(), b.data_ptr(), out.data_ptr(), n,
                                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
            "vmas_test_exact_math")
    o = out.view(4, n).cpu()
    for x, ref, what in ((o[0], o[1], "div"), (o[2], o[3], "sqrt")):
        same = (x.view(torch.int32) == ref.view(torch.int32)) | (torch.isnan(x) & torch.isnan(ref))
        bad = (~same).nonzero().flatten()
        assert bad.numel() == 0, (what, bad[:5].tolist(), x[bad[:5]].tolist(), ref[bad[:5]].tolist())
