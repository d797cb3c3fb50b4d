"""Graph mode (make_env(..., graph_step=True), simulator/environment/_graph.py): a step replayed
from one HIP graph returns the same observations / rewards / dones / infos and leaves the same
world state as the eager step, bit for bit, including across reset_at / reset between steps;
scenarios whose step cannot be captured (host syncs) stay eager with the same results."""

import pytest
import torch

from vectorizedmultiagentsimulator_amd import make_env
from vectorizedmultiagentsimulator_amd.simulator.environment import Environment


def test_graph_step_needs_gpu_device():
    with pytest.raises(ValueError, match="ROCm"):
        make_env("balance", num_envs=4, device="cpu", seed=0, graph_step=True)


def _flat(tree, acc):
    if isinstance(tree, torch.Tensor):
        acc.append(tree)
    elif isinstance(tree, (list, tuple)):
        for x in tree:
            _flat(x, acc)
    elif isinstance(tree, dict):
        for k in sorted(tree):
            _flat(tree[k], acc)
    return acc


def _state(env):
    out = []
    for e in env.world.entities:
        s = e.state
        out += [s.pos, s.vel, s.rot, s.ang_vel]
    return out


def _write_only_attrs(env):
    """The attributes the package's classes declare write-only within a step (not carried between
    replays: environment/_graph.py _write_only), as bound now."""
    objs = [env.scenario] + [s for a in env.agents for s in (a.sensors or ())]
    out = []
    for o in objs:
        for k in sorted(type(o).__dict__.get("_vmas_graph_write_only", ())):
            v = o.__dict__.get(k)
            if isinstance(v, torch.Tensor):
                out.append(v)
    return out


def _rng_save():
    return ([x.clone() if isinstance(x, torch.Tensor) else x for x in Environment.vmas_random_state],
            torch.cuda.get_rng_state())


def _rng_load(saved):
    Environment.vmas_random_state[:] = [x.clone() if isinstance(x, torch.Tensor) else x for x in saved[0]]
    torch.cuda.set_rng_state(saved[1])


def _assert_same(a, b, what):
    fa, fb = _flat(a, []), _flat(b, [])
    assert len(fa) == len(fb), what
    for i, (x, y) in enumerate(zip(fa, fb)):
        assert x.shape == y.shape and x.dtype == y.dtype, (what, i)
        assert torch.equal(x, y), (what, i, (x.float() - y.float()).abs().max().item())


CASES = [
    ("balance", dict(n_agents=4), 10, "graph"),
    ("transport", dict(n_agents=4), None, "graph"),
    ("flocking", dict(n_agents=4), None, "graph"),     # scripted agent: range assert on the device
    ("discovery", dict(n_agents=4), None, "graph"),    # spawn sampler: inside the graph (spawn channel)
    ("discovery-hole", dict(n_agents=4), None, "graph"),  # the segmented form: a host hole, two graphs
    # every respawn handed over to the reference loop (VMAS_SPAWN_TEST_MAX_TRIES=1): undone from the
    # launch's backup and redone after the replay, the step's observations recomputed
    ("discovery-redo", dict(n_agents=4), None, "graph"),
    # the package's debug worlds, which the default graph step (graph_step=None) also replays
    # (ADVICE r5): joints in exact math, a world needing several fixed-point passes, masses re-drawn
    # by every reset (a parameter change between replays: recaptured), every physics feature
    ("waterfall", {}, None, "graph"),
    # (45 entities: the step's fixed point is host-driven here, a host wait per pass -- the watched
    # step sees it, so the env stays eager; every step still equal to the eager env's)
    ("pollock", {}, None, "eager"),
    ("het_mass", {}, None, "graph"),  # (recaptured after each reset: the masses change)
    ("features", {}, None, "eager"),  # (communication actions: the per-agent action path)
]
MIN_REPLAYS = {"het_mass": 2}  # (replays since its last recapture, after the reset of step 10)


# fused scenarios whose outputs the replays write directly: categories (obs, rewards, done)
DIRECT = {"balance": 3, "transport": 3, "flocking": 2, "discovery": 3}


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps,expect", CASES, ids=[c[0] for c in CASES])
def test_graph_replay_matches_eager_gpu(gpu_device, monkeypatch, name, kw, substeps, expect):
    hole = False
    if name == "discovery-hole":
        monkeypatch.setenv("VMAS_GRAPH_DEFERRED_SPAWN", "0")
        name = "discovery"
        hole = True
    elif name == "discovery-redo":
        monkeypatch.setenv("VMAS_SPAWN_TEST_MAX_TRIES", "1")
        name = "discovery"
    envs = []
    for graph in (False, True):
        saved = _rng_save()
        env = make_env(name, num_envs=512, device=gpu_device, seed=1, graph_step=graph, **kw)
        if substeps:
            env.world._substeps = substeps
            env.world._sub_dt = env.world._dt / substeps
        envs.append(env)
        if not graph:
            _rng_load(saved)
    eager, graph = envs
    held = None
    for t in range(14):
        actions = eager.get_random_actions()
        if t == 7:  # in-place edit between steps (reset_at -> set_pos(batch_index))
            s = _rng_save()
            eager.reset_at(3)
            _rng_load(s)
            graph.reset_at(3)
        if t == 10:  # full reset re-binds every state tensor
            s = _rng_save()
            eager.reset()
            _rng_load(s)
            graph.reset()
        s = _rng_save()  # the step itself may draw (discovery respawns its targets)
        out_e = eager.step([a.clone() for a in actions])
        _rng_load(s)
        out_g = graph.step([a.clone() for a in actions])
        _assert_same(out_e, out_g, f"{name} outputs step {t}")
        _assert_same(_state(eager), _state(graph), f"{name} state step {t}")
        # (re-bound each step, not carried between replays: the step's values all the same)
        _assert_same(_write_only_attrs(eager), _write_only_attrs(graph), f"{name} write-only attributes step {t}")
        assert torch.equal(eager.steps, graph.steps), (name, t)  # (folded into the post-replay launch)
        if t == 4:
            held = [(x.clone(), x) for x in _flat(out_g, [])]
    # returned tensors are fresh: a later replay does not overwrite them (copies, or -- the fused
    # scenarios' obs / rewards / done -- tensors the replay wrote directly, DirectOutputs)
    assert all(torch.equal(v, x) for v, x in held)
    assert graph.graph_status == expect, graph.graph_reason
    if name == "pollock":
        assert "host wait" in graph.graph_reason, graph.graph_reason
    if name == "features":
        assert "communication actions" in graph.graph_reason, graph.graph_reason
    if name in DIRECT and not hole:  # (every category of the fused launch written directly)
        assert len(graph._graph._direct.enabled) == DIRECT[name], [r["dtype"] for r in graph._graph._direct.enabled]
    if expect == "graph":
        assert graph._graph.replays >= MIN_REPLAYS.get(name, 5)
        if name in DIRECT:  # (each declares write-only attributes: none of them carried)
            wo = {id(t) for t in graph._graph._write_only_ys}
            assert wo and not wo & {id(y) for y in graph._graph._carry_ys}
        assert graph._graph._steps_folded  # no max_steps: steps += 1 left the graph
    if name == "discovery":  # the targets' respawn is one native call: inside the one graph with
        # its host side after the replay (a spawn channel), or one host hole between two graphs
        n_holes, n_segments = len(graph._graph._holes), len(graph._graph._segments)
        assert (n_holes, n_segments, len(graph._graph._deferred)) == ((1, 2, 0) if hole else (0, 1, 1))


def _twin_envs(gpu_device, name, **kw):
    envs = []
    for graph in (False, True):
        saved = _rng_save()
        envs.append(make_env(name, num_envs=256, device=gpu_device, seed=0, graph_step=graph, **kw))
        if not graph:
            _rng_load(saved)
    return envs


def _step_both(eager, graph, actions, expect_raise=None):
    outs = []
    for env in (eager, graph):
        s = _rng_save()
        if expect_raise is not None:
            with pytest.raises(AssertionError, match=expect_raise):
                env.step([a.clone() for a in actions])
            outs.append(None)
        else:
            outs.append(env.step([a.clone() for a in actions]))
        if env is eager:
            _rng_load(s)
    return outs


@pytest.mark.gpu
def test_scripted_action_assert_raised_from_step_gpu(gpu_device):
    """A scripted agent's out-of-range action (core.py:977-980) raises from the step() that
    computed it, eagerly and from a replayed graph (where the check runs on the device); the
    replayed step is rolled back, so both worlds continue identically."""
    eager, graph = _twin_envs(gpu_device, "flocking", n_agents=3)
    scale = torch.ones(1, device=gpu_device)
    for env in (eager, graph):
        sc = env.scenario

        def script(agent, world, sc=sc):
            t = sc.t / 30
            agent.action.u = torch.stack([torch.cos(t), torch.sin(t)], dim=1) * scale

        sc._target._action_script = script
    for _ in range(5):
        _step_both(eager, graph, eager.get_random_actions())
    assert graph.graph_status == "graph", graph.graph_reason
    scale.fill_(2.0)  # read by the captured step: |u| = 2|cos t| > u_range 1 in most envs
    _step_both(eager, graph, eager.get_random_actions(), "Scripted physical action of target is out of range")
    _assert_same(_state(eager), _state(graph), "state after the failed step")
    assert torch.equal(eager.scenario.t, graph.scenario.t)
    scale.fill_(1.0)
    for t in range(3):  # the channel keeps working and the worlds stay identical
        out_e, out_g = _step_both(eager, graph, eager.get_random_actions())
        _assert_same(out_e, out_g, f"outputs after the failed step {t}")
        _assert_same(_state(eager), _state(graph), f"state after the failed step {t}")


@pytest.mark.gpu
@pytest.mark.parametrize("deferred", [False, True], ids=["hole", "channel"])
def test_failed_segmented_capture_restores_state_gpu(gpu_device, monkeypatch, deferred):
    """A capture that fails after host holes already ran the graphs before them (discovery's
    spawn sampler) restores the world and the generator, and the env continues eagerly with the
    eager twin's results."""
    monkeypatch.setenv("VMAS_GRAPH_DEFERRED_SPAWN", "1" if deferred else "0")
    eager, graph = _twin_envs(gpu_device, "discovery", n_agents=4)
    orig = graph.scenario.info

    def info(agent):
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("injected capture failure")
        return orig(agent)

    graph.scenario.info = info
    for t in range(6):
        out_e, out_g = _step_both(eager, graph, eager.get_random_actions())
        _assert_same(out_e, out_g, f"outputs step {t}")
        _assert_same(_state(eager), _state(graph), f"state step {t}")
    assert graph.graph_status == "eager" and "injected" in graph.graph_reason


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["balance", "discovery"])
@pytest.mark.parametrize("bad", ["nan", "range"])
@pytest.mark.parametrize("speculative", [False, True], ids=["wait", "speculative"])
def test_failed_action_check_leaves_world_as_eager_gpu(gpu_device, monkeypatch, bad, speculative, name):
    """A NaN / out-of-range action raises the reference's AssertionError and leaves the world as
    the eager step leaves it -- also when the replay was launched before the action flags were
    known (speculative, rolled back, where the agents' u are exact too: the agents before the
    failing one hold their new u, the rest their old one)."""
    monkeypatch.setattr(Environment, "_SPECULATE", speculative)
    eager, graph = _twin_envs(gpu_device, name, n_agents=4)
    for _ in range(5):
        _step_both(eager, graph, eager.get_random_actions())
    assert graph.graph_status == "graph", graph.graph_reason
    before_u = [a.action.u.clone() for a in graph.agents]
    actions = eager.get_random_actions()
    actions[2][5, 1] = float("nan") if bad == "nan" else 3.0
    _step_both(eager, graph, actions, "^$" if bad == "nan" else "out of its range")
    _assert_same(_state(eager), _state(graph), "state after the failed step")
    # (a rolled-back replay restores the write-only attributes from its backups)
    _assert_same(_write_only_attrs(eager), _write_only_attrs(graph), "write-only attributes after the failed step")
    for i, (ae, ag) in enumerate(zip(eager.agents, graph.agents)):
        if i < 2 or speculative:  # (documented: without speculation the failing agent and those
            # after it hold the rejected actions in their persistent u, until the next step)
            assert torch.equal(ae.action.u, ag.action.u), i
        if i >= 2 and speculative:
            assert torch.equal(ag.action.u, before_u[i]), i
    assert torch.equal(eager.steps, graph.steps)
    for t in range(4):
        out_e, out_g = _step_both(eager, graph, eager.get_random_actions())
        _assert_same(out_e, out_g, f"outputs after the failed step {t}")
        _assert_same(_state(eager), _state(graph), f"state after the failed step {t}")
    assert graph.graph_status == "graph"
    assert graph._can_speculate() == speculative


@pytest.mark.gpu
def test_replay_leaves_host_rng_states_as_the_swap_does_gpu(gpu_device):
    """A replayed step skips local_seed's host RNG swap (it runs no host RNG code): the user's
    torch / numpy / python streams and the simulator's saved states are what the swap leaves."""
    import random

    import numpy as np

    env = make_env("balance", num_envs=256, device=gpu_device, seed=0, graph_step=True, n_agents=4)
    for _ in range(4):
        env.step(env.get_random_actions())
    assert env.graph_status == "graph"
    sim_before = [torch.random.get_rng_state(), np.random.get_state(), random.getstate()]
    sim_before = list(Environment.vmas_random_state)
    torch.manual_seed(3)
    np.random.seed(3)
    random.seed(3)
    want = (torch.rand(3), np.random.rand(3), random.random())
    torch.manual_seed(3)
    np.random.seed(3)
    random.seed(3)
    env.step(env.get_random_actions())
    got = (torch.rand(3), np.random.rand(3), random.random())
    assert torch.equal(want[0], got[0]) and np.array_equal(want[1], got[1]) and want[2] == got[2]
    assert torch.equal(Environment.vmas_random_state[0], sim_before[0])
    # an exception inside a replayed step leaves the simulator's states swapped in (reference)
    bad = env.get_random_actions()
    bad[0][0, 0] = float("nan")
    torch.manual_seed(99)
    with pytest.raises(AssertionError):
        env.step(bad)
    assert torch.equal(torch.random.get_rng_state(), Environment.vmas_random_state[0])


@pytest.mark.gpu
def test_graph_parameter_change_recaptures_gpu(gpu_device):
    env = make_env("balance", num_envs=256, device=gpu_device, seed=0, graph_step=True, n_agents=4)
    for _ in range(4):
        env.step(env.get_random_actions())
    assert env.graph_status == "graph"
    env.world.agents[0].mass = 2.0  # static-table change: the graph is dropped, then re-captured
    env.step(env.get_random_actions())
    assert env.graph_status == "dropped"
    for _ in range(4):
        env.step(env.get_random_actions())
    assert env.graph_status == "graph"


@pytest.mark.gpu
def test_graph_kernel_timing_gpu(gpu_device):
    """The in-kernel device timer counts replayed launches (HIP records no events inside a
    graph) and agrees with HIP events on eager launches."""
    env = make_env("balance", num_envs=32768, device=gpu_device, seed=0, graph_step=True, n_agents=4)
    eng = env.world.engine
    env.step(env.get_random_actions())  # builds the engine
    eng.set_timing(True)  # before the capture: the timer pointer is a captured kernel argument
    for _ in range(4):
        env.step(env.get_random_actions())
    assert env.graph_status == "graph"
    eng.get_timing(reset=True)
    eng.device_timing(reset=True)
    for _ in range(5):
        env.step(env.get_random_actions())
    ms, n = eng.device_timing(reset=True)
    assert n == 5 and ms > 0
    eager = make_env("balance", num_envs=32768, device=gpu_device, seed=0, n_agents=4, graph_step=False)
    eager.step(eager.get_random_actions())
    e2 = eager.world.engine
    e2.set_timing(True)
    for _ in range(3):
        eager.step(eager.get_random_actions())
    e2.get_timing(reset=True)
    e2.device_timing(reset=True)
    for _ in range(5):
        eager.step(eager.get_random_actions())
    ev_ms, ev_n = e2.get_timing(reset=True)
    dt_ms, dt_n = e2.device_timing(reset=True)
    assert ev_n == dt_n == 5
    # the in-kernel window misses the launch ramp and the exit tail: up to ~7 us of a ~15 us
    # one-substep launch
    assert 0.5 * ev_ms < dt_ms <= 1.05 * ev_ms, (ev_ms, dt_ms)


def test_trial_step_detects_host_waits():
    """The native host-wait counter moves on a synchronising call (CPU: the host backend does
    not wait, the counter is still exported and readable)."""
    from vectorizedmultiagentsimulator_amd import _native as N

    lib = N.load_library()
    assert isinstance(lib.vmas_host_waits(), int)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["python_counter", "numpy_rng", "torch_cpu_rng"])
def test_graph_refuses_host_side_step_state_gpu(gpu_device, kind):
    """A step that keeps Python-side state (a Python-int counter) or draws from a host RNG would
    be frozen by a replay: graph mode must detect it in the trial step and stay eager."""
    import numpy as np

    env = make_env("balance", num_envs=64, device=gpu_device, seed=0, graph_step=True, n_agents=2)
    sc = env.scenario
    orig = sc.post_step
    sc.count = 0

    def post_step():
        orig()
        if kind == "python_counter":
            sc.count += 1
        elif kind == "numpy_rng":
            np.random.rand()
        else:
            torch.rand(1)

    sc.post_step = post_step
    for _ in range(5):
        env.step(env.get_random_actions())
    assert env.graph_status == "eager", env.graph_reason
    expect = "Python-side state" if kind == "python_counter" else "host RNG"
    assert expect in env.graph_reason, env.graph_reason


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps", [("balance", dict(n_agents=4), 10), ("flocking", dict(n_agents=4), None),
                                               ("discovery", dict(n_agents=4), None),
                                               ("discovery-redo", dict(n_agents=4), None),
                                               ("balance-2pass", dict(n_agents=4), 10),
                                               ("transport-2pass", dict(n_agents=4), None),
                                               ("balance-carry", dict(n_agents=4), 10),
                                               ("balance-notail", dict(n_agents=4), 10)],
                         ids=["balance", "flocking", "discovery", "discovery-redo", "balance-2pass", "transport-2pass",
                              "balance-carry", "balance-notail"])
def test_preapplied_random_actions_match_eager_gpu(gpu_device, monkeypatch, name, kw, substeps):
    """env.step(env.get_random_actions()) in graph mode: the draw kernel also writes the applied
    actions into the graph's action buffer, and the step launches no action kernel.  Bit-identical
    to the eager step on the same draws; an in-place edit of the drawn tensors, or other tensors,
    take the normal action path.  Discovery: the next draw is made ahead at the generator offset
    the in-graph respawn leaves on the device; "discovery-redo" hands every respawn over to the
    reference loop (VMAS_SPAWN_TEST_MAX_TRIES=1), so every such draw is dropped and made anew.
    A pre-applied replay of a kernel chain writes the step's state back into its inputs (no carry,
    StepGraph._writeback_ready); "-2pass" forces a second fixed-point pass on every step
    (VMAS_JIT_TEST_PASSES=2), whose re-run reads the pre-step state from the first pass's backup."""
    redo = name == "discovery-redo"
    if redo:
        monkeypatch.setenv("VMAS_SPAWN_TEST_MAX_TRIES", "1")
        name = "discovery"
    from vectorizedmultiagentsimulator_amd import _native as N
    from vectorizedmultiagentsimulator_amd.simulator.environment._graph import StepGraph
    carry = name.endswith("-carry")
    if carry:  # (a carried state above the write-back's size limit: the post-replay carry instead)
        monkeypatch.setattr(StepGraph, "_WRITEBACK_MAX_BYTES", 0)
        name = name[:-len("-carry")]
    notail = name.endswith("-notail")
    if notail:  # (the post-replay launch of its own, VMAS_GRAPH_TAIL=0)
        monkeypatch.setattr(StepGraph, "_TAIL", False)
        name = name[:-len("-notail")]
    tails0 = N.load_host().tail_launches()
    two_pass = name.endswith("-2pass")
    if two_pass:
        monkeypatch.setenv("VMAS_JIT_TEST_PASSES", "2")
        name = name[:-len("-2pass")]
    eager, graph = _twin_envs(gpu_device, name, **kw)
    for env in (eager, graph):
        if substeps:
            env.world._substeps = substeps
            env.world._sub_dt = env.world._dt / substeps
    for t in range(12):
        s = _rng_save()
        if t == 5:  # a device draw between the step and get_random_actions: the draw made ahead by
            torch.rand(7, device=gpu_device)  # the post-replay launch is not handed out
        a_e = eager.get_random_actions()
        _rng_load(s)
        if t == 5:
            torch.rand(7, device=gpu_device)
        a_g = graph.get_random_actions()
        _assert_same(a_e, a_g, f"draws step {t}")
        # the draw leaves the agents alone: between the draw and the step, action.u
        # and state.force still hold the last step's values (graph mode: the draw's snapshot)
        if t > 0:
            _assert_same([a.action.u for a in eager.agents], [a.action.u for a in graph.agents], f"u after draw {t}")
            _assert_same([a.state.force for a in eager.agents], [a.state.force for a in graph.agents],
                         f"force after draw {t}")
        if t == 8:  # an in-place edit of a drawn tensor: the step applies the edited values
            for a in (a_e, a_g):
                a[0][:5] = 0.25
        if t == 9:  # other tensors than the draw's
            a_g = [a.clone() for a in a_g]
        s = _rng_save()
        out_e = eager.step(a_e)
        _rng_load(s)
        out_g = graph.step(a_g)
        _assert_same(out_e, out_g, f"{name} outputs step {t}")
        _assert_same(_state(eager), _state(graph), f"{name} state step {t}")
        _assert_same([a.action.u for a in eager.agents], [a.action.u for a in graph.agents], f"u step {t}")
        assert torch.equal(eager.steps, graph.steps), (name, t)
    assert graph.graph_status == "graph", graph.graph_reason
    assert graph.preapplied_steps >= (0 if redo else 5)  # (a redone respawn edits state between steps)
    if name in ("balance", "discovery", "flocking") and not redo:  # (no device asserts: draws made ahead, handed out)
        assert graph._SPEC_DRAW and getattr(graph, "drawn_ahead", 0) >= 3
    if redo:
        assert getattr(graph, "drawn_ahead", 0) == 0
    if carry:
        assert graph._graph._wb is False
    elif name in ("balance", "flocking", "transport"):  # (kernel-chain replays: the state written back by k_world)
        wb = graph._graph._wb
        assert isinstance(wb, dict) and wb["chain"] is graph._graph._chain, (wb, graph._graph.chain_why)
        x = graph._graph._carry_dst[graph._graph._state_idx]
        tbl = graph._graph._post_cache_wb[4]["tbl"]
        assert x.data_ptr() not in {int(r["dst"]) for r in tbl}  # (no carry span into the state buffer)
    if two_pass:
        assert "VMAS_GRID_MIN_PASSES 2" in graph.world.engine.jit_source()
        assert graph.world.engine.last_iterations == 2
    # balance's post-replay work ran as the tail of its one fused launch (csrc/vmas_tail.hpp): the
    # draws made ahead, the carry (the state too, without the write-back) and the info copies
    tails = N.load_host().tail_launches() - tails0
    if name in ("balance", "transport") and not notail:
        assert tails >= 3, tails  # (as drawn_ahead: the steps after the warm-up and the capture)
    elif name == "balance":
        assert tails == 0


@pytest.mark.gpu
@pytest.mark.parametrize("other", ["clone", "policy"])
def test_draw_ahead_dropped_by_caller_actions_gpu(gpu_device, other):
    """random -> step -> step(caller's own actions) -> random -> step.  The
    post-replay launch of the second step drew the next actions ahead into the persistent action
    buffer; the caller's step rewrote that buffer, so the following get_random_actions must not
    hand out the draw made ahead as pre-applied (its applied values are gone).  Bit-identical to
    the eager twin at every step."""
    eager, graph = _twin_envs(gpu_device, "balance", n_agents=4)
    for t in range(10):
        s = _rng_save()
        if t % 3 == 2:  # the caller's own actions: a heuristic-like policy with no device draw
            if other == "clone":
                acts = [(a.action.u.clone() / a.action.u_multiplier_tensor).clamp_(-1, 1) for a in eager.agents]
            else:
                acts = [torch.full((256, 2), 0.1 * (i + 1), device=gpu_device).clamp_(-1, 1)
                        for i in range(len(eager.agents))]
            a_e, a_g = acts, [a.clone() for a in acts]
        else:
            a_e = eager.get_random_actions()
            _rng_load(s)
            a_g = graph.get_random_actions()
            _assert_same(a_e, a_g, f"draws step {t}")
        s = _rng_save()
        out_e = eager.step(a_e)
        _rng_load(s)
        out_g = graph.step(a_g)
        _assert_same(out_e, out_g, f"{other} outputs step {t}")
        _assert_same(_state(eager), _state(graph), f"{other} state step {t}")
        _assert_same([a.action.u for a in eager.agents], [a.action.u for a in graph.agents], f"u step {t}")
    assert graph.graph_status == "graph", graph.graph_reason
    assert graph.preapplied_steps > 0


@pytest.mark.gpu
def test_max_steps_keeps_the_counter_in_the_graph_gpu(gpu_device):
    """With max_steps the done program reads the step counter (ref environment.py:415-418), so the
    capture keeps `steps += 1` inside the graph; dones (terminated + truncated) match the eager
    step across the truncation and a reset_at, and setting max_steps on a folded graph drops it."""
    envs = []
    for graph in (False, True):
        saved = _rng_save()
        envs.append(make_env("balance", num_envs=256, device=gpu_device, seed=0, graph_step=graph, n_agents=3,
                             max_steps=6))
        if not graph:
            _rng_load(saved)
    eager, graph = envs
    for t in range(10):
        actions = eager.get_random_actions()
        if t == 7:
            for env in (eager, graph):
                s = _rng_save()
                env.reset_at(5)
                if env is eager:
                    _rng_load(s)
        out_e, out_g = _step_both(eager, graph, actions)
        _assert_same(out_e, out_g, f"max_steps outputs step {t}")
        assert torch.equal(eager.steps, graph.steps), t
    assert graph.graph_status == "graph", graph.graph_reason
    assert not graph._graph._steps_folded
    # a folded capture, then max_steps set: the graph is dropped and the next steps stay exact
    eager, graph = _twin_envs(gpu_device, "balance", n_agents=3)
    for t in range(8):
        if t == 5:
            eager.max_steps = graph.max_steps = 6
        actions = eager.get_random_actions()
        out_e, out_g = _step_both(eager, graph, actions)
        _assert_same(out_e, out_g, f"max_steps set later, step {t}")
        assert torch.equal(eager.steps, graph.steps), t


@pytest.mark.gpu
@pytest.mark.parametrize("fresh", ["1", "0"])
def test_state_alias_keeps_its_step_values_gpu(gpu_device, monkeypatch, fresh):
    """The reference's integration creates new state tensors every step (core.py:2866-2907) and its
    _set_action a new action.u: a reference kept to entity.state.pos / vel / agent.action.u /
    state.force from one step keeps that step's values after later steps.  Graph mode re-binds
    them to fresh tensors on first use after each replay (_FreshState); VMAS_GRAPH_FRESH_STATES=0
    is the measured opt-out, where such an alias follows the graph's buffers."""
    monkeypatch.setattr("vectorizedmultiagentsimulator_amd.simulator.environment._graph.StepGraph._FRESH_STATES",
                        fresh == "1")
    eager, graph = _twin_envs(gpu_device, "balance", n_agents=4)
    for _ in range(4):
        _step_both(eager, graph, eager.get_random_actions())
    assert graph.graph_status == "graph", graph.graph_reason
    held = {}
    for name, env in (("eager", eager), ("graph", graph)):
        ag, pkg = env.world.agents[0], env.scenario.package
        refs = [ag.state.pos, ag.state.vel, pkg.state.pos, env.scenario.line.state.rot, ag.action.u, ag.state.force]
        held[name] = (refs, [r.clone() for r in refs])
    for _ in range(3):
        _step_both(eager, graph, eager.get_random_actions())
    refs_e, vals_e = held["eager"]
    assert all(torch.equal(r, v) for r, v in zip(refs_e, vals_e))  # (the reference's semantics)
    refs_g, vals_g = held["graph"]
    kept = [torch.equal(r, v) for r, v in zip(refs_g, vals_g)]
    if fresh == "1":
        assert all(kept), kept
    else:
        assert not all(kept)  # (the opt-out: the aliases see the later steps)
    _assert_same(_state(eager), _state(graph), "state after the aliased steps")
    # an in-place write through a fresh state tensor reaches the next replayed step (reset_at)
    for env in (eager, graph):
        env.world.agents[1].state.pos[5] = 0.25
    out_e, out_g = _step_both(eager, graph, eager.get_random_actions())
    _assert_same(out_e, out_g, "outputs after an in-place write between steps")
    _assert_same(_state(eager), _state(graph), "state after an in-place write between steps")


@pytest.mark.gpu
def test_deferred_respawn_with_other_device_draws_gpu(gpu_device):
    """A step that draws device random numbers besides discovery's respawn (here one torch.rand in
    post_step): the deferred (in-graph) respawn would read the generator before the
    replay and share those numbers, so the capture keeps the respawn as a host hole.  Outputs,
    state, the extra draw and the generator's consumption equal the eager step's, bit for bit."""
    eager, graph = _twin_envs(gpu_device, "discovery", n_agents=4)
    for env in (eager, graph):
        sc = env.scenario

        def post_step(sc=sc, env=env):
            sc.noise = torch.rand(env.num_envs, 3, device=env.device)

        sc.post_step = post_step
    for t in range(8):
        actions = eager.get_random_actions()
        s = _rng_save()
        out_e = eager.step([a.clone() for a in actions])
        after_e = torch.cuda.get_rng_state()
        _rng_load(s)
        out_g = graph.step([a.clone() for a in actions])
        assert torch.equal(torch.cuda.get_rng_state(), after_e), f"generator consumption step {t}"
        _assert_same(out_e, out_g, f"outputs step {t}")
        _assert_same(_state(eager), _state(graph), f"state step {t}")
        assert torch.equal(eager.scenario.noise, graph.scenario.noise), t
    assert graph.graph_status == "graph", graph.graph_reason
    assert len(graph._graph._deferred) == 0 and len(graph._graph._holes) == 1


CHAIN_CASES = [("balance", dict(n_agents=4), 10), ("transport", dict(n_agents=4), None),
               ("flocking", dict(n_agents=4), None), ("discovery", dict(n_agents=4, use_agent_lidar=True), None)]


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps", CHAIN_CASES, ids=[c[0] for c in CHAIN_CASES])
def test_kernel_chain_replay_matches_graph_launch_gpu(gpu_device, name, kw, substeps):
    """A replay launched as the captured graph's kernels on the stream (_KernelChain,
    vmas_graph_chain_launch) -- balance's k_world running the scenario program as its epilogue --
    gives bit-identical outputs and state to hipGraphLaunch of the same graph (two launches),
    through a reset_at and a full reset."""
    envs = []
    for chain in (True, False):
        saved = _rng_save()
        env = make_env(name, num_envs=1024, device=gpu_device, seed=2, graph_step=True, **kw)
        env._graph._CHAIN = chain
        if substeps:
            env.world._substeps = substeps
            env.world._sub_dt = env.world._dt / substeps
        envs.append(env)
        if chain:
            _rng_load(saved)
    a, b = envs
    gen = torch.Generator(device=gpu_device).manual_seed(5)
    for t in range(16):
        actions = [torch.rand(1024, ag.action_size, device=gpu_device, generator=gen) * 2 - 1 for ag in a.agents]
        if t == 9:
            for env in (a, b):
                s = _rng_save()
                env.reset_at(5)
                _rng_load(s)
        if t == 12:
            for env in (a, b):
                s = _rng_save()
                env.reset()
                _rng_load(s)
        outs = _step_both(a, b, actions)
        _assert_same(outs[0], outs[1], f"{name} outputs step {t}")
        _assert_same(_state(a), _state(b), f"{name} state step {t}")
    assert a.graph_status == b.graph_status == "graph", (a.graph_reason, b.graph_reason)
    assert b._graph._chain is None
    if name != "discovery":  # (discovery's graph holds the respawn's deferred channel launch)
        assert a._graph._chain is not None, a._graph.chain_why
        # balance / transport: k_world with the scenario program as its epilogue, one launch per replay
        fused = name in ("balance", "transport")
        assert a._graph._chain.fused == int(fused)
        assert a._graph._chain.n_nodes == 1 if fused else a._graph._chain.n_nodes >= 2


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,substeps", CHAIN_CASES[:2], ids=[c[0] for c in CHAIN_CASES[:2]])
def test_fused_epilogue_rerun_by_a_second_pass_matches_eager_gpu(gpu_device, monkeypatch, name, kw, substeps):
    """a replay whose k_world runs the scenario program as its epilogue re-runs the
    program after every fixed-point pass of a group.  With a second pass forced on every step
    (VMAS_JIT_TEST_PASSES=2: the decider treats pass 0 as violated) the fused replay still equals
    the one-pass eager step bit for bit -- the programs are idempotent (global shaping written out of
    place, the old pos_rew zeroed) -- through a reset_at and a full reset."""
    envs = []
    for forced in (True, False):
        if forced:
            monkeypatch.setenv("VMAS_JIT_TEST_PASSES", "2")
        else:
            monkeypatch.delenv("VMAS_JIT_TEST_PASSES", raising=False)
        saved = _rng_save()
        env = make_env(name, num_envs=1024, device=gpu_device, seed=3, graph_step=forced, **kw)
        if substeps:
            env.world._substeps = substeps
            env.world._sub_dt = env.world._dt / substeps
        env.world.engine._ensure()  # (the knob is read when the kernel is generated)
        envs.append(env)
        if forced:
            _rng_load(saved)
    a, b = envs
    gen = torch.Generator(device=gpu_device).manual_seed(6)
    for t in range(12):
        actions = [torch.rand(1024, ag.action_size, device=gpu_device, generator=gen) * 2 - 1 for ag in a.agents]
        if t in (7, 10):
            for env in (a, b):
                s = _rng_save()
                env.reset_at(5) if t == 7 else env.reset()
                _rng_load(s)
        outs = _step_both(a, b, actions)
        _assert_same(outs[0], outs[1], f"{name} outputs step {t}")
        _assert_same(_state(a), _state(b), f"{name} state step {t}")
    assert a.graph_status == "graph", a.graph_reason
    assert a._graph._chain is not None and a._graph._chain.fused == 1, a._graph.chain_why
    assert "VMAS_GRID_MIN_PASSES 2" in a.world.engine.jit_source()
    assert a.world.engine.last_iterations == 2 and b.world.engine.last_iterations == 1


# ---- a user's scenario (not one of the package's) on the default step (VERDICT r5 "Next" #7) -----
from vectorizedmultiagentsimulator_amd.simulator.core import Agent, Box, Landmark, Line, Sphere, World  # noqa: E402
from vectorizedmultiagentsimulator_amd.simulator.scenario import BaseScenario  # noqa: E402


class PushScenario(BaseScenario):
    """A small scenario written the way a user writes one (reference API only): agents push a box to
    a goal past a wall line; shaping reward kept in a device tensor, per-agent collision counts."""

    def make_world(self, batch_dim, device, n_agents=3, history=False):
        world = World(batch_dim, device, substeps=3, x_semidim=1.2, y_semidim=1.2)
        for i in range(n_agents):
            world.add_agent(Agent(name=f"agent_{i}", shape=Sphere(0.05), u_multiplier=0.8))
        self.box = Landmark(name="box", shape=Box(length=0.3, width=0.2), movable=True, rotatable=True, mass=2.0)
        world.add_landmark(self.box)
        self.goal = Landmark(name="goal", shape=Sphere(0.08), collide=False)
        world.add_landmark(self.goal)
        world.add_landmark(Landmark(name="wall", shape=Line(length=1.0)))
        self.shaping = torch.zeros(batch_dim, device=device)
        self.history = [] if history else None
        return world

    def reset_world_at(self, env_index=None):
        n = 1 if env_index is not None else self.world.batch_dim
        dev = self.world.device
        for i, a in enumerate(self.world.agents):
            a.set_pos(torch.rand(n, 2, device=dev) * 1.6 - 0.8, batch_index=env_index)
        self.box.set_pos(torch.rand(n, 2, device=dev) * 0.8 - 0.4, batch_index=env_index)
        self.box.set_rot(torch.rand(n, 1, device=dev) * 3.0, batch_index=env_index)
        self.goal.set_pos(torch.tensor([[0.9, 0.9]], device=dev).expand(n, 2), batch_index=env_index)
        wall = self.world.landmarks[2]
        wall.set_pos(torch.tensor([[0.0, -0.9]], device=dev).expand(n, 2), batch_index=env_index)
        d = torch.linalg.vector_norm(self.box.state.pos - self.goal.state.pos, dim=-1)
        if env_index is None:
            self.shaping = d * 10
        else:
            self.shaping[env_index] = d[env_index] * 10

    def reward(self, agent):
        if agent is self.world.agents[0]:
            d = torch.linalg.vector_norm(self.box.state.pos - self.goal.state.pos, dim=-1)
            new = d * 10
            self.rew = self.shaping - new
            self.shaping = new
            if self.history is not None:
                self.history.append(1)  # (Python-side step state: a replay would freeze it)
        close = torch.linalg.vector_norm(agent.state.pos - self.box.state.pos, dim=-1) < 0.25
        return self.rew + close.float() * 0.01

    def observation(self, agent):
        return torch.cat([agent.state.pos, agent.state.vel, self.box.state.pos - agent.state.pos,
                          self.box.state.rot, self.goal.state.pos - self.box.state.pos], dim=-1)

    def info(self, agent):
        return {"dist": torch.linalg.vector_norm(self.box.state.pos - self.goal.state.pos, dim=-1)}


@pytest.mark.gpu
def test_user_scenario_replays_by_default_and_matches_eager_gpu(gpu_device):
    """A scenario defined outside the package gets the graph step from make_env's default
    (graph_step=None; environment.py _auto_graph_step) -- untrusted: no write-only attributes, no
    direct outputs, no state write-back -- and matches its eager twin bit for bit through reset_at
    and reset."""
    envs = []
    for graph in (None, False):
        saved = _rng_save()
        envs.append(make_env(PushScenario(), num_envs=512, device=gpu_device, seed=4, graph_step=graph))
        if graph is None:
            _rng_load(saved)
    auto, eager = envs
    assert auto.graph_auto and auto._graph is not None
    gen = torch.Generator(device=gpu_device).manual_seed(8)
    for t in range(14):
        actions = [torch.rand(512, 2, device=gpu_device, generator=gen) * 2 - 1 for _ in auto.agents]
        if t == 6:
            for env in (auto, eager):
                s2 = _rng_save()
                env.reset_at(7)
                _rng_load(s2)
        if t == 10:
            for env in (auto, eager):
                s2 = _rng_save()
                env.reset()
                _rng_load(s2)
        outs = _step_both(eager, auto, actions)
        _assert_same(outs[0], outs[1], f"user scenario outputs step {t}")
        _assert_same(_state(eager), _state(auto), f"user scenario state step {t}")
    assert auto.graph_status == "graph", auto.graph_reason
    g = auto._graph
    assert g.replays >= 5 and not g._write_only_ys and not (g._direct and g._direct.enabled)
    assert g._wb in (None, False)  # (untrusted: the carry stays)


@pytest.mark.gpu
def test_user_scenario_with_python_step_state_stays_eager_gpu(gpu_device):
    """The same scenario keeping Python-side step state in a list it appends to (an in-place change
    the plain-attribute watch cannot see): the strict watch of an untrusted scenario keeps it eager."""
    env = make_env(PushScenario(), num_envs=64, device=gpu_device, seed=0, history=True)
    for _ in range(5):
        env.step(env.get_random_actions())
    assert env.graph_status == "eager", env.graph_reason
    assert "Python-side state" in env.graph_reason and "history" in env.graph_reason, env.graph_reason
