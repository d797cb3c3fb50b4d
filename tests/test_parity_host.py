"""Host backend of libvmas_mi355x.so (device="cpu", same arithmetic as the gfx950 kernels) vs the
CPU oracle: one teacher-forced World.step per check, LIDAR scans and distance queries.
Tolerances: oracle.vmas_oracle.compare (fp32 atol/rtol + 4x the system's 1-ulp sensitivity)."""
import pytest

from tests._parity import SCENARIOS, distance_parity, lidar_parity, make, step_parity, summarize


@pytest.mark.parametrize("name,kw,substeps", SCENARIOS, ids=[s[0] for s in SCENARIOS])
def test_step_parity_host(name, kw, substeps):
    env = make(name, kw, substeps, "cpu", num_envs=48, seed=0)
    reps = step_parity(env, n_steps=4)
    summarize(f"{name} 48 envs (host backend)", env, reps)
    for rep in reps:
        assert rep["ok"], rep


@pytest.mark.parametrize("name,kw,substeps", SCENARIOS, ids=[s[0] for s in SCENARIOS])
def test_lidar_and_distance_parity_host(name, kw, substeps):
    env = make(name, kw, substeps, "cpu", num_envs=32, seed=1)
    for _ in range(3):
        env.step(env.get_random_actions())
    rep = lidar_parity(env)
    assert rep["ok"], rep
    rep = distance_parity(env)
    assert rep["ok"], rep


def test_env_broadphase_mode_host():
    """broadphase='env' (every candidate pair in every env) equals the oracle without the
    batch-any test."""
    env = make("pollock", dict(n_agents=4, n_lines=3, n_boxes=3), None, "cpu", num_envs=32, seed=2)
    for rep in step_parity(env, n_steps=3, broadphase="env"):
        assert rep["ok"], rep


def test_batch_broadphase_fixed_point_host():
    """Reference semantics of World.collides (core.py:2796-2800): a pair in no env's circumscribed
    range is skipped even where its thin-shell force (dist <= r + LINE_MIN_DIST) is non-zero.
    The engine's dense first pass detects the violation and re-runs with the activity mask."""
    import torch

    from oracle import vmas_oracle as O

    env = make("pollock", dict(n_agents=1, n_lines=1, n_boxes=0), None, "cpu", num_envs=2, seed=0)
    w = env.world
    line, agent = w.landmarks[0], w.agents[0]
    d = line.shape.length / 2 + agent.shape.radius + 0.002
    agent.set_pos(torch.tensor([[d, 0.0], [d, 0.0]]), batch_index=None)
    agent.set_vel(torch.zeros(2, 2), batch_index=None)
    line.set_pos(torch.zeros(2, 2), batch_index=None)
    line.set_rot(torch.zeros(2, 1), batch_index=None)
    rep = O.compare_one_step(w)
    assert rep["ok"], rep
    assert rep["iterations"] == 2, rep  # dense pass violated -> masked re-run
    # under per-env broadphase the thin-shell force does act
    agent.set_pos(torch.tensor([[d, 0.0], [d, 0.0]]), batch_index=None)
    agent.set_vel(torch.zeros(2, 2), batch_index=None)
    line.set_pos(torch.zeros(2, 2), batch_index=None)
    line.set_rot(torch.zeros(2, 1), batch_index=None)
    w.broadphase = "env"
    w.step()
    assert float(agent.state.vel[0, 0]) > 0.0
