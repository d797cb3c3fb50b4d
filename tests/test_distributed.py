"""bench.py's multi-GPU path (one process per GPU, replicas, max-over-ranks timing) rehearsed
with world_size=2 on CPU over gloo."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_gloo():
    env = dict(os.environ, OMP_NUM_THREADS="2", VMAS_HOST_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--envs", "64", "--cpu-steps", "0", "--device", "cpu"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints exactly one JSON line
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["scaling"] == "weak"
    assert rec["config"]["global_envs"] == 128
    assert rec["value"] > 0 and rec["steps"] == 3
    # the live process group, not the launcher's environment (VERDICT r4 "Next" #7)
    pg = rec["process_group"]
    assert pg["world_size"] == 2 and pg["backend"] == "gloo"
    rates = pg["per_rank_env_steps_per_s"]
    assert len(rates) == 2 and all(r > 0 for r in rates)
    # value = all ranks' env-steps over the slowest rank's time: <= the sum of the ranks' own rates
    # (the per-rank rates are printed rounded to 0.1 env-steps/s)
    assert rec["value"] <= sum(rates) + 0.1 * len(rates) and rec["value"] >= 2 * (min(rates) - 0.05) - 1e-6
    assert "balance" in rec["metric"] and "@64 envs on CPU" in rec["metric"]
    # each rank's own device identity (VERDICT r5 "Next" #8): distinct ranks, distinct devices
    devs = pg["devices"]
    assert [d["rank"] for d in devs] == [0, 1] and pg["distinct_devices"] == 2
    assert len({d["key"] for d in devs}) == 2 and len({d["pid"] for d in devs}) == 2


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` with no launcher starts the two ranks itself (torch.distributed.run as
    a child process): the driver's BENCH command shape."""
    env = dict(os.environ, OMP_NUM_THREADS="2", VMAS_HOST_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--envs", "64", "--cpu-steps", "0", "--device", "cpu"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_envs"] == 128


def test_bench_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--envs", "8",
           "--cpu-steps", "0", "--device", "cpu"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


def test_bench_presets():
    """C5 needs no extra flags: flocking's own substeps (ref flocking.py:36: substeps=5), not C2's 10."""
    sys.path.insert(0, str(ROOT))
    import bench

    argv = sys.argv
    try:
        sys.argv = ["bench.py", "--scenario", "flocking", "--envs", "32768", "--n-agents", "8"]
        a = bench.parse()
        assert a.substeps == 0 and a.envs == 32768 and a.n_agents == 8
        sys.argv = ["bench.py"]
        a = bench.parse()
        assert (a.scenario, a.envs, a.n_agents, a.substeps) == ("balance", 32768, 4, 10)
        sys.argv = ["bench.py", "--scenario", "discovery"]
        a = bench.parse()
        assert a.envs == 16384 and a.n_agents == 8 and json.loads(a.kw) == {"use_agent_lidar": True}
    finally:
        sys.argv = argv
