"""Benchmark: env-steps/s of ``env.step(env.get_random_actions())`` (BASELINE.json metric).

Default workload (BASELINE configs[1], C2): 'balance', 32 768 envs per GPU, n_agents=4,
10 physics substeps, continuous random actions U(-1, 1).  One process per GPU (weak scaling:
every rank simulates its own 32 768 independent envs, no data-path collective).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Prints ONE JSON line (rank 0) with the driver's contract fields plus:
  roofline      -- HBM roofline of the dominant kernel (k_world, the world-specialised step
                   kernel; k_step on worlds it cannot specialise): algorithmic bytes per env-step
                   from SURVEY.md §8d (24*E_all + 24*E_dyn + 12*A) over its time per
                   launch, HIP events on the stream it runs on; `frac` is the variant the timed
                   steps run (with the scenario program as its epilogue when the replay fuses it),
                   `plain` the step kernel alone
  process_group -- (N > 1) the live group: backend, world size, per-rank rates and each rank's
                   device identity (PCI address / UUID of its GPU)
  cpu_baseline  -- the CPU oracle (PyTorch restatement of the reference tensor program) driving
                   the same host layer, timed on this host on a bounded sample (rank 0, N=1)
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import statistics
import subprocess
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--scenario", default="balance")
    p.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the scenario's §8(d) config)")
    p.add_argument("--n-agents", type=int, default=None, help="default: the scenario's §8(d) config")
    p.add_argument("--substeps", type=int, default=None,
                   help="physics substeps; default: the scenario's §8(d) config (balance C2: 10), else the "
                        "scenario's own World(substeps=...); 0 = the scenario's own")
    p.add_argument("--broadphase", default="batch", choices=["batch", "env"])
    p.add_argument("--cpu-steps", type=int, default=2, help="timed CPU-oracle steps per repeat (0 = skip)")
    p.add_argument("--cpu-repeats", type=int, default=5, help="CPU-oracle repeats (the median is reported)")
    p.add_argument("--cpu-envs", type=int, default=32768)
    p.add_argument("--event-launches", type=int, default=20,
                   help="extra eager step launches timed with HIP events after the timed region")
    p.add_argument("--device", default=None, help="override device (e.g. cpu for plumbing tests)")
    p.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                   help="auto: make_env without graph_step, the reference API's call (the package's "
                        "scenarios on a ROCm device then replay each step as one HIP graph once warm, with "
                        "the eager step's results); on: graph_step=True; off: graph_step=False (eager)")
    p.add_argument("--kw", default=None, help='extra scenario kwargs as JSON, e.g. \'{"use_agent_lidar": true}\' '
                                                '(default: the scenario\'s §8(d) config)')
    args = p.parse_args()
    preset = PRESETS.get(args.scenario, {})
    for k in ("envs", "n_agents", "substeps"):
        if getattr(args, k) is None:
            setattr(args, k, preset.get(k, {"envs": 32768, "n_agents": 4, "substeps": 0}[k]))
    if args.kw is None:
        args.kw = json.dumps(preset.get("kw", {}))
    return args


# SURVEY.md §8(d) configurations (BASELINE.json configs[1..4]); flags override each field.
# substeps 0 = the scenario's own World(substeps=...) (transport 1, discovery 2, flocking 5 --
# ref flocking.py:36); only C2 sets 10 on the world after make_env (§8(d) C2).
PRESETS = {
    "balance": {"envs": 32768, "n_agents": 4, "substeps": 10},                          # C2
    "transport": {"envs": 32768, "n_agents": 4, "substeps": 0},                         # C3
    "discovery": {"envs": 16384, "n_agents": 8, "substeps": 0, "kw": {"use_agent_lidar": True}},  # C4
    "flocking": {"envs": 32768, "n_agents": 8, "substeps": 0},                          # C5 (per GPU)
}


def make_world_env(args, device, seed):
    from vectorizedmultiagentsimulator_amd import make_env

    kw = {"n_agents": args.n_agents} if args.scenario in ("balance", "transport", "discovery", "flocking") else {}
    kw.update(json.loads(args.kw))
    cuda = str(device).startswith("cuda")
    graph = {"auto": None, "on": cuda, "off": False}[args.graph] if cuda else False
    env = make_env(args.scenario, num_envs=args.envs if device != "cpu-baseline" else args.cpu_envs,
                   device=device if device != "cpu-baseline" else "cpu", seed=seed, graph_step=graph, **kw)
    if args.substeps:
        env.world._substeps = args.substeps
        env.world._sub_dt = env.world._dt / args.substeps
    env.world.broadphase = args.broadphase
    return env


def _tail_launches() -> int:
    """Graph steps whose post-replay work ran as the tail of their fused launch (csrc/vmas_tail.hpp)."""
    from vectorizedmultiagentsimulator_amd import _native as N
    return int(N.load_host().tail_launches())


def tail_bytes_per_env_step(env) -> int:
    """Algorithmic bytes of the post-replay tail per env-step (csrc/vmas_tail.hpp): every copy's
    read + write, every increment's read + write, the store words, and the next step's random
    actions drawn ahead -- each drawn element written to the returned tensor and to the action
    buffer, whose previous value is read and written to the snapshot (16 B per element)."""
    g = getattr(env, "_graph", None)
    t = None if g is None else getattr(g, "_post_cache_wb" if g._wb else "_post_cache", None)
    if t is None:
        return 0
    from vectorizedmultiagentsimulator_amd import _native as N
    n = 0
    for r in t[4]["tbl"]:
        nb = int(r["nbytes"])
        n += 8 if nb == N.VMAS_COPY_STORE64 else 2 * max(nb, 0)
    elems = sum(int(env.get_agent_action_size(a)) for a in env.agents) * env.num_envs  # (the draw's elements)
    return round((n + 16 * elems) / env.num_envs)


def alg_bytes_per_env_step(world) -> int:
    """SURVEY.md §8d, the physics step's share: read pos/vel/rot/ang_vel of every entity (24 B),
    write them for every movable-or-rotatable entity (24 B), read every agent's force + torque
    (12 B).  The LIDAR ray distances (§8d's 4 B per ray) are written by the scenario program, not
    by the step kernel, so they are charged to that kernel (program_bytes_per_env_step)."""
    ents = world.entities
    e_dyn = sum(1 for e in ents if e.movable or e.rotatable)
    n_agents = len(world.agents)
    return 24 * len(ents) + 24 * e_dyn + 12 * n_agents


def lidar_rays(world) -> int:
    return sum(s._angles.shape[-1] for a in world.agents for s in a.sensors if hasattr(s, "_angles"))


def program_bytes_per_env_step(env) -> int:
    """Algorithmic bytes of the scenario's observation / reward / done program per env-step:
    read pos, vel, rot of every entity once (20 B; its inputs), write every agent's observation
    and reward (4 B per float, including the LIDAR distances inside the observations -- §8d's
    4 B per ray) and the done flag (1 B)."""
    world = env.world
    out = 20 * len(world.entities) + 1
    for a in env.agents:  # (the policy agents: those the environment asks for observations)
        obs = env.scenario.observation(a)
        out += 4 * sum(int(o.shape[-1]) for o in (obs.values() if isinstance(obs, dict) else [obs])) + 4
    return out


def time_program(env, n: int):
    """GPU time of the scenario program per step: the first agent's reward + observation calls
    (those launch the fused program(s) k_balance / k_transport / k_flocking / k_discovery_*; the
    other agents' calls return cached results) after a fresh eager step, captured into a HIP
    graph and replayed ``n`` times between HIP events, so that the host time of the eager calls
    is not counted.  Returns (ms per step, timer description); eager events if the calls cannot
    be captured."""
    world = env.world
    pol = getattr(world, "policy_agents", None) or world.agents
    a0 = pol[0]  # (the programs launch at the first policy agent's calls)

    def calls():
        env.scenario.reward(a0)
        env.scenario.observation(a0)

    world.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            calls()
        g.replay()
        e0.record()
        for _ in range(n):
            g.replay()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / n, f"HIP events around {n} replays of the captured calls"
    except Exception as exc:  # noqa: BLE001 -- report how it was timed instead
        ms = []
        for _ in range(n):
            world.step()
            e0.record()
            calls()
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        return statistics.median(ms), f"HIP events around eager calls (capture failed: {type(exc).__name__})"


def time_step_kernel_graph(world, n_graphs: int = 5, per_graph: int = 10):
    """The step kernel's launch duration as the timed region runs it (back to back, replayed from a
    HIP graph): ``per_graph`` chained World.step() calls -- one k_world launch each, nothing else --
    captured into one graph, replayed ``n_graphs`` times between HIP events on the stream the
    replays run on.  Returns (us per launch, launches timed).  This includes the gap between two
    kernel nodes (dispatch ramp + completion), as a kernel-trace duration does."""
    world.step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            world.step()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n_graphs):
        g.replay()
    e1.record()
    e1.synchronize()
    n = n_graphs * per_graph
    return 1e3 * e0.elapsed_time(e1) / n, n


def time_fused_chain(env, n: int = 50, warm: int = 5):
    """The step kernel as the timed steps launch it when a replay fuses the scenario program into it
    (k_world with the program as its epilogue, the one launch of a C2 replay's kernel chain): the
    chain's launch ``n`` times back to back between HIP events on the stream it runs on, after
    ``warm`` untimed launches.  (Each launch reads the same inputs -- the chain's plain variant, no
    state write-back -- so every launch does the timed steps' work.)  Returns us per launch, or None
    when the replay is not a one-launch fused chain."""
    from vectorizedmultiagentsimulator_amd import _native as N

    g = getattr(env, "_graph", None)
    ch = getattr(g, "_chain", None)
    if ch is None or not ch.fused or ch.n_nodes != 1:
        return None
    lib = N.load_library()
    dev = torch.device(env.device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    st = N.stream_ptr(idx)
    for _ in range(warm):
        N.check(lib.vmas_graph_chain_launch(ch.handle, st), "vmas_graph_chain_launch")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        N.check(lib.vmas_graph_chain_launch(ch.handle, st), "vmas_graph_chain_launch")
    e1.record()
    e1.synchronize()
    return 1e3 * e0.elapsed_time(e1) / n


def load_rocprof(kernel: str, src_hash: str, workload: str) -> dict:
    """The committed rocprofv3 kernel-trace summary of the same bench command for this exact
    kernel (profiles/rocprof_kernel.json, written by tools/rocprof_record.py), if any."""
    f = ROOT / "profiles" / "rocprof_kernel.json"
    if not f.exists():
        return {}
    try:
        d = json.loads(f.read_text())
    except Exception:
        return {}
    if d.get("kernel") != kernel or d.get("workload") != workload or d.get("kernel_source_sha256") != src_hash:
        return {"stale": "record is for another kernel source / workload"}
    return d


def kernel_source_hash(world) -> str:
    """sha256 of the generated step kernel's source (k_world) -- what a PMC record must match."""
    src = world.engine.jit_source()
    if not src:
        return ""
    # the generated source #includes these at compile time (hipRTC reads them from csrc/ and
    # include/): the kernel's identity is the source AND their text
    h = hashlib.sha256(src.encode())
    for f in ("vectorizedmultiagentsimulator_amd/csrc/vmas_jit_ops.hpp",
              "vectorizedmultiagentsimulator_amd/csrc/vmas_physics.hpp",
              "vectorizedmultiagentsimulator_amd/csrc/vmas_tail.hpp", "include/vmas_mi355x.h") + (
            ("vectorizedmultiagentsimulator_amd/csrc/vmas_programs.hpp",
             "vectorizedmultiagentsimulator_amd/csrc/vmas_query.hpp") if '#include "vmas_programs.hpp"' in src else ()):
        h.update((ROOT / f).read_bytes())
    return h.hexdigest()


def load_pmc(workload: str, kernel: str, src_hash: str) -> dict:
    """Per-launch PMC record of the step kernel (profiles/pmc_traffic.json, written by
    tools/pmc_traffic.py from rocprofv3 CSVs kept under profiles/), only if it was measured on
    this workload AND on this exact kernel (the generated source's sha256)."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return {}
    try:
        d = json.loads(f.read_text())
    except Exception:
        return {}
    if d.get("workload") != workload or d.get("kernel") != kernel:
        return {"stale": "record is for another workload / kernel"}
    if not src_hash or d.get("kernel_source_sha256") != src_hash:
        return {"stale": "record was measured on another k_world source (sha256 mismatch)"}
    return d


def cpu_model() -> str:
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


# VALU issue peak of the MI355X (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs, one wave64 VALU
# instruction per 2 cycles per SIMD, 2.4 GHz -> 1.23e12 wave-instructions/s (= the 157.3 TF/s
# fp32 vector peak / 128 flop per wave-FMA)
VALU_PEAK_WAVE_INSTS = 256 * 4 * 0.5 * 2.4e9


def cpu_baseline(args):
    """Oracle physics (torch CPU, reference op sequence) under the same host layer: the median of
    ``--cpu-repeats`` timings of ``--cpu-steps`` steps, at the bench's substeps and at substeps=1
    (BASELINE.md's reference number is quoted at substeps=1)."""
    from oracle import vmas_oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)

    def timed(substeps):
        a = argparse.Namespace(**vars(args))
        a.substeps = substeps
        env = make_world_env(a, "cpu-baseline", seed=0)
        vmas_oracle.install(env.world)
        env.step(env.get_random_actions())  # warm-up
        rates = []
        for _ in range(args.cpu_repeats):
            t0 = time.perf_counter()
            for _ in range(args.cpu_steps):
                env.step(env.get_random_actions())
            rates.append(args.cpu_envs * args.cpu_steps / (time.perf_counter() - t0))
        return statistics.median(rates), rates

    med, rates = timed(args.substeps)
    med1, rates1 = timed(1)
    return {
        "value": med,
        "unit": "env-steps/s",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "cpu_model": cpu_model(),
        "sample": f"{args.scenario} {args.cpu_envs} envs, median of {args.cpu_repeats} x {args.cpu_steps} steps "
                  f"(after 1 warm-up), substeps={args.substeps}, PyTorch-CPU oracle physics, "
                  f"{torch.get_num_threads()} threads",
        "repeats": [round(r, 1) for r in rates],
        "substeps1": {"value": med1, "repeats": [round(r, 1) for r in rates1],
                      "note": "same sample at substeps=1 (the configuration of BASELINE.md's reference CPU number)"},
    }


def device_identity(device: str, rank: int, local_rank: int) -> dict:
    """Which device this rank ran on, as the rank itself sees it: the PCI address and UUID of its
    GPU (torch.cuda.get_device_properties), the visible-device lists it was started with, its host
    and pid -- so a multi-GPU line can show that N distinct GPUs ran (VERDICT r5 "Next" #8)."""
    ident = {"rank": rank, "local_rank": local_rank, "device": device, "host": socket.gethostname(),
             "pid": os.getpid()}
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if os.environ.get(k) is not None:
            ident[k] = os.environ[k]
    if device.startswith("cuda"):
        pr = torch.cuda.get_device_properties(torch.device(device))
        ident["pci"] = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
        ident["uuid"] = str(getattr(pr, "uuid", ""))
        ident["name"] = pr.name
        ident["key"] = f"{ident['host']}/{ident['pci']}"
    else:  # (CPU ranks: distinct processes)
        ident["key"] = f"{ident['host']}/cpu/pid{ident['pid']}"
    return ident


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, device) -> int:
    """``--gpus N`` without a launcher: start N ranks (one process per GPU) under
    torch.distributed.run as a CHILD process and return its exit code.  Runs before this process
    touches the GPU (no HIP call has been made yet; counting devices does not initialise it)."""
    if device is None or str(device).startswith("cuda"):
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(Path(__file__).resolve()),
           *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, args.device))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size != args.gpus:
        print(f"bench.py: WORLD_SIZE={world_size} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world_size > 1:
        import torch.distributed as dist

        backend = "nccl" if (torch.cuda.is_available() and args.device != "cpu") else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend)
    if args.device is not None:
        device = args.device
    else:
        device = f"cuda:{local_rank}" if torch.cuda.is_available() else "cpu"
    on_gpu = device.startswith("cuda")
    if on_gpu:
        torch.cuda.set_device(torch.device(device))

    env = make_world_env(args, device, seed=rank)
    world = env.world

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            if on_gpu:
                dist.barrier(device_ids=[torch.device(device).index])
            else:
                dist.barrier()

    if on_gpu:
        world.engine.set_timing(True)
    for _ in range(args.warmup):
        env.step(env.get_random_actions())
    if on_gpu:
        world.engine.get_timing(reset=True)
        world.engine.device_timing(reset=True)
    sync()
    barrier()
    sync()
    handovers = type(env.scenario).make_world.__globals__.get("HANDOVERS", [0])  # (discovery's respawn)
    h0 = handovers[0]
    tails0 = _tail_launches() if on_gpu else 0
    ev_region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if on_gpu else None
    if ev_region:
        ev_region[0].record()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        env.step(env.get_random_actions())
    if ev_region:
        ev_region[1].record()
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    tails = (_tail_launches() - tails0) if on_gpu else 0
    # the GPU time of the timed region itself (HIP events on the step stream around the loop); per
    # launch when every step was exactly one launch (a one-launch kernel chain that also ran the
    # post-replay work as its tail: nothing else is queued per step)
    region_us = ev_region[0].elapsed_time(ev_region[1]) * 1e3 / args.steps if ev_region else None
    gch = getattr(getattr(env, "_graph", None), "_chain", None)
    one_launch = bool(on_gpu and env.graph_status == "graph" and gch is not None and gch.n_nodes == 1
                      and tails == args.steps)
    kernel_ms, launches, timer, clock_ghz = 0.0, 0, None, 0.0
    event_us = fused_us = None
    if on_gpu:
        # (the timed region's own launches: read before the fused timer's launches add to the count)
        dev_ms, dev_n, clock_ghz = world.engine.device_timing(reset=True, with_clock=True)
    if on_gpu and args.event_launches > 0 and env.graph_status == "graph":
        # (first launches after the timed region: tools/rocprof_record.py finds these 5 + 50 there)
        fused_us = time_fused_chain(env)
    if on_gpu:
        if env.graph_status == "graph":
            # replayed launches: HIP records no events inside a graph; the kernel's own timer
            kernel_ms, launches = dev_ms, dev_n
            world.engine.get_timing(reset=True)
            timer = "in-kernel s_memrealtime (workgroup 0 start -> final pass decided), graph replays"
        else:
            kernel_ms, launches = world.engine.get_timing(reset=True)
            timer = "HIP events on the launch's dispatch packet (hipExtModuleLaunchKernel)"
        if args.event_launches > 0:
            # after the timed region: eager launches of the same step kernel on the same state
            # chain, timed by HIP events on their own dispatch packets (what rocprofv3's kernel
            # trace measures; the in-kernel timer misses the launch ramp and the exit tail)
            world.engine.get_timing(reset=True)
            for _ in range(args.event_launches):
                world.step()
            ev_ms, ev_n = world.engine.get_timing(reset=True)
            event_us = 1e3 * ev_ms / ev_n if ev_n else None
    program = None
    if on_gpu and args.event_launches > 0:
        prog_ms, prog_timer = time_program(env, args.event_launches)
        p_env = program_bytes_per_env_step(env)
        ach = p_env * args.envs / (prog_ms * 1e-3) / 1e9
        program = {
            "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 5),
            "kernel": f"{args.scenario} scenario program (first agent's reward + observation calls)",
            "us_per_step": round(prog_ms * 1e3, 3), "alg_bytes_per_env_step": p_env,
            "lidar_rays_per_env": lidar_rays(world),
            "timer": prog_timer,
        }
    group = None
    graph_us = None
    if on_gpu and args.event_launches > 0 and env.graph_status == "graph":
        try:
            graph_us, graph_n = time_step_kernel_graph(world)
        except Exception as exc:  # noqa: BLE001 -- the eager events stay the headline then
            print(f"bench.py: graph-replay kernel timer unavailable ({type(exc).__name__}: {exc})", file=sys.stderr)
    if dist is not None:
        # what the live process group saw (not the launcher's environment): its size, backend and
        # every rank's own rate, gathered once after the timed region
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if on_gpu else "cpu")
        ranks = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(ranks, t)
        per_rank = [args.envs * args.steps / float(r.item()) for r in ranks]
        elapsed = max(float(r.item()) for r in ranks)
        idents = [None] * dist.get_world_size()
        dist.all_gather_object(idents, device_identity(device, rank, local_rank))
        group = {"backend": str(dist.get_backend()), "world_size": dist.get_world_size(),
                 "per_rank_env_steps_per_s": [round(r, 1) for r in per_rank],
                 "timing": "max over ranks of each rank's barrier-bracketed wall time",
                 "devices": idents,
                 "distinct_devices": len({d["key"] for d in idents})}
        world_size = dist.get_world_size()

    total_envs = args.envs * world_size
    value = total_envs * args.steps / elapsed
    workload = (f"{args.scenario} {args.envs} envs/GPU, n_agents={args.n_agents}, substeps={world._substeps}, "
                f"broadphase={args.broadphase}")
    step_mode = env.graph_status if env.graph_status != "off" else "eager"
    if env.graph_auto:
        step_mode += " (chosen by make_env's default graph_step=None)"
    g = getattr(env, "_graph", None)
    if g is not None and env.graph_status == "graph":
        # how a replay is launched: the graph's kernels on the stream, or hipGraphLaunch
        step_mode += (f"; replay: {g._chain.n_nodes}-launch kernel chain"
                      + (f" ({g._chain.fused} scenario program as k_world's epilogue)" if g._chain.fused else "")
                      if g._chain is not None
                      else f"; replay: hipGraphLaunch ({g.chain_why or 'torch replay'})")
        if tails:  # (csrc/vmas_tail.hpp: the post-replay work inside the same launch)
            step_mode += f"; post-replay work as that launch's tail in {tails} of {args.steps} timed steps"
    if json.loads(args.kw):
        workload += f", {args.kw}"
    b_env = alg_bytes_per_env_step(world)
    src = world.engine.jit_source() if on_gpu else ""
    # relaxed: the generated step kernel uses hardware rcp / sqrt / exp / log / sin / cos (fp32,
    # within the oracle tolerance); exact: IEEE div / sqrt, ocml transcendentals
    math_mode = ("relaxed" if "VMAS_PHYS_RELAXED" in (src or "") else "exact") if on_gpu else "exact (host backend)"
    roofline = None
    if on_gpu and launches:
        inkernel_ms = kernel_ms / launches
        # the headline: HIP events around back-to-back graph replays of the step kernel alone (the
        # timed region's launch mode; includes the dispatch ramp and completion between kernel
        # nodes).  Beside it: events on eager launches (an idle GPU between launches) and the
        # in-kernel timer of the timed region itself (workgroup 0 start -> final pass decided).
        plain = fused_no_tail = None
        if graph_us:
            per_launch_ms, headline_timer = graph_us * 1e-3, (
                f"HIP events around {graph_n} back-to-back launches replayed from a HIP graph of "
                f"World.step() calls (the step kernel alone), after the timed region")
            if fused_us:
                # the headline is the variant the timed steps run (VERDICT r5 "Next" #1): k_world with
                # the scenario program as its epilogue; the step kernel alone beside it
                plain = {"kernel_us": round(graph_us, 3),
                         "achieved": round(b_env * args.envs / (graph_us * 1e-6) / 1e9, 2),
                         "frac": round(b_env * args.envs / (graph_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5),
                         "timer": headline_timer}
                per_launch_ms, headline_timer = fused_us * 1e-3, (
                    "HIP events around 50 back-to-back launches of the replay's one-launch kernel chain "
                    "(k_world with the scenario program as its epilogue: what the timed steps launch), "
                    "after the timed region")
                if one_launch and region_us:
                    # every timed step was ONE k_world launch (physics + the program as its epilogue +
                    # the post-replay work as its tail, csrc/vmas_tail.hpp): the headline is that
                    # launch, timed over the timed region itself; the chain without the tail beside it
                    fused_no_tail = {"kernel_us": round(fused_us, 3),
                                     "achieved": round(b_env * args.envs / (fused_us * 1e-6) / 1e9, 2),
                                     "frac": round(b_env * args.envs / (fused_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5),
                                     "timer": headline_timer.replace("(k_world with the scenario program as its "
                                                                     "epilogue: what the timed steps launch)",
                                                                     "(k_world with the scenario program as its "
                                                                     "epilogue, without the tail)")}
                    per_launch_ms, headline_timer = region_us * 1e-3, (
                        f"HIP events on the step stream around the timed region / {args.steps} steps: one "
                        f"k_world launch per step, back to back (nothing else queued)")
        elif event_us:
            per_launch_ms, headline_timer = event_us * 1e-3, "HIP events on the dispatch packets of eager launches"
        else:
            per_launch_ms, headline_timer = inkernel_ms, timer
        achieved = b_env * args.envs / (per_launch_ms * 1e-3) / 1e9
        src_hash = kernel_source_hash(world)
        pmc = load_pmc(workload, world.engine.kernel_name, src_hash)
        traffic = pmc.get("hbm_bytes_per_launch")
        rp = load_rocprof(world.engine.kernel_name, src_hash, workload)
        roofline = {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "kernel": world.engine.kernel_name,
            "variant": ("k_world + the scenario program as its epilogue + the post-replay tail (the timed "
                        "steps' one launch)" if fused_no_tail else
                        "k_world + the scenario program as its epilogue (the timed steps' launch)" if plain
                        else "the step kernel alone"),
            "kernel_us_per_launch": round(per_launch_ms * 1e3, 3),
            "timer": headline_timer,
            "plain": plain,
            "fused_no_tail": fused_no_tail,
            "kernel_us_eager_events": round(event_us, 3) if event_us else None,
            "launches_per_step": round(launches / args.steps, 3),
            "alg_bytes_per_env_step": b_env,
            "kernel_us_timed_region": round(inkernel_ms * 1e3, 3),
            "timer_timed_region": timer,
            "frac_timed_region": round(b_env * args.envs / (inkernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "kernel_source_sha256": src_hash,
            "pmc_record": ("profiles/pmc_traffic.json" if traffic else pmc.get("stale", "none")),
        }
        if plain:
            # the fused launch's own algorithmic bytes: the physics step's (above) plus the scenario
            # program's outputs (observations, rewards, done; its state inputs are the step's own
            # outputs, read back inside the launch) -- what its PMC traffic compares with
            b_fused = b_env + program_bytes_per_env_step(env) - 20 * len(world.entities)
            b_tail = tail_bytes_per_env_step(env) if fused_no_tail else 0
            b_fused += b_tail
            roofline["fused_alg"] = {
                "bytes_per_env_step": b_fused,
                "tail_bytes_per_env_step": b_tail,
                "achieved": round(b_fused * args.envs / (per_launch_ms * 1e-3) / 1e9, 2),
                "frac": round(b_fused * args.envs / (per_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                "traffic_over_alg": round(traffic / (b_fused * args.envs), 3) if traffic else None,
                "note": ("roofline.achieved / frac keep SURVEY 8(d)'s physics bytes (384 B) over the launch's "
                         "time; this adds the epilogue's outputs and the post-replay tail's items (the next "
                         "step's draw and its snapshot, the carry, the step counter).  PMC traffic above it = "
                         "the state write-back's two extra stores (inputs + first-pass backup; DESIGN.md) and "
                         "the FETCH_SIZE x2 correction applied to narrow reads"),
            }
        if rp.get("avg_us"):
            # the same command under rocprofv3 --kernel-trace (committed record, same kernel sha):
            # the profiler's own dispatch handling slows the kernel itself (DESIGN.md Measurement).
            # Headline = the fused variant: compared with the record's fused-timer launches
            # (fused_timer_us), else the timed steps' (in_step_us); the plain figure with avg_us.
            rp_us = (rp.get("in_step_us") if fused_no_tail else
                     (rp.get("fused_timer_us") or rp.get("in_step_us")) if plain else rp["avg_us"])
            roofline["rocprof"] = {"kernel_us": rp_us, "calls": rp.get("calls"),
                                   "frac": round(b_env * args.envs / (rp_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5),
                                   "ratio_to_headline": round(rp_us / (per_launch_ms * 1e3), 4),
                                   "plain_kernel_us": rp["avg_us"],
                                   "in_step_us": rp.get("in_step_us"),
                                   "summary": rp.get("summary")}
        elif rp:
            roofline["rocprof"] = rp
        if pmc.get("valu_insts_per_launch"):
            # the bound the kernel actually meets: VALU issue, from PMC SQ_INSTS_VALU
            rate = pmc["valu_insts_per_launch"] / (per_launch_ms * 1e-3)
            roofline["valu_issue"] = {
                "achieved": round(rate / 1e9, 1),
                "peak": round(VALU_PEAK_WAVE_INSTS / 1e9, 1),
                "unit": "G wave-instructions/s",
                "frac": round(rate / VALU_PEAK_WAVE_INSTS, 4),
                "valu_insts_per_launch": round(pmc["valu_insts_per_launch"]),
            }
            if clock_ghz > 0:
                # the same peak at the shader clock the chip held inside the kernel (in-kernel
                # s_memtime / s_memrealtime): DVFS lowers it well below 2.4 GHz under this load
                peak_at_clock = 256 * 4 * 0.5 * clock_ghz * 1e9
                roofline["valu_issue"]["clock_ghz"] = round(clock_ghz, 3)
                roofline["valu_issue"]["frac_at_clock"] = round(rate / peak_at_clock, 4)
    if args.scenario == "balance" and args.envs == 32768:
        metric = "env-steps/sec (num_envs x steps / wall-s), 'balance' @32k envs, 1->8 GPU"  # BASELINE.json
    else:
        metric = (f"env-steps/sec (num_envs x steps / wall-s), '{args.scenario}' @{args.envs} envs"
                  + ("/GPU" if on_gpu else " on CPU"))
    out = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: scenario reset states (seed = rank), random actions U(-u_range, u_range) each step",
        "config": {
            "workload": workload,
            "scenario": args.scenario,
            "num_envs_per_gpu": args.envs,
            "global_envs": total_envs,
            "n_agents": args.n_agents,
            "substeps": world._substeps,
            "parallelism": f"replicas x{world_size} (one process per GPU, no collective in the step)",
            "step_mode": step_mode,
            "math": math_mode,
        },
        "roofline": roofline,
        "roofline_program": program,
    }
    if group is not None:
        out["process_group"] = group
    if args.scenario == "discovery":  # (one-launch respawns redone: by the per-target kernels or the reference loop)
        g_ = type(env.scenario).make_world.__globals__
        out["config"]["respawn_handovers"] = {
            "timed": handovers[0] - h0, "total": handovers[0],
            "to_reference_loop": g_.get("REFERENCE_LOOP", [None])[0],
            "why": g_.get("HANDOVER_LOG", [])}
    if rank == 0 and world_size == 1 and args.cpu_steps > 0:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
