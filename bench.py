"""Benchmark: env-steps/s of ``env.step(env.get_random_actions())`` (BASELINE.json metric).

Default workload (BASELINE configs[1], C2): 'balance', 32 768 envs per GPU, n_agents=4,
10 physics substeps, continuous random actions U(-1, 1).  One process per GPU (weak scaling:
every rank simulates its own 32 768 independent envs, no data-path collective).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Prints ONE JSON line (rank 0) with the driver's contract fields plus:
  roofline      -- HBM roofline of the dominant kernel (k_step), timed with HIP events on its
                   launch stream inside the library; algorithmic bytes per env-step from
                   SURVEY.md §8d (24*E_all + 24*E_dyn + 12*A)
  cpu_baseline  -- the CPU oracle (PyTorch restatement of the reference tensor program) driving
                   the same host layer, timed on this host on a bounded sample (rank 0, N=1)
"""
from __future__ import annotations

import argparse
import json
import os
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
    p.add_argument("--envs", type=int, default=32768, help="envs per GPU")
    p.add_argument("--n-agents", type=int, default=4)
    p.add_argument("--substeps", type=int, default=10)
    p.add_argument("--broadphase", default="batch", choices=["batch", "env"])
    p.add_argument("--cpu-steps", type=int, default=6, help="timed CPU-oracle steps (0 = skip)")
    p.add_argument("--cpu-envs", type=int, default=32768)
    p.add_argument("--device", default=None, help="override device (e.g. cpu for plumbing tests)")
    p.add_argument("--graph", default="on", choices=["on", "off"],
                   help="on: make_env(graph_step=True) -- each step replayed as one HIP graph once warm "
                        "(same results as eager; falls back to eager if the step cannot be captured)")
    p.add_argument("--kw", default="{}", help='extra scenario kwargs as JSON, e.g. \'{"use_agent_lidar": true}\'')
    return p.parse_args()


def make_world_env(args, device, seed):
    from vectorizedmultiagentsimulator_amd import make_env

    kw = {"n_agents": args.n_agents} if args.scenario in ("balance", "transport", "discovery", "flocking") else {}
    kw.update(json.loads(args.kw))
    graph = args.graph == "on" and str(device).startswith("cuda")
    env = make_env(args.scenario, num_envs=args.envs if device != "cpu-baseline" else args.cpu_envs,
                   device=device if device != "cpu-baseline" else "cpu", seed=seed, graph_step=graph, **kw)
    if args.substeps:
        env.world._substeps = args.substeps
        env.world._sub_dt = env.world._dt / args.substeps
    env.world.broadphase = args.broadphase
    return env


def alg_bytes_per_env_step(world) -> int:
    """read pos/vel/rot/ang_vel of every entity (24 B), write them for every
    movable-or-rotatable entity (24 B), read every agent's force + torque (12 B)."""
    ents = world.entities
    e_dyn = sum(1 for e in ents if e.movable or e.rotatable)
    n_agents = len(world.agents)
    return 24 * len(ents) + 24 * e_dyn + 12 * n_agents


def load_pmc(workload: str, kernel: str) -> dict:
    """Per-launch PMC record of the step kernel (profiles/pmc_traffic.json, written by
    tools/pmc_traffic.py), if it was measured on this workload and this kernel."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return {}
    try:
        d = json.loads(f.read_text())
        if d.get("workload") == workload and d.get("kernel") == kernel:
            return d
    except Exception:
        return {}
    return {}


# VALU issue peak of the MI355X (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs, one wave64 VALU
# instruction per 2 cycles per SIMD, 2.4 GHz -> 1.23e12 wave-instructions/s (= the 157.3 TF/s
# fp32 vector peak / 128 flop per wave-FMA)
VALU_PEAK_WAVE_INSTS = 256 * 4 * 0.5 * 2.4e9


def cpu_baseline(args):
    """Oracle physics (torch CPU, reference op sequence) under the same host layer."""
    from oracle import vmas_oracle

    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    env = make_world_env(args, "cpu-baseline", seed=0)
    vmas_oracle.install(env.world)
    env.step(env.get_random_actions())  # warm-up
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        env.step(env.get_random_actions())
    dt = time.perf_counter() - t0
    return {
        "value": args.cpu_envs * args.cpu_steps / dt,
        "unit": "env-steps/s",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "sample": f"{args.scenario} {args.cpu_envs} envs x {args.cpu_steps} steps (after 1 warm-up), "
                  f"substeps={args.substeps}, PyTorch-CPU oracle physics",
        "ms_per_step": 1e3 * dt / args.cpu_steps,
    }


def main():
    args = parse()
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
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
    t0 = time.perf_counter()
    for _ in range(args.steps):
        env.step(env.get_random_actions())
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    kernel_ms, launches, timer, clock_ghz = 0.0, 0, None, 0.0
    if on_gpu:
        dev_ms, dev_n, clock_ghz = world.engine.device_timing(reset=True, with_clock=True)
        if env.graph_status == "graph":
            # replayed launches: HIP records no events inside a graph; the kernel's own timer
            kernel_ms, launches = dev_ms, dev_n
            world.engine.get_timing(reset=True)
            timer = "in-kernel s_memrealtime (workgroup 0 start -> final reduction), graph replays"
        else:
            kernel_ms, launches = world.engine.get_timing(reset=True)
            timer = "HIP events on the launch's dispatch packet (hipExtModuleLaunchKernel)"
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if on_gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_envs = args.envs * world_size
    value = total_envs * args.steps / elapsed
    workload = (f"{args.scenario} {args.envs} envs/GPU, n_agents={args.n_agents}, substeps={world._substeps}, "
                f"broadphase={args.broadphase}")
    step_mode = env.graph_status if env.graph_status != "off" else "eager"
    if json.loads(args.kw):
        workload += f", {args.kw}"
    b_env = alg_bytes_per_env_step(world)
    roofline = None
    if on_gpu and launches:
        per_launch_ms = kernel_ms / launches
        achieved = b_env * args.envs / (per_launch_ms * 1e-3) / 1e9
        pmc = load_pmc(workload, world.engine.kernel_name)
        traffic = pmc.get("hbm_bytes_per_launch")
        roofline = {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "kernel": world.engine.kernel_name,
            "kernel_us_per_launch": round(per_launch_ms * 1e3, 3),
            "launches_per_step": round(launches / args.steps, 3),
            "alg_bytes_per_env_step": b_env,
            "timer": timer,
        }
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
    out = {
        "metric": "env-steps/sec (num_envs x steps / wall-s), 'balance' @32k envs, 1->8 GPU",
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
        },
        "roofline": roofline,
    }
    if rank == 0 and world_size == 1 and args.cpu_steps > 0:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
