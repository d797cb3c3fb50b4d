"""Static ISA of a world's generated k_world, without a GPU: the source the library generates for
the world (vmas_jit_compile_check, relaxed math as on the GPU), compiled here with hipcc for gfx950
and disassembled; prints instruction counts by class for the whole kernel and per wave body
(run<w>), so code-generation changes can be A/B'd on CPU before a PMC session.
usage: python tools/kworld_isa.py [scenario] [--src OUT.hip] [--asm OUT.s]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

p = argparse.ArgumentParser()
p.add_argument("scenario", nargs="?", default="balance")
p.add_argument("--src", default=None)
p.add_argument("--asm", default=None)
args = p.parse_args()

from tests._parity import make  # noqa: E402

PRESET = {"balance": (dict(n_agents=4), 10), "transport": (dict(n_agents=4), None),
          "discovery": (dict(n_agents=8, use_agent_lidar=True), None), "flocking": (dict(n_agents=8), None)}
kw, sub = PRESET.get(args.scenario, ({}, None))
env = make(args.scenario, kw, sub, "cpu", num_envs=64, seed=0)
src = env.world.engine.jit_compile_check()
flags = re.search(r"// vmas-cflags:(.*)", src)
extra = flags.group(1).split() if flags else []
tmp = Path(tempfile.mkdtemp())
(tmp / "k.hip").write_text(src)
if args.src:
    Path(args.src).write_text(src)
csrc = ROOT / "vectorizedmultiagentsimulator_amd" / "csrc"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-std=c++17", "-ffp-contract=off",
       "-fno-fast-math", f"-I{csrc}", f"-I{ROOT / 'include'}", *extra, "-S", "-o", str(tmp / "k.s"), str(tmp / "k.hip")]
subprocess.run(cmd, check=True)
asm = (tmp / "k.s").read_text()
if args.asm:
    Path(args.asm).write_text(asm)
body = asm[asm.find("k_world:"):]
body = body[:body.find(".Lfunc_end")]
cls = collections.Counter()
for line in body.splitlines():
    t = line.strip()
    if not t or t.startswith((".", ";", "//")) or t.endswith(":"):
        continue
    op = t.split()[0]
    if op.startswith("v_"):
        cls["valu" if not op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")) else "v_lane"] += 1
    elif op.startswith("s_"):
        cls["branch" if op.startswith(("s_cbranch", "s_branch")) else "salu/smem"] += 1
    elif op.startswith("ds_"):
        cls["lds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        cls["vmem"] += 1
    else:
        cls["other"] += 1
meta = {k: re.search(rf"\.{k}:\s*(\d+)", asm) for k in ("vgpr_count", "sgpr_count", "private_segment_fixed_size")}
print(f"{args.scenario}: k_world static instructions {sum(cls.values())}: {dict(cls)}")
print("  " + ", ".join(f"{k} {m.group(1)}" for k, m in meta.items() if m))
