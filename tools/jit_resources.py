"""Resource usage (VGPRs, SGPRs, scratch, LDS, occupancy) of a world's generated step kernels,
without a GPU: dump the k_world source for a scenario and compile it with hipcc
-Rpass-analysis=kernel-resource-usage, the same flags hipRTC uses (csrc/vmas_jit.hip compile()).

usage: python tools/jit_resources.py [scenario] [n_agents] [substeps]
"""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "balance"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    sub = int(sys.argv[3]) if len(sys.argv) > 3 else (10 if name == "balance" else 0)
    from tests._parity import make

    kw = {"n_agents": n} if name in ("balance", "transport", "discovery", "flocking", "features", "pollock") else {}
    env = make(name, kw, sub or None, "cpu", num_envs=8, seed=0)
    src = env.world.engine.jit_compile_check()
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "world.hip"
        f.write_text(src)
        inc = ROOT / "vectorizedmultiagentsimulator_amd" / "csrc"
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
               "-fno-fast-math", "-I", str(inc), "-I", str(ROOT / "include"), "--cuda-device-only", "-c",
               "-Rpass-analysis=kernel-resource-usage", str(f), "-o", str(Path(d) / "world.o")]
        for line in src.splitlines():  # the options compile() reads from the source
            if line.startswith("// vmas-cflags:"):
                cmd[5:5] = line.split(":", 1)[1].split()
        out = subprocess.run(cmd, capture_output=True, text=True)
        for line in out.stderr.splitlines():
            if "remark" in line:
                print(line.split("remark: ")[-1])
        if out.returncode:
            print(out.stderr[-2000:])


if __name__ == "__main__":
    main()
