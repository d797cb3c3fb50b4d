"""Build checks of libvmas_mi355x.so's gfx950 code object (no GPU needed): every kernel runs out
of registers / LDS -- no private (scratch) memory, whose traffic silently multiplies a kernel's
HBM bytes (a partly unrolled loop indexing a register array dynamically put k_flocking_fast's
arrays in scratch: 8x the output bytes written).  The exceptions: k_step<true>, the generic step
for worlds beyond the LDS budget, whose rows live in a global slab by design, and the gradient
kernels (vmas_grad.hip: one env's step in dual numbers with 8 tangents per thread, the backward
of grad_enabled worlds, not a hot path)."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "vectorizedmultiagentsimulator_amd" / "libvmas_mi355x.so"
LLVM = Path("/opt/rocm/lib/llvm/bin")
ALLOWED_SCRATCH = {"_Z6k_stepILb1EEv5StepK", "_ZN12_GLOBAL__N_16k_gradENS_8GradArgsE",
                   "_ZN12_GLOBAL__N_110k_dist_vjpENS_8DistArgsE", "_ZN12_GLOBAL__N_19k_ray_vjpENS_10RayVjpArgsE"}


def _kernel_private_sizes(tmp_path):
    objcopy, bundler, readelf = LLVM / "llvm-objcopy", LLVM / "clang-offload-bundler", LLVM / "llvm-readelf"
    if not all(p.exists() for p in (objcopy, bundler, readelf)):
        pytest.skip("ROCm LLVM tools not found")
    fb = tmp_path / "fatbin.bin"
    subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fb}", LIB, tmp_path / "stripped.so"], check=True)
    # one offload bundle per translation unit, concatenated in the section
    data = fb.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = {}
    for k, a in enumerate(starts):
        part, co = tmp_path / f"bundle{k}.bin", tmp_path / f"gfx950_{k}.o"
        part.write_bytes(data[a:starts[k + 1] if k + 1 < len(starts) else len(data)])
        subprocess.run([bundler, "--type=o", f"--input={part}", "--unbundle",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([readelf, "--notes", co], check=True, capture_output=True, text=True).stdout
        names = re.findall(r"^\s+\.name:\s+(\S+)", notes, re.M)
        sizes = [int(x) for x in re.findall(r"^\s+\.private_segment_fixed_size:\s+(\d+)", notes, re.M)]
        assert len(names) == len(sizes)
        out.update(zip(names, sizes))
    assert out
    return out


def test_kernels_use_no_scratch(tmp_path):
    sizes = _kernel_private_sizes(tmp_path)
    assert any("k_flocking_fast" in n for n in sizes)
    bad = {n: s for n, s in sizes.items() if s and n not in ALLOWED_SCRATCH}
    assert not bad, bad


def test_no_memset_calls_that_a_capture_could_record():
    """No hipMemsetAsync in the library's sources (a stream capture would record it as a memset
    node; two graph-mode failures traced to captured memset nodes on ROCm 7.2 / MI355X, DESIGN.md
    "Graph mode"): stream-ordered clears go through a kernel (vmas_aux::fill_u32_async)."""
    csrc = ROOT / "vectorizedmultiagentsimulator_amd" / "csrc"
    for f in sorted(csrc.glob("*.hip")) + sorted(csrc.glob("*.hpp")) + sorted(csrc.glob("*.cpp")):
        code = re.sub(r"//[^\n]*", "", f.read_text())  # (comments may name it)
        assert "hipMemsetAsync" not in code and "hipMemsetD" not in code, f.name
