"""The C-ABI library loads (no GPU needed) and exports every entry point include/*.h declares;
struct layouts seen by Python match the header."""
import ctypes
import re
import subprocess
from pathlib import Path

from vectorizedmultiagentsimulator_amd import _native as N

ROOT = Path(__file__).resolve().parent.parent


def declared_functions():
    text = (ROOT / "include" / "vmas_mi355x.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|const char\*)\s+(vmas_\w+)\s*\(", text, re.M)))


def test_library_loads_and_abi_version():
    lib = N.load_library()
    assert lib.vmas_abi_version() == N.VMAS_ABI_VERSION
    assert lib.vmas_device_count() >= 0


def test_exports_every_declared_symbol():
    decl = declared_functions()
    assert set(decl) == set(N.EXPORTED_SYMBOLS), (decl, N.EXPORTED_SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (vmas_\w+)", out))
    missing = set(decl) - exported
    assert not missing, missing


def test_struct_sizes_match_header_compilation():
    # compile a tiny C probe of the header with gcc and compare sizeof() of every struct
    probe = r'''
#include <stdio.h>
#include "vmas_mi355x.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(VmasEntityDesc), sizeof(VmasPairDesc),
    sizeof(VmasJointDesc), sizeof(VmasWorldConfig), sizeof(VmasEntityIO), sizeof(VmasAgentIO), sizeof(VmasJointIO),
    sizeof(VmasStepIO), sizeof(VmasRayTarget), sizeof(VmasShapeRef), sizeof(VmasActionRef), sizeof(int),
    sizeof(VmasActionApplyRef), sizeof(VmasUniformColumn), sizeof(VmasVec), sizeof(VmasBalanceIO),
    sizeof(VmasFlockingIO), sizeof(VmasCopySpan), sizeof(VmasTransportIO), sizeof(VmasDiscoveryIO),
    sizeof(VmasSpawnTargetsIO), sizeof(VmasGradIO));
  return 0; }
'''
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        src = Path(d) / "probe.c"
        src.write_text(probe)
        exe = Path(d) / "probe"
        subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
        sizes = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()))
    py = [ctypes.sizeof(N.VmasEntityDesc), ctypes.sizeof(N.VmasPairDesc), ctypes.sizeof(N.VmasJointDesc),
          ctypes.sizeof(N.VmasWorldConfig), N.ENTITY_IO_DTYPE.itemsize, N.AGENT_IO_DTYPE.itemsize,
          N.JOINT_IO_DTYPE.itemsize, ctypes.sizeof(N.VmasStepIO), N.RAY_TARGET_DTYPE.itemsize,
          ctypes.sizeof(N.VmasShapeRef), N.ACTION_REF_DTYPE.itemsize, 4, N.ACTION_APPLY_REF_DTYPE.itemsize,
          N.UNIFORM_COLUMN_DTYPE.itemsize, ctypes.sizeof(N.VmasVec), ctypes.sizeof(N.VmasBalanceIO),
          ctypes.sizeof(N.VmasFlockingIO), ctypes.sizeof(N.VmasCopySpan), ctypes.sizeof(N.VmasTransportIO),
          ctypes.sizeof(N.VmasDiscoveryIO), ctypes.sizeof(N.VmasSpawnTargetsIO), ctypes.sizeof(N.VmasGradIO)]
    assert sizes == py
    assert N.COPY_SPAN_DTYPE.itemsize == ctypes.sizeof(N.VmasCopySpan)


def test_invalid_arguments_return_errors_not_crashes():
    lib = N.load_library()
    h = ctypes.c_void_p()
    assert lib.vmas_world_create(None, None, None, None, ctypes.byref(h)) == -1
    assert b"null" in lib.vmas_last_error()
    assert lib.vmas_world_step(None, None, None, None) == -1


def test_host_extension_loads():
    """The _vmas_host torch extension (csrc/vmas_host.cpp: the host half of a graph-mode step)
    loads next to the library and carries the library's ABI version (no GPU call is made)."""
    h = N.load_host()
    assert h.ABI_VERSION == N.VMAS_ABI_VERSION
    assert hasattr(h, "OutputAlloc") and hasattr(h, "UniformDraw")
    assert N.fn_addr("vmas_copy_spans") and N.fn_addr("vmas_uniform_columns")
    import torch

    ts = [torch.zeros(3), torch.zeros(2)]
    ts[1].add_(1)
    assert h.versions(ts) == (0, 1)
