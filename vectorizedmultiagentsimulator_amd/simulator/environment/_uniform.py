"""Many torch ``uniform_`` calls in one native launch (``vmas_uniform_columns``), with the same
numbers and the same generator advance.

The reference draws random-action columns (environment.py:524-606) and spawn proposals
(utils.py:272-319) with one ``uniform_`` call per [B] column: on ROCm one philox kernel each.
``vmas_uniform_columns`` reproduces PyTorch's distribution kernel (grid, philox subsequences and
offsets, float mapping) for many columns at once.  Two float roundings of that kernel may or may
not be fused depending on how PyTorch was compiled, so the library has a mode for each and
``mode()`` probes, once per (device, batch), which one equals torch bit for bit -- numbers and
generator advance -- or returns None (callers then draw with torch).
"""
from __future__ import annotations

import ctypes
from typing import Any, Dict, Optional

import numpy as np
import torch

MODES: Dict[Any, Optional[int]] = {}

# bounds of the probe's columns (f32-exact values, as torch casts them)
_PROBE_BOUNDS = [(-0.7, 0.7), (-1.0, 1.0), (0.0, 1.0), (-0.30000001192092896, 0.30000001192092896)]


def _native():
    from ... import _native as N

    return N


def launch(idx: int, B: int, cols: np.ndarray, mode: int, gen: torch.Generator, cols_addr: Optional[int] = None) -> None:
    """Draws len(cols) columns of B floats at the generator's current (seed, offset) and advances
    the generator's offset as the equivalent uniform_ calls would (cols: UNIFORM_COLUMN_DTYPE
    rows with out / stride / from_ / to set; cols_addr: its address, when the caller has it)."""
    N = _native()
    inc = ctypes.c_uint64(0)
    stream = N.stream_ptr(idx)
    off = gen.get_offset()
    N.check_aux(N.load_library().vmas_uniform_columns(idx, B, cols.ctypes.data if cols_addr is None else cols_addr,
                                                       len(cols), gen.initial_seed(), off, mode, ctypes.byref(inc),
                                                       stream),
                "vmas_uniform_columns")
    gen.set_offset(off + inc.value)


def mode(device: torch.device, B: int) -> Optional[int]:
    """The mode whose draws equal per-column torch uniform_ calls on [B] tensors, bit for bit,
    with the same generator advance; None if no mode does.  The device generator is saved and
    restored around the probe."""
    key = (str(device), B)
    if key in MODES:
        return MODES[key]
    N = _native()
    idx = device.index if device.index is not None else torch.cuda.current_device()
    gen = torch.cuda.default_generators[idx]
    saved = gen.get_state()
    found = None
    try:
        ref = [torch.empty(B, device=device, dtype=torch.float32).uniform_(lo, hi) for lo, hi in _PROBE_BOUNDS]
        after = gen.get_state()
        for m in (3, 0, 1, 2):
            gen.set_state(saved)
            out = torch.empty(B, len(_PROBE_BOUNDS), device=device, dtype=torch.float32)
            cols = np.zeros(len(_PROBE_BOUNDS), dtype=N.UNIFORM_COLUMN_DTYPE)
            for i, (lo, hi) in enumerate(_PROBE_BOUNDS):
                cols[i] = (out.data_ptr() + 4 * i, len(_PROBE_BOUNDS), lo, hi, 0, 0, 0, 0, 0, 0, 0)
            launch(idx, B, cols, m, gen)
            if all(torch.equal(out[:, i], r) for i, r in enumerate(ref)) and torch.equal(gen.get_state(), after):
                found = m
                break
    finally:
        gen.set_state(saved)
    MODES[key] = found
    return found
