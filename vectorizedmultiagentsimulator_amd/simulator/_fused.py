"""Host side of the fused scenario programs (csrc/vmas_scenarios.hip).

A benchmark scenario restated in ``scenarios/`` computes its per-step rewards / observations /
dones with one native launch on GPU worlds instead of the reference's eager tensor program
(~37 kernels per balance step).  The scenario keeps the reference's attributes and return
values; this module holds what every fused scenario needs:

* ``enabled(world)``: GPU world and ``VMAS_FUSED_SCENARIOS`` not "0" (the torch program
  otherwise -- CPU worlds always run it);
* ``vec`` / ``ref``: tensors and entities as the ABI's ``VmasVec`` / ``VmasShapeRef``;
* ``state_key``: identity + version counters of the tensors a cached result was computed from.
  A program computes the outputs of every agent in one launch at the first agent's call; the
  other agents' calls return the cached tensors only while every input is the same tensor
  object with the same version counter (the reference recomputes per call, so any change
  between the calls -- a user's in-place edit, a re-bound state -- recomputes here too).
"""
from __future__ import annotations

import ctypes
import os

import torch

from .. import _native as N

_ON = os.environ.get("VMAS_FUSED_SCENARIOS", "1") != "0"
# The programs' LIDAR: fast (default; the direct ray-sphere form, within the LIDAR parity
# tolerance of the oracle, tests/test_fused.py) or, with VMAS_FUSED_EXACT_LIDAR=1, bit-identical
# to World.cast_rays (k_cast_rays) and so to the scenario's torch program.
EXACT_LIDAR = os.environ.get("VMAS_FUSED_EXACT_LIDAR", "0") == "1"


_OFF_DEPTH = [0]


def enabled(world) -> bool:
    if not _ON or _OFF_DEPTH[0] or torch.device(world.device).type != "cuda":
        return False
    # autograd (Environment(grad_enabled=True)): the programs have no backward
    return not (getattr(world, "_grad_enabled", False) and torch.is_grad_enabled())


class disabled:
    """Context: the scenario programs run as torch ops (a fused program's fallback)."""

    def __enter__(self):
        _OFF_DEPTH[0] += 1

    def __exit__(self, *exc):
        _OFF_DEPTH[0] -= 1


def device_index(world) -> int:
    dev = torch.device(world.device)
    return dev.index if dev.index is not None else torch.cuda.current_device()


def stream(world):
    return N.stream_ptr(device_index(world))


def f32(t: torch.Tensor, dev) -> torch.Tensor:
    if t.dtype is not torch.float32 or t.device != dev:
        t = t.to(device=dev, dtype=torch.float32)
    return t


def vec(t: torch.Tensor, keep: list) -> "N.VmasVec":
    """A [B, 2] / [B, 1] / [B] fp32 device tensor as a VmasVec (kept alive in ``keep``)."""
    keep.append(t)
    v = N.VmasVec()
    v.p = t.data_ptr()
    v.s0 = t.stride(0)
    v.s1 = t.stride(1) if t.dim() > 1 else 0
    return v


def ref(world, entity, keep: list, slot: int = 0) -> "N.VmasShapeRef":
    """Shape + pos/rot of an entity (the distance queries' VmasShapeRef)."""
    dev = torch.device(world.device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return world.engine._ref(entity, dev, keep, slot)


def state_key(tensors) -> tuple:
    return tuple((id(t), t.data_ptr(), t._version) for t in tensors)


def bump_version(t: torch.Tensor) -> None:
    """A kernel wrote ``t`` in place through a raw pointer: advance its version counter as the
    reference's in-place torch op would (graph mode finds in-place writes by version)."""
    torch.autograd.graph.increment_version(t)


_ORDER_CACHE = {}


def reduce_order(dev: torch.device, n: int):
    """The summation order of torch's .mean(-1) over a contiguous [B, n] fp32 tensor on this
    device, as the accumulator count of the fused kernels' ordered_sum (vmas_scenarios.hip):
    acc strided accumulators combined by an adjacent-pair tree.  Probed once per (device, n)
    against torch itself on random values of mixed magnitude (tools/probe_mean_order.py: on
    MI355X / ROCm 7.2 the largest power of two <= n); None if no count reproduces it bit for
    bit (the scenario then keeps its torch program)."""
    key = (str(dev), n)
    if key in _ORDER_CACHE:
        return _ORDER_CACHE[key]
    g = torch.Generator(device="cpu").manual_seed(1234 + n)
    x = (torch.rand(4096, n, generator=g) * torch.exp2(torch.randint(-12, 12, (4096, n), generator=g).float()))
    x = x.to(dev).contiguous()
    ref = x.mean(-1)
    cols = [x[:, i] for i in range(n)]
    found = None
    acc = 1
    while acc <= min(n, N.VMAS_FLOCK_MAX_AGENTS):
        y = []
        for i in range(acc):
            a = cols[i]
            for j in range(i + acc, n, acc):
                a = a + cols[j]
            y.append(a)
        w = 1
        while w < len(y):
            for i in range(0, len(y) - w, 2 * w):
                y[i] = y[i] + y[i + w]
            w *= 2
        if torch.equal(y[0] * (1.0 / n), ref):
            found = acc
            break
        acc *= 2
    _ORDER_CACHE[key] = found
    return found


def ray_target(world, e, keep: list, dev) -> "N.VmasRayTarget":
    """An entity as a VmasRayTarget (shape + state pointers), as World.cast_rays tables it."""
    from ._engine import _f32, _shape_code, _shape_dims

    code = _shape_code(e.shape)
    dims = _shape_dims(e.shape, code)
    r = N.VmasRayTarget()
    r.shape = code
    if code == N.VMAS_SPHERE:
        r.radius = _f32(dims[0])
    else:
        r.length = _f32(dims[0])
        r.width = _f32(dims[1]) if code == N.VMAS_BOX else 0.0
    p, rot = f32(e.state.pos, dev), f32(e.state.rot, dev)
    keep += [p, rot]
    r.pos, r.rot = p.data_ptr(), rot.data_ptr()
    r.pos_s0, r.pos_s1, r.rot_s0 = p.stride(0), p.stride(1), rot.stride(0)
    return r


def direct_outputs(world, specs):
    """The step outputs of one fused launch during a graph-mode capture (StepGraph's
    DirectOutputs): ``specs`` per category (obs, rewards, done) None or (dtype, member shape, n
    members).  Returns (the launch's out_delta address, per category its n member tensors -- views
    of one buffer whose replays the graph relocates to fresh tensors -- or None).  Outside a
    capture (None, [None, None, None]): the scenario allocates its outputs as before."""
    d = getattr(world, "_direct_out", None)
    if d is None:
        return None, [None, None, None]
    return d.launch(specs)


def check(rc: int, what: str) -> None:
    N.check_aux(rc, what)


def lib():
    return N.load_library()
