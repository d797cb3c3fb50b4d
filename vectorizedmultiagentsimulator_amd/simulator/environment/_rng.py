"""Exact save/restore of numpy's and Python's process-global RNGs for ``local_seed``.

The reference swaps the simulator's RNG states in and out around every ``Environment`` call
(environment.py:30-46) with ``np.random.get_state()`` / ``set_state()``.  Those copy the 624-word
MT19937 key element by element (~40 us each, four per call), the largest host cost of a step.

The same state is two pieces:
  * the MT19937 key + position, reachable through the bit generator's public ctypes interface
    (``bit_generator.ctypes.state_address`` -> ``{uint32_t key[624]; int pos;}``): one memmove;
  * the legacy gaussian cache (``has_gauss``, ``gauss``) kept inside the RandomState object.
    It has no public accessor, so its offset is found once by probing with ``set_state`` and
    validated with ``get_state`` round trips; if anything does not match, every snapshot falls
    back to ``get_state`` / ``set_state``.
Both paths save and restore exactly what ``get_state`` / ``set_state`` do (tests/test_rng.py
compares every draw against the reference's swap, gaussian cache included).

Python's ``random.getstate()`` / ``setstate()`` build and parse a 625-int tuple (~14 + 6 us).
``PythonGlobalRng`` does the same swap with one memmove of the C object's ``{int index; uint32_t
state[624]}`` (located once by a probe, validated by round trips) plus the ``gauss_next``
attribute; tuples from ``getstate()`` are still accepted by ``restore``.
"""
from __future__ import annotations

import ctypes
import sys

import numpy as np

_MT_BYTES = 624 * 4 + 4  # uint32 key[624] + int pos


class NumpyGlobalRng:
    def __init__(self):
        self.rs = np.random.mtrand._rand
        self.fast = False
        try:
            self.bg = self.rs._bit_generator
            self.mt = self.bg.ctypes.state_address
            self.gauss_at = self._find_gauss()
            self.fast = self.gauss_at is not None and self._validate()
        except Exception:
            self.fast = False

    # -- probing ----------------------------------------------------------------------------------
    def _read(self, off, ctype):
        return ctype.from_address(id(self.rs) + off).value

    def _find_gauss(self):
        st = np.random.get_state()
        try:
            size = sys.getsizeof(self.rs)
            cand = None
            for has, g in ((1, 1.2345678901234567), (0, -7.654321e-3), (1, 3.0e-300)):
                np.random.set_state((st[0], st[1], st[2], has, g))
                hits = {o for o in range(16, size - 16, 4)
                        if self._read(o, ctypes.c_int32) == has and self._read(o + 8, ctypes.c_double) == g}
                cand = hits if cand is None else (cand & hits)
            return min(cand) if cand and len(cand) == 1 else None
        finally:
            np.random.set_state(st)

    def _validate(self) -> bool:
        st = np.random.get_state()
        try:
            for has, g in ((1, 0.5), (0, 0.0), (1, -2.25)):
                snap = self.snapshot()
                np.random.set_state((st[0], st[1], st[2], has, g))
                if self._gauss() != (has, g):
                    return False
                self.restore(snap)
                if tuple(np.random.get_state()[3:]) != tuple(st[3:]) or not np.array_equal(
                        np.random.get_state()[1], st[1]):
                    return False
            return True
        finally:
            np.random.set_state(st)

    def _gauss(self):
        return self._read(self.gauss_at, ctypes.c_int32), self._read(self.gauss_at + 8, ctypes.c_double)

    # -- snapshot / restore --------------------------------------------------------------------
    def snapshot(self):
        """Current global numpy RNG state (opaque; pass back to restore)."""
        if not self.fast:
            return np.random.get_state()
        buf = ctypes.create_string_buffer(_MT_BYTES)
        ctypes.memmove(buf, self.mt, _MT_BYTES)
        return buf, self._gauss()

    def restore(self, snap) -> None:
        """Make ``snap`` (from snapshot(), or a np.random.get_state() tuple) the global state."""
        if isinstance(snap, tuple) and len(snap) == 5:  # legacy get_state() tuple
            np.random.set_state(snap)
            return
        buf, (has, g) = snap
        ctypes.memmove(self.mt, buf, _MT_BYTES)
        base = id(self.rs) + self.gauss_at
        ctypes.c_int32.from_address(base).value = has
        ctypes.c_double.from_address(base + 8).value = g


class PythonGlobalRng:
    """The same for ``random``'s module-level generator (``random._inst``)."""

    _WORDS = 624

    def __init__(self):
        import random

        self.random = random
        self.inst = random._inst
        self.fast = False
        try:
            self.off = self._find_state()
            self.fast = self.off is not None and self._validate()
        except Exception:
            self.fast = False

    def _find_state(self):
        r = self.random
        st = r.getstate()
        try:
            key = tuple((0x9E3779B9 * (i + 7) + 0x7F4A7C15) & 0xFFFFFFFF for i in range(self._WORDS))
            r.setstate((st[0], key + (self._WORDS,), None))
            pattern = np.array(key, dtype=np.uint32).tobytes()
            mem = ctypes.string_at(id(self.inst), self.inst.__sizeof__())  # the object, no GC header
            at = mem.find(pattern)
            if at < 4 or mem.find(pattern, at + 1) != -1:
                return None
            if ctypes.c_int32.from_address(id(self.inst) + at - 4).value != self._WORDS:
                return None
            return at - 4  # {int index; uint32_t state[624]}
        finally:
            r.setstate(st)

    def _validate(self) -> bool:
        r = self.random
        st = r.getstate()
        try:
            for seed, n, g in ((1, 3, None), (2, 0, 0.25), (3, 700, -1.5)):
                r.seed(seed)
                for _ in range(n):
                    r.random()
                self.inst.gauss_next = g
                snap = self.snapshot()
                want = r.getstate()
                r.seed(seed + 100)
                r.random()
                self.restore(snap)
                if r.getstate() != want:
                    return False
            return True
        finally:
            r.setstate(st)

    def snapshot(self):
        if not self.fast:
            return self.random.getstate()
        buf = ctypes.create_string_buffer(4 + 4 * self._WORDS)
        ctypes.memmove(buf, id(self.inst) + self.off, 4 + 4 * self._WORDS)
        return buf, self.inst.gauss_next

    def restore(self, snap) -> None:
        if isinstance(snap, tuple) and len(snap) == 3:  # a random.getstate() tuple
            self.random.setstate(snap)
            return
        buf, g = snap
        ctypes.memmove(id(self.inst) + self.off, buf, 4 + 4 * self._WORDS)
        self.inst.gauss_next = g


_instance = None
_py_instance = None


def numpy_global_rng() -> NumpyGlobalRng:
    global _instance
    if _instance is None:
        _instance = NumpyGlobalRng()
    return _instance


def python_global_rng() -> PythonGlobalRng:
    global _py_instance
    if _py_instance is None:
        _py_instance = PythonGlobalRng()
    return _py_instance
