# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Minimal action/observation spaces.

The reference builds its spaces with ``gym.spaces`` (environment.py:13).  Neither gym nor
gymnasium is installed in this image, so when they are absent these small classes provide the
same constructor arguments and attributes the simulator and its tests use (``shape``, ``low``,
``high``, ``n``, ``nvec``, ``spaces``, ``contains``/``in``, ``sample``).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

try:  # prefer the real thing when it exists
    from gym import spaces as _gym_spaces  # type: ignore
except Exception:  # pragma: no cover - depends on the image
    try:
        from gymnasium import spaces as _gym_spaces  # type: ignore
    except Exception:
        _gym_spaces = None


class Space:
    def __contains__(self, x) -> bool:
        return self.contains(x)


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.ndim(low) else np.shape(high)
        self.shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def sample(self):
        low = np.where(np.isfinite(self.low), self.low, -1.0)
        high = np.where(np.isfinite(self.high), self.high, 1.0)
        return np.random.uniform(low, high).astype(self.dtype)

    def __repr__(self):
        return f"Box({self.low.min() if self.low.size else ''}, {self.high.max() if self.high.size else ''}, {self.shape}, {self.dtype})"


class Discrete(Space):
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()

    def contains(self, x) -> bool:
        x = np.asarray(x)
        if x.size != 1 or not np.issubdtype(x.dtype, np.integer):
            return False
        return 0 <= int(x) < self.n

    def sample(self):
        return np.random.randint(self.n)

    def __repr__(self):
        return f"Discrete({self.n})"


class MultiDiscrete(Space):
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return (
            x.shape == self.shape
            and np.issubdtype(x.dtype, np.integer)
            and bool(np.all(x >= 0) and np.all(x < self.nvec))
        )

    def sample(self):
        return (np.random.random(self.nvec.shape) * self.nvec).astype(np.int64)

    def __repr__(self):
        return f"MultiDiscrete({self.nvec})"


class Tuple(Space):
    def __init__(self, spaces):
        self.spaces = tuple(spaces)

    def contains(self, x) -> bool:
        return len(x) == len(self.spaces) and all(s.contains(v) for s, v in zip(self.spaces, x))

    def __getitem__(self, i):
        return self.spaces[i]

    def __len__(self):
        return len(self.spaces)

    def sample(self):
        return tuple(s.sample() for s in self.spaces)


class Dict(Space):
    def __init__(self, spaces):
        self.spaces = OrderedDict(spaces)

    def contains(self, x) -> bool:
        return set(x.keys()) == set(self.spaces.keys()) and all(
            self.spaces[k].contains(v) for k, v in x.items()
        )

    def __getitem__(self, k):
        return self.spaces[k]

    def sample(self):
        return OrderedDict((k, s.sample()) for k, s in self.spaces.items())


if _gym_spaces is not None:  # pragma: no cover
    Box, Discrete, MultiDiscrete, Tuple, Dict = (  # noqa: F811
        _gym_spaces.Box,
        _gym_spaces.Discrete,
        _gym_spaces.MultiDiscrete,
        _gym_spaces.Tuple,
        _gym_spaces.Dict,
    )
