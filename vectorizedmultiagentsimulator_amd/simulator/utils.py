# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Constants and helpers of the simulator surface (restates vmas/simulator/utils.py).

Physical constants are the reference's (utils.py:27-34).  ``TorchUtils`` keeps the reference's
tensor helpers for scenario code; the physics step itself does not use them (it runs in the
native engine, see ``_engine.py``).
"""
from __future__ import annotations

import ctypes
import typing
import warnings
from abc import ABC, abstractmethod
from enum import Enum
from typing import Dict, List, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor

X = 0
Y = 1
Z = 2
ALPHABET = "ABCDEFGHIJKLMNOPQRSTUVWXYZ"
VIEWER_DEFAULT_ZOOM = 1.2
INITIAL_VIEWER_SIZE = (700, 700)
LINE_MIN_DIST = 4 / 6e2
COLLISION_FORCE = 100
JOINT_FORCE = 130
TORQUE_CONSTRAINT_FORCE = 1

DRAG = 0.25
LINEAR_FRICTION = 0.0
ANGULAR_FRICTION = 0.0

DEVICE_TYPING = Union[torch.device, str, int]

AGENT_OBS_TYPE = Union[Tensor, Dict[str, Tensor]]
AGENT_INFO_TYPE = Dict[str, Tensor]
AGENT_REWARD_TYPE = Tensor

OBS_TYPE = Union[List[AGENT_OBS_TYPE], Dict[str, AGENT_OBS_TYPE]]
INFO_TYPE = Union[List[AGENT_INFO_TYPE], Dict[str, AGENT_INFO_TYPE]]
REWARD_TYPE = Union[List[AGENT_REWARD_TYPE], Dict[str, AGENT_REWARD_TYPE]]
DONE_TYPE = Tensor


class Color(Enum):
    # utils.py:49-61 defines YELLOW twice, which makes the reference's Enum raise at import;
    # the first definition is kept here.
    YELLOW = (0.75, 0.75, 0.25)
    RED = (0.75, 0.25, 0.25)
    GREEN = (0.25, 0.75, 0.25)
    BLUE = (0.25, 0.25, 0.75)
    LIGHT_GREEN = (0.45, 0.95, 0.45)
    WHITE = (0.75, 0.75, 0.75)
    GRAY = (0.25, 0.25, 0.25)
    BLACK = (0.15, 0.15, 0.15)
    ORANGE = (1.00, 0.50, 0)
    PINK = (0.97, 0.51, 0.75)
    PURPLE = (0.60, 0.31, 0.64)


def override(cls):
    """Decorator documenting a method override (checks that the name exists on ``cls``)."""

    def check_override(method):
        if method.__name__ not in dir(cls):
            raise NameError(f"{method} does not override any method of {cls}")
        return method

    return check_override


class Observable:
    def __init__(self):
        self._observers = []

    def subscribe(self, observer):
        self._observers.append(observer)

    def notify_observers(self, *args, **kwargs):
        for obs in self._observers:
            obs.notify(self, *args, **kwargs)

    def unsubscribe(self, observer):
        self._observers.remove(observer)


class Observer(ABC):
    @abstractmethod
    def notify(self, observable, *args, **kwargs):
        raise NotImplementedError


def extract_nested_with_index(data: Union[Tensor, Dict[str, Tensor]], index: int):
    if isinstance(data, Tensor):
        return data[index]
    if isinstance(data, Dict):
        return {k: extract_nested_with_index(v, index) for k, v in data.items()}
    raise NotImplementedError(f"Invalid type of data {data}")


class TorchUtils:
    @staticmethod
    def clamp_with_norm(tensor: Tensor, max_norm: float):
        norm = torch.linalg.vector_norm(tensor, dim=-1)
        new_tensor = (tensor / norm.unsqueeze(-1)) * max_norm
        cond = (norm > max_norm).unsqueeze(-1).expand(tensor.shape)
        return torch.where(cond, new_tensor, tensor)

    @staticmethod
    def rotate_vector(vector: Tensor, angle: Tensor):
        if len(angle.shape) == len(vector.shape):
            angle = angle.squeeze(-1)
        assert vector.shape[:-1] == angle.shape
        assert vector.shape[-1] == 2
        cos = torch.cos(angle)
        sin = torch.sin(angle)
        return torch.stack(
            [vector[..., X] * cos - vector[..., Y] * sin, vector[..., X] * sin + vector[..., Y] * cos],
            dim=-1,
        )

    @staticmethod
    def cross(vector_a: Tensor, vector_b: Tensor):
        return (vector_a[..., X] * vector_b[..., Y] - vector_a[..., Y] * vector_b[..., X]).unsqueeze(-1)

    @staticmethod
    def compute_torque(f: Tensor, r: Tensor) -> Tensor:
        return TorchUtils.cross(r, f)

    @staticmethod
    def to_numpy(data):
        if isinstance(data, Tensor):
            return data.cpu().detach().numpy()
        if isinstance(data, Dict):
            return {k: TorchUtils.to_numpy(v) for k, v in data.items()}
        if isinstance(data, Sequence):
            return [TorchUtils.to_numpy(v) for v in data]
        raise NotImplementedError(f"Invalid type of data {data}")

    @staticmethod
    def recursive_clone(value):
        if isinstance(value, Tensor):
            return value.clone()
        return {k: TorchUtils.recursive_clone(v) for k, v in value.items()}

    @staticmethod
    def recursive_require_grad_(value):
        if isinstance(value, Tensor) and torch.is_floating_point(value):
            value.requires_grad_(True)
        elif isinstance(value, Dict):
            for v in value.values():
                TorchUtils.recursive_require_grad_(v)
        else:
            for v in value:
                TorchUtils.recursive_require_grad_(v)

    @staticmethod
    def where_from_index(env_index, new_value, old_value):
        mask = torch.zeros_like(old_value, dtype=torch.bool, device=old_value.device)
        mask[env_index] = True
        return torch.where(mask, new_value, old_value)


# tries consumed by the last find_random_pos_for_entity call of a given shape
_SPAWN_HINT: Dict[tuple, int] = {}


class ScenarioUtils:
    """Reset-time helpers (utils.py:239-330)."""

    @staticmethod
    def spawn_entities_randomly(
        entities,
        world,
        env_index: int,
        min_dist_between_entities: float,
        x_bounds: Tuple[int, int],
        y_bounds: Tuple[int, int],
        occupied_positions: Tensor = None,
        disable_warn: bool = False,
    ):
        batch_size = world.batch_dim if env_index is None else 1
        if occupied_positions is None:
            occupied_positions = torch.zeros((batch_size, 0, world.dim_p), device=world.device)
        for entity in entities:
            pos = ScenarioUtils.find_random_pos_for_entity(
                occupied_positions, env_index, world, min_dist_between_entities, x_bounds, y_bounds,
                disable_warn,
            )
            occupied_positions = torch.cat([occupied_positions, pos], dim=1)
            entity.set_pos(pos.squeeze(1), batch_index=env_index)

    @staticmethod
    def find_random_pos_for_entity(
        occupied_positions: Tensor,
        env_index: int,
        world,
        min_dist_between_entities: float,
        x_bounds: Tuple[int, int],
        y_bounds: Tuple[int, int],
        disable_warn: bool = False,
    ):
        """Rejection sampling of utils.py:272-319 with the same random numbers and the same
        generator consumption, resolved natively (``vmas_spawn_resolve``).

        The reference draws a [B,1,2] proposal per try (x then y), replaces the positions of the
        envs that overlap an occupied position (torch.cdist < min_dist), and stops at the first
        try where no env overlaps; each env thus keeps its first non-overlapping candidate and the
        loop consumes 1 try (all envs accept try 0) or max accepted index + 2 tries.  Here the
        tries are drawn with the reference's uniform_ calls in batches, one native call per batch
        finds every env's first non-overlapping candidate (one sync per batch instead of one per
        try), and the generator is rewound to the state after exactly the reference's tries.
        """
        sink = getattr(world, "_hole_sink", None)
        if sink is not None:  # a graph-mode capture: this loop waits on the device, so it stays on the host
            return sink(ScenarioUtils._find_random_pos_native,
                        (occupied_positions, env_index, world, min_dist_between_entities, x_bounds, y_bounds,
                         disable_warn))
        return ScenarioUtils._find_random_pos_native(occupied_positions, env_index, world, min_dist_between_entities,
                                                     x_bounds, y_bounds, disable_warn)

    @staticmethod
    def _find_random_pos_native(occupied_positions, env_index, world, min_dist_between_entities, x_bounds, y_bounds,
                                disable_warn=False, out: Tensor = None):
        """find_random_pos_for_entity's body; ``out`` (a replayed graph-mode step) receives the
        positions in place of a new tensor."""
        batch_size = world.batch_dim if env_index is None else 1
        dev = torch.device(world.device)

        def draw(shape_x, out_x=None, out_y=None):
            x = torch.empty(shape_x, device=dev, dtype=torch.float32) if out_x is None else out_x
            y = torch.empty(shape_x, device=dev, dtype=torch.float32) if out_y is None else out_y
            return x.uniform_(*x_bounds), y.uniform_(*y_bounds)

        if occupied_positions.shape[1] == 0:
            x, y = draw((batch_size, 1, 1))
            if out is not None:
                return torch.cat([x, y], dim=2, out=out)
            return torch.cat([x, y], dim=2)

        from .. import _native as N

        lib = N.load_library()
        if dev.type == "cuda":
            dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
            gen = torch.cuda.default_generators[dev_index]
            stream = torch.cuda.current_stream(dev_index).cuda_stream
        else:
            dev_index, gen, stream = -1, torch.default_generator, None
        occ = occupied_positions.detach()
        if occ.dtype != torch.float32:
            occ = occ.float()
        pos = torch.empty((batch_size, 1, 2), device=dev, dtype=torch.float32) if out is None else out
        resolved = torch.full((batch_size,), -1, device=dev, dtype=torch.int32)
        states = []  # generator state after each try, to rewind to the reference's consumption
        # On a GPU the tries of a batch are drawn in one launch (vmas_uniform_columns: the same
        # numbers and generator advance as their uniform_ calls, probed per device and batch);
        # the rewind is then an offset: start + tries * (offset advance per try).
        fused = None
        if dev.type == "cuda":
            from .environment import _uniform

            m = _uniform.mode(torch.device("cuda", dev_index), batch_size)
            if m is not None:
                f32 = lambda v: float(np.float32(v))  # noqa: E731 -- torch casts the bounds to float
                fused = (m, gen.get_offset(), f32(x_bounds[0]), f32(x_bounds[1]), f32(y_bounds[0]), f32(y_bounds[1]))
        drawn = 0
        # first batch sized from the last consumption at this call shape (over-drawn tries are
        # rewound, so the size only trades draws for syncs)
        key = (batch_size, occ.shape[1], float(min_dist_between_entities), tuple(x_bounds), tuple(y_bounds))
        first, n = 0, min(64, max(4, _SPAWN_HINT.get(key, 6) + 2))
        mx, un = N._i32(0), N._i32(0)
        while True:
            cand = torch.empty((n, 2, batch_size), device=dev, dtype=torch.float32)
            if fused is not None:
                m, _, x0, x1, y0, y1 = fused
                base = cand.data_ptr()
                for k0 in range(0, n, 16):  # <= 32 columns per launch
                    k1 = min(n, k0 + 16)
                    cols = np.zeros(2 * (k1 - k0), dtype=N.UNIFORM_COLUMN_DTYPE)
                    for k in range(k0, k1):
                        j = 2 * (k - k0)
                        cols[j] = (base + 4 * (2 * k) * batch_size, 1, x0, x1, 0, 0, 0, 0, 0, 0, 0)
                        cols[j + 1] = (base + 4 * (2 * k + 1) * batch_size, 1, y0, y1, 0, 0, 0, 0, 0, 0, 0)
                    _uniform.launch(dev_index, batch_size, cols, m, gen)
            else:
                for k in range(n):
                    draw(None, cand[k, 0], cand[k, 1])
                    states.append(gen.get_state())
            drawn += n
            N.check_aux(lib.vmas_spawn_resolve(
                dev_index, batch_size, occ.data_ptr(), occ.shape[1], occ.stride(0), occ.stride(1), occ.stride(2),
                cand.data_ptr(), first, n, float(torch.tensor(min_dist_between_entities, dtype=torch.float32)),
                pos.data_ptr(), resolved.data_ptr(), ctypes.byref(mx), ctypes.byref(un), stream),
                "vmas_spawn_resolve")
            if un.value == 0:
                break
            first += n
            n = min(2 * n, 64)
            if first > 50_000 and not disable_warn:
                warnings.warn(
                    "It is taking many iterations to spawn the entity, make sure the bounds or "
                    "the min_dist_between_entities are not too tight to fit all entities."
                    "You can disable this warning by setting disable_warn=True"
                )
        consumed = 1 if mx.value == 0 else mx.value + 2
        _SPAWN_HINT[key] = consumed
        if fused is not None:
            start = fused[1]
            per_try = (gen.get_offset() - start) // drawn
            gen.set_offset(start + min(consumed, drawn) * per_try)
            if consumed > drawn:  # the reference's final (unused) proposal lies just past the last batch
                draw((batch_size, 1, 1))
        elif consumed <= len(states):
            gen.set_state(states[consumed - 1])
        else:  # the reference's final (unused) proposal lies just past the last batch
            draw((batch_size, 1, 1))
        return pos

    @staticmethod
    def check_kwargs_consumed(dictionary_of_kwargs: Dict, warn: bool = True):
        if len(dictionary_of_kwargs) > 0:
            message = f"Scenario kwargs: {dictionary_of_kwargs} passed but not used by the scenario."
            if warn:
                warnings.warn(message + " This will turn into an error in future versions.")
            else:
                raise ValueError(message)
