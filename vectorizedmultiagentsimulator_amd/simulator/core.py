# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Entity / World surface of the simulator (restates vmas/simulator/core.py's public API).

The classes keep the reference's names, constructor arguments, properties and side effects so
that scenario code written against ``vmas.simulator.core`` runs unchanged.  What changes is the
hot path: ``World.step`` (core.py:1971-2014), ``World.cast_rays`` / ``cast_ray``
(core.py:1627-1785) and the distance queries (core.py:1787-1968) are executed by the native
engine (``_engine.py`` -> ``libvmas_mi355x.so``: gfx950 kernels on ROCm devices, the same
arithmetic on host threads for ``device="cpu"``) instead of hundreds of PyTorch ops.
"""
from __future__ import annotations

import math
import os
import typing
from abc import ABC, abstractmethod
from typing import Callable, List, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor

from .dynamics.common import Dynamics
from .dynamics.holonomic import Holonomic
from .joints import Joint
from .sensors import Sensor
from .utils import (
    ANGULAR_FRICTION,
    COLLISION_FORCE,
    Color,
    DRAG,
    JOINT_FORCE,
    LINEAR_FRICTION,
    Observable,
    override,
    TorchUtils,
    TORQUE_CONSTRAINT_FORCE,
    X,
    Y,
)


# Version of the attributes the physics engine's static tables are built from (simulator/_engine.py
# _signature): bumped by every assignment to one of them (the __setattr__ hooks below and the
# world's add_* methods), so the engine rebuilds its per-step structure signature only after
# something it depends on was assigned (graph mode compares it every step: ~3-6 us of host time).
STATIC_VERSION = [0]
_ENTITY_STATIC = frozenset({
    "_shape", "_movable", "_rotatable", "_collide", "_collision_filter", "_mass", "_drag", "_linear_friction",
    "_angular_friction", "_max_speed", "_v_range", "_gravity", "_max_f", "_f_range", "_max_t", "_t_range",
    # (and what the environment's random-action plans depend on: environment.py _uniform_sig)
    "_action", "_silent", "action_size", "_batch_dim", "_action_script", "__class__",
})
_WORLD_STATIC = frozenset({
    "_agents", "_landmarks", "_joints", "_drag", "_linear_friction", "_angular_friction", "_x_semidim",
    "_y_semidim", "_collision_force", "_joint_force", "_torque_constraint_force", "_contact_margin", "_gravity",
    "_collidable_pairs", "_batch_dim", "_device", "export_forces", "_dim_c",
})


class TorchVectorizedObject(object):
    def __init__(self, batch_dim: int = None, device: torch.device = None):
        self._batch_dim = batch_dim
        self._device = device

    @property
    def batch_dim(self):
        return self._batch_dim

    @batch_dim.setter
    def batch_dim(self, batch_dim: int):
        assert self._batch_dim is None, "You can set batch dim only once"
        self._batch_dim = batch_dim

    @property
    def device(self):
        return self._device

    @device.setter
    def device(self, device: torch.device):
        self._device = device

    def _check_batch_index(self, batch_index: int):
        if batch_index is not None:
            assert 0 <= batch_index < self.batch_dim, (
                f"Index must be between 0 and {self.batch_dim}, got {batch_index}"
            )

    def to(self, device: torch.device):
        self.device = device
        for attr, value in self.__dict__.items():
            if isinstance(value, Tensor):
                self.__dict__[attr] = value.to(device)


# ------------------------------------------------------------------------------------------------
# shapes (core.py:84-202)
class Shape(ABC):
    @abstractmethod
    def moment_of_inertia(self, mass: float):
        raise NotImplementedError

    @abstractmethod
    def get_delta_from_anchor(self, anchor: Tuple[float, float]) -> Tuple[float, float]:
        raise NotImplementedError

    @abstractmethod
    def circumscribed_radius(self):
        raise NotImplementedError

    def get_geometry(self):
        raise NotImplementedError("rendering is not part of the MI355X engine")


class Box(Shape):
    def __setattr__(self, name, value):
        object.__setattr__(self, name, value)
        if name == "hollow":
            STATIC_VERSION[0] += 1

    def __init__(self, length: float = 0.3, width: float = 0.1, hollow: bool = False):
        super().__init__()
        assert length > 0, f"Length must be > 0, got {length}"
        assert width > 0, f"Width must be > 0, got {length}"
        self._length = length
        self._width = width
        self.hollow = hollow

    @property
    def length(self):
        return self._length

    @property
    def width(self):
        return self._width

    def get_delta_from_anchor(self, anchor):
        return anchor[X] * self.length / 2, anchor[Y] * self.width / 2

    def moment_of_inertia(self, mass: float):
        return (1 / 12) * mass * (self.length**2 + self.width**2)

    def circumscribed_radius(self):
        return math.sqrt((self.length / 2) ** 2 + (self.width / 2) ** 2)


class Sphere(Shape):
    def __init__(self, radius: float = 0.05):
        super().__init__()
        assert radius > 0, f"Radius must be > 0, got {radius}"
        self._radius = radius

    @property
    def radius(self):
        return self._radius

    def get_delta_from_anchor(self, anchor):
        # core.py:150-157 (fp32 tensor arithmetic, including its normalisation quirk)
        delta = torch.tensor([anchor[X] * self.radius, anchor[Y] * self.radius]).to(torch.float32)
        delta_norm = torch.linalg.vector_norm(delta)
        if delta_norm > self.radius:
            delta /= delta_norm * self.radius
        return tuple(delta.tolist())

    def moment_of_inertia(self, mass: float):
        return (1 / 2) * mass * self.radius**2

    def circumscribed_radius(self):
        return self.radius


class Line(Shape):
    def __init__(self, length: float = 0.5):
        super().__init__()
        assert length > 0, f"Length must be > 0, got {length}"
        self._length = length
        self._width = 2

    @property
    def length(self):
        return self._length

    @property
    def width(self):
        return self._width

    def moment_of_inertia(self, mass: float):
        return (1 / 12) * mass * (self.length**2)

    def circumscribed_radius(self):
        return self.length / 2

    def get_delta_from_anchor(self, anchor):
        return anchor[X] * self.length / 2, 0.0


# ------------------------------------------------------------------------------------------------
# state containers (core.py:205-409).  Setters keep the reference's checks and replace the
# tensor object; the engine reads whatever tensor an entity holds at step time.
def _check_state_set(obj, value: Tensor):
    assert obj._batch_dim is not None and obj._device is not None, (
        "First add an entity to the world before setting its state"
    )
    assert value.shape[0] == obj._batch_dim, (
        f"Internal state must match batch dim, got {value.shape[0]}, expected {obj._batch_dim}"
    )


class EntityState(TorchVectorizedObject):
    # graph mode: the StepGraph's _FreshState (simulator/environment/_graph.py) -- after a replay
    # the first read of a state attribute re-binds the states to fresh tensors, as the reference's
    # integration creates new ones every step (core.py:2866-2907)
    _fresh = None

    def __init__(self):
        super().__init__()
        self._pos = None
        self._vel = None
        self._rot = None
        self._ang_vel = None

    @property
    def pos(self):
        f = self._fresh
        if f is not None and f.pending:
            f.materialize()
        return self._pos

    @pos.setter
    def pos(self, pos: Tensor):
        _check_state_set(self, pos)
        if self._vel is not None:
            assert pos.shape == self._vel.shape, (
                f"Position shape must match velocity shape, got {pos.shape} expected {self._vel.shape}"
            )
        self._pos = pos.to(self._device)

    @property
    def vel(self):
        f = self._fresh
        if f is not None and f.pending:
            f.materialize()
        return self._vel

    @vel.setter
    def vel(self, vel: Tensor):
        _check_state_set(self, vel)
        if self._pos is not None:
            assert vel.shape == self._pos.shape, (
                f"Velocity shape must match position shape, got {vel.shape} expected {self._pos.shape}"
            )
        self._vel = vel.to(self._device)

    @property
    def ang_vel(self):
        f = self._fresh
        if f is not None and f.pending:
            f.materialize()
        return self._ang_vel

    @ang_vel.setter
    def ang_vel(self, ang_vel: Tensor):
        _check_state_set(self, ang_vel)
        self._ang_vel = ang_vel.to(self._device)

    @property
    def rot(self):
        f = self._fresh
        if f is not None and f.pending:
            f.materialize()
        return self._rot

    @rot.setter
    def rot(self, rot: Tensor):
        _check_state_set(self, rot)
        self._rot = rot.to(self._device)

    def _reset(self, env_index: typing.Optional[int]):
        for attr_name in ["pos", "rot", "vel", "ang_vel"]:
            attr = self.__getattribute__(attr_name)
            if attr is not None:
                if env_index is None:
                    self.__setattr__(attr_name, torch.zeros_like(attr))
                else:
                    self.__setattr__(attr_name, TorchUtils.where_from_index(env_index, 0, attr))

    def zero_grad(self):
        for attr_name in ["pos", "rot", "vel", "ang_vel"]:
            attr = self.__getattribute__(attr_name)
            if attr is not None:
                self.__setattr__(attr_name, attr.detach())

    def _spawn(self, dim_c: int, dim_p: int):
        self.pos = torch.zeros(self.batch_dim, dim_p, device=self.device, dtype=torch.float32)
        self.vel = torch.zeros(self.batch_dim, dim_p, device=self.device, dtype=torch.float32)
        self.rot = torch.zeros(self.batch_dim, 1, device=self.device, dtype=torch.float32)
        self.ang_vel = torch.zeros(self.batch_dim, 1, device=self.device, dtype=torch.float32)


class AgentState(EntityState):
    def __init__(self):
        super().__init__()
        self._c = None
        self._force = None
        self._torque = None

    @property
    def c(self):
        return self._c

    @c.setter
    def c(self, c: Tensor):
        _check_state_set(self, c)
        self._c = c.to(self._device)

    _shadow = None  # graph mode: the environment's _ActionShadow (see Action.u)

    @property
    def force(self):
        sh = self._shadow
        if sh is not None and sh.active:
            return sh.view(self._force)
        f = self._fresh
        if f is not None and f.pending:
            f.materialize()
        return self._force

    @force.setter
    def force(self, value):
        _check_state_set(self, value)
        self._force = value.to(self._device)

    @property
    def torque(self):
        f = self._fresh
        if f is not None and f.pending:
            f.materialize()
        return self._torque

    @torque.setter
    def torque(self, value):
        _check_state_set(self, value)
        self._torque = value.to(self._device)

    @override(EntityState)
    def _reset(self, env_index: typing.Optional[int]):
        for attr_name in ["c", "force", "torque"]:
            attr = self.__getattribute__(attr_name)
            if attr is not None:
                if env_index is None:
                    self.__setattr__(attr_name, torch.zeros_like(attr))
                else:
                    self.__setattr__(attr_name, TorchUtils.where_from_index(env_index, 0, attr))
        super()._reset(env_index)

    @override(EntityState)
    def zero_grad(self):
        for attr_name in ["c", "force", "torque"]:
            attr = self.__getattribute__(attr_name)
            if attr is not None:
                self.__setattr__(attr_name, attr.detach())
        super().zero_grad()

    @override(EntityState)
    def _spawn(self, dim_c: int, dim_p: int):
        if dim_c > 0:
            self.c = torch.zeros(self.batch_dim, dim_c, device=self.device, dtype=torch.float32)
        self.force = torch.zeros(self.batch_dim, dim_p, device=self.device, dtype=torch.float32)
        self.torque = torch.zeros(self.batch_dim, 1, device=self.device, dtype=torch.float32)
        super()._spawn(dim_c, dim_p)


class Action(TorchVectorizedObject):
    """Agent action container (core.py:413-533)."""

    def __setattr__(self, name, value):
        object.__setattr__(self, name, value)
        if name == "_u_range":  # (environment.py _uniform_sig)
            STATIC_VERSION[0] += 1

    def __init__(self, u_range, u_multiplier, u_noise, action_size: int):
        super().__init__()
        self._u_noise = u_noise
        self._u_range = u_range
        self._u_multiplier = u_multiplier
        self.action_size = action_size
        self._u = None
        self._c = None
        self._u_range_tensor = None
        self._u_multiplier_tensor = None
        self._u_noise_tensor = None
        for attr in (self.u_multiplier, self.u_range, self.u_noise):
            if isinstance(attr, List):
                assert len(attr) == self.action_size, (
                    "Action attributes u_... must be either a float or a list of floats"
                    " (one per action) all with same length"
                )

    # Graph mode: between a random-action draw that pre-applies its actions into the persistent
    # action buffer and the step that consumes them, u (and a holonomic agent's state.force, a view
    # of u) shows the draw's snapshot of the buffer -- the values of the last step, as the
    # reference, whose draw leaves the agents alone (environment/environment.py _ActionShadow).
    _shadow = None
    _fresh = None  # graph mode: see EntityState._fresh

    @property
    def u(self):
        sh = self._shadow
        if sh is not None and sh.active:
            return sh.view(self._u)
        f = self._fresh
        if f is not None and f.pending:
            f.materialize()
        return self._u

    @u.setter
    def u(self, u: Tensor):
        assert self._batch_dim is not None and self._device is not None, (
            "First add an agent to the world before setting its action"
        )
        assert u.shape[0] == self._batch_dim, (
            f"Action must match batch dim, got {u.shape[0]}, expected {self._batch_dim}"
        )
        self._u = u.to(self._device)

    @property
    def c(self):
        return self._c

    @c.setter
    def c(self, c: Tensor):
        assert self._batch_dim is not None and self._device is not None, (
            "First add an agent to the world before setting its action"
        )
        assert c.shape[0] == self._batch_dim, (
            f"Action must match batch dim, got {c.shape[0]}, expected {self._batch_dim}"
        )
        self._c = c.to(self._device)

    @property
    def u_range(self):
        return self._u_range

    @property
    def u_multiplier(self):
        return self._u_multiplier

    @property
    def u_noise(self):
        return self._u_noise

    @property
    def u_range_tensor(self):
        if self._u_range_tensor is None:
            self._u_range_tensor = self._to_tensor(self.u_range)
        return self._u_range_tensor

    @property
    def u_multiplier_tensor(self):
        if self._u_multiplier_tensor is None:
            self._u_multiplier_tensor = self._to_tensor(self.u_multiplier)
        return self._u_multiplier_tensor

    @property
    def u_noise_tensor(self):
        if self._u_noise_tensor is None:
            self._u_noise_tensor = self._to_tensor(self.u_noise)
        return self._u_noise_tensor

    def _to_tensor(self, value):
        return torch.tensor(
            value if isinstance(value, Sequence) else [value] * self.action_size,
            device=self.device,
            dtype=torch.float,
        )

    def _reset(self, env_index: typing.Optional[int]):
        for attr_name in ["u", "c"]:
            attr = self.__getattribute__(attr_name)
            if attr is not None:
                if env_index is None:
                    self.__setattr__(attr_name, torch.zeros_like(attr))
                else:
                    self.__setattr__(attr_name, TorchUtils.where_from_index(env_index, 0, attr))

    def zero_grad(self):
        for attr_name in ["u", "c"]:
            attr = self.__getattribute__(attr_name)
            if attr is not None:
                self.__setattr__(attr_name, attr.detach())


# ------------------------------------------------------------------------------------------------
# entities (core.py:537-1085)
class Entity(TorchVectorizedObject, Observable, ABC):
    def __setattr__(self, name, value):
        object.__setattr__(self, name, value)
        if name in _ENTITY_STATIC:
            STATIC_VERSION[0] += 1

    def __init__(
        self,
        name: str,
        movable: bool = False,
        rotatable: bool = False,
        collide: bool = True,
        density: float = 25.0,
        mass: float = 1.0,
        shape: Shape = None,
        v_range: float = None,
        max_speed: float = None,
        color=Color.GRAY,
        is_joint: bool = False,
        drag: float = None,
        linear_friction: float = None,
        angular_friction: float = None,
        gravity: typing.Union[float, Tensor] = None,
        collision_filter: Callable[["Entity"], bool] = lambda _: True,
    ):
        if shape is None:
            shape = Sphere()
        TorchVectorizedObject.__init__(self)
        Observable.__init__(self)
        self._name = name
        self._movable = movable
        self._rotatable = rotatable
        self._collide = collide
        self._density = density
        self._mass = mass
        self._max_speed = max_speed
        self._v_range = v_range
        self._color = color
        self._shape = shape
        self._is_joint = is_joint
        self._collision_filter = collision_filter
        self._state = EntityState()
        self._drag = drag
        self._linear_friction = linear_friction
        self._angular_friction = angular_friction
        if isinstance(gravity, Tensor):
            self._gravity = gravity
        else:
            self._gravity = (
                torch.tensor(gravity, device=self.device, dtype=torch.float32)
                if gravity is not None
                else gravity
            )
        self._goal = None
        self._render = None

    @TorchVectorizedObject.batch_dim.setter
    def batch_dim(self, batch_dim: int):
        TorchVectorizedObject.batch_dim.fset(self, batch_dim)
        self._state.batch_dim = batch_dim

    @property
    def is_rendering(self):
        if self._render is None:
            self.reset_render()
        return self._render

    def reset_render(self):
        self._render = torch.full((self.batch_dim,), True, device=self.device)

    def collides(self, entity: "Entity"):
        if not self.collide:
            return False
        return self._collision_filter(entity)

    @property
    def is_joint(self):
        return self._is_joint

    @property
    def mass(self):
        return self._mass

    @mass.setter
    def mass(self, mass: float):
        self._mass = mass

    @property
    def moment_of_inertia(self):
        return self.shape.moment_of_inertia(self.mass)

    @property
    def state(self):
        return self._state

    @property
    def movable(self):
        return self._movable

    @property
    def collide(self):
        return self._collide

    @property
    def shape(self):
        return self._shape

    @property
    def max_speed(self):
        return self._max_speed

    @property
    def v_range(self):
        return self._v_range

    @property
    def name(self):
        return self._name

    @property
    def rotatable(self):
        return self._rotatable

    @property
    def color(self):
        if isinstance(self._color, Color):
            return self._color.value
        return self._color

    @color.setter
    def color(self, color):
        self._color = color

    @property
    def goal(self):
        return self._goal

    @goal.setter
    def goal(self, goal: "Entity"):
        self._goal = goal

    @property
    def drag(self):
        return self._drag

    @property
    def linear_friction(self):
        return self._linear_friction

    @linear_friction.setter
    def linear_friction(self, value):
        self._linear_friction = value

    @property
    def gravity(self):
        return self._gravity

    @gravity.setter
    def gravity(self, value):
        self._gravity = value

    @property
    def angular_friction(self):
        return self._angular_friction

    @property
    def collision_filter(self):
        return self._collision_filter

    @collision_filter.setter
    def collision_filter(self, collision_filter: Callable[["Entity"], bool]):
        self._collision_filter = collision_filter

    def _spawn(self, dim_c: int, dim_p: int):
        self.state._spawn(dim_c, dim_p)

    def _reset(self, env_index: int):
        self.state._reset(env_index)

    def zero_grad(self):
        self.state.zero_grad()

    def set_pos(self, pos: Tensor, batch_index: int):
        self._set_state_property(EntityState.pos, self.state, pos, batch_index)

    def set_vel(self, vel: Tensor, batch_index: int):
        self._set_state_property(EntityState.vel, self.state, vel, batch_index)

    def set_rot(self, rot: Tensor, batch_index: int):
        self._set_state_property(EntityState.rot, self.state, rot, batch_index)

    def set_ang_vel(self, ang_vel: Tensor, batch_index: int):
        self._set_state_property(EntityState.ang_vel, self.state, ang_vel, batch_index)

    def _set_state_property(self, prop, entity: EntityState, new: Tensor, batch_index: int):
        assert self.batch_dim is not None, f"Tried to set property of {self.name} without adding it to the world"
        self._check_batch_index(batch_index)
        new = new.to(self.device)
        if batch_index is None:
            if len(new.shape) > 1 and new.shape[0] == self.batch_dim:
                prop.fset(entity, new)
            else:
                prop.fset(entity, new.repeat(self.batch_dim, 1))
        else:
            value = prop.fget(entity)
            value[batch_index] = new
        self.notify_observers()

    @override(TorchVectorizedObject)
    def to(self, device: torch.device):
        super().to(device)
        self.state.to(device)

    def render(self, env_index: int = 0):
        raise NotImplementedError("rendering is not part of the MI355X engine")


class Landmark(Entity):
    def __init__(
        self,
        name: str,
        shape: Shape = None,
        movable: bool = False,
        rotatable: bool = False,
        collide: bool = True,
        density: float = 25.0,
        mass: float = 1.0,
        v_range: float = None,
        max_speed: float = None,
        color=Color.GRAY,
        is_joint: bool = False,
        drag: float = None,
        linear_friction: float = None,
        angular_friction: float = None,
        gravity: float = None,
        collision_filter: Callable[[Entity], bool] = lambda _: True,
    ):
        super().__init__(
            name, movable, rotatable, collide, density, mass, shape, v_range, max_speed, color,
            is_joint, drag, linear_friction, angular_friction, gravity, collision_filter,
        )


def _range_proven(u, action) -> bool:
    """The scripted-action range check of core.py:978-981, ``((u / u_multiplier).abs() <=
    u_range).all()``, decided without reading u: a script that builds u from bounded functions
    (the package's flocking target: cos / sin of the step counter, |u| <= 1) tags the tensor with
    ``_vmas_abs_bound``.  fp32 division is monotone in |u|, so the check holds for every element
    when it holds at |u| = bound in every column.  Saves a device check per step and, in graph
    mode, the rollback machinery such a check needs (backups of what the step modifies in place,
    no draw made ahead)."""
    bound = getattr(u, "_vmas_abs_bound", None)
    if bound is None:
        return False
    n = u.shape[-1]
    m, r = action.u_multiplier, action.u_range
    ms = list(m) if isinstance(m, Sequence) else [m] * n
    rs = list(r) if isinstance(r, Sequence) else [r] * n
    if len(ms) != n or len(rs) != n:
        return False
    b = np.float32(bound)
    with np.errstate(divide="ignore", invalid="ignore"):
        return all(np.abs(b / np.float32(mi)) <= np.float32(ri) for mi, ri in zip(ms, rs))


class Agent(Entity):
    def __init__(
        self,
        name: str,
        shape: Shape = None,
        movable: bool = True,
        rotatable: bool = True,
        collide: bool = True,
        density: float = 25.0,
        mass: float = 1.0,
        f_range: float = None,
        max_f: float = None,
        t_range: float = None,
        max_t: float = None,
        v_range: float = None,
        max_speed: float = None,
        color=Color.BLUE,
        alpha: float = 0.5,
        obs_range: float = None,
        obs_noise: float = None,
        u_noise: Union[float, Sequence[float]] = 0.0,
        u_range: Union[float, Sequence[float]] = 1.0,
        u_multiplier: Union[float, Sequence[float]] = 1.0,
        action_script: Callable[["Agent", "World"], None] = None,
        sensors: List[Sensor] = None,
        c_noise: float = 0.0,
        silent: bool = True,
        adversary: bool = False,
        drag: float = None,
        linear_friction: float = None,
        angular_friction: float = None,
        gravity: float = None,
        collision_filter: Callable[[Entity], bool] = lambda _: True,
        render_action: bool = False,
        dynamics: Dynamics = None,
        action_size: int = None,
        discrete_action_nvec: List[int] = None,
    ):
        super().__init__(
            name, movable, rotatable, collide, density, mass, shape, v_range, max_speed, color,
            is_joint=False, drag=drag, linear_friction=linear_friction,
            angular_friction=angular_friction, gravity=gravity, collision_filter=collision_filter,
        )
        if obs_range == 0.0:
            assert sensors is None, f"Blind agent cannot have sensors, got {sensors}"
        if action_size is not None and discrete_action_nvec is not None:
            if action_size != len(discrete_action_nvec):
                raise ValueError(
                    f"action_size {action_size} is inconsistent with discrete_action_nvec {discrete_action_nvec}"
                )
        if discrete_action_nvec is not None:
            if not all(n > 1 for n in discrete_action_nvec):
                raise ValueError(
                    f"All values in discrete_action_nvec must be greater than 1, got {discrete_action_nvec}"
                )
        self._obs_range = obs_range
        self._obs_noise = obs_noise
        self._f_range = f_range
        self._max_f = max_f
        self._t_range = t_range
        self._max_t = max_t
        self._action_script = action_script
        self._sensors = []
        if sensors is not None:
            [self.add_sensor(sensor) for sensor in sensors]
        self._c_noise = c_noise
        self._silent = silent
        self._render_action = render_action
        self._adversary = adversary
        self._alpha = alpha
        self.dynamics = dynamics if dynamics is not None else Holonomic()
        if action_size is not None:
            self.action_size = action_size
        elif discrete_action_nvec is not None:
            self.action_size = len(discrete_action_nvec)
        else:
            self.action_size = self.dynamics.needed_action_size
        if discrete_action_nvec is None:
            self.discrete_action_nvec = [3] * self.action_size
        else:
            self.discrete_action_nvec = discrete_action_nvec
        self.dynamics.agent = self
        self._action = Action(
            u_range=u_range, u_multiplier=u_multiplier, u_noise=u_noise, action_size=self.action_size
        )
        self._state = AgentState()

    def add_sensor(self, sensor: Sensor):
        sensor.agent = self
        self._sensors.append(sensor)

    @Entity.batch_dim.setter
    def batch_dim(self, batch_dim: int):
        Entity.batch_dim.fset(self, batch_dim)
        self._action.batch_dim = batch_dim

    @property
    def action_script(self):
        return self._action_script

    def action_callback(self, world: "World"):
        self._action_script(self, world)
        if self._silent or world.dim_c == 0:
            assert self._action.c is None, (
                f"Agent {self.name} should not communicate but action script communicates"
            )
        assert self._action.u is not None, f"Action script of {self.name} should set u action"
        assert self._action.u.shape[1] == self.action_size, (
            f"Scripted action of agent {self.name} has wrong shape"
        )
        if _range_proven(self._action.u, self.action):
            return  # every element passes by construction: no check to run (see _range_proven)
        sink = world._assert_sink
        rsink = getattr(world, "_assert_range_sink", None)
        if sink is not None and rsink is not None and rsink(self._action.u, self.action.u_multiplier_tensor,
                                                            self.action.u_range_tensor,
                                                            f"Scripted physical action of {self.name} is out of range"):
            return  # (graph mode: the check evaluated and published by one native kernel)
        ok = ((self._action.u / self.action.u_multiplier_tensor).abs() <= self.action.u_range_tensor).all()
        if sink is None:
            assert ok, f"Scripted physical action of {self.name} is out of range"
        else:  # graph mode: checked on the device, raised from the same step() (environment/_graph.py)
            sink(ok, f"Scripted physical action of {self.name} is out of range")

    @property
    def u_range(self):
        return self.action.u_range

    @property
    def obs_noise(self):
        return self._obs_noise if self._obs_noise is not None else 0

    @property
    def action(self) -> Action:
        return self._action

    @property
    def u_multiplier(self):
        return self.action.u_multiplier

    @property
    def max_f(self):
        return self._max_f

    @property
    def f_range(self):
        return self._f_range

    @property
    def max_t(self):
        return self._max_t

    @property
    def t_range(self):
        return self._t_range

    @property
    def silent(self):
        return self._silent

    @property
    def sensors(self) -> List[Sensor]:
        return self._sensors

    @property
    def u_noise(self):
        return self.action.u_noise

    @property
    def c_noise(self):
        return self._c_noise

    @property
    def adversary(self):
        return self._adversary

    @override(Entity)
    def _spawn(self, dim_c: int, dim_p: int):
        if dim_c == 0:
            assert self.silent, f"Agent {self.name} must be silent when world has no communication"
        if self.silent:
            dim_c = 0
        super()._spawn(dim_c, dim_p)

    @override(Entity)
    def _reset(self, env_index: int):
        self.action._reset(env_index)
        self.dynamics.reset(env_index)
        super()._reset(env_index)

    def zero_grad(self):
        self.action.zero_grad()
        self.dynamics.zero_grad()
        super().zero_grad()

    @override(Entity)
    def to(self, device: torch.device):
        super().to(device)
        self.action.to(device)
        for sensor in self.sensors:
            sensor.to(device)


# ------------------------------------------------------------------------------------------------
class World(TorchVectorizedObject):
    """Multi-agent world (core.py:1089-2918).

    Extra (non-reference) knobs:
      * ``broadphase``: ``"batch"`` (default) reproduces the reference's batch-global broadphase
        (core.py:2796-2800) exactly; ``"env"`` simulates every static candidate pair in every env
        (what an independent single-env simulator would do; no host handshake per step).
    """
    def __setattr__(self, name, value):
        object.__setattr__(self, name, value)
        if name in _WORLD_STATIC:
            STATIC_VERSION[0] += 1


    def __init__(
        self,
        batch_dim: int,
        device: torch.device,
        dt: float = 0.1,
        substeps: int = 1,
        drag: float = DRAG,
        linear_friction: float = LINEAR_FRICTION,
        angular_friction: float = ANGULAR_FRICTION,
        x_semidim: float = None,
        y_semidim: float = None,
        dim_c: int = 0,
        collision_force: float = COLLISION_FORCE,
        joint_force: float = JOINT_FORCE,
        torque_constraint_force: float = TORQUE_CONSTRAINT_FORCE,
        contact_margin: float = 1e-3,
        gravity: Tuple[float, float] = (0.0, 0.0),
    ):
        assert batch_dim > 0, f"Batch dim must be greater than 0, got {batch_dim}"
        super().__init__(batch_dim, device)
        self._agents = []
        self._landmarks = []
        self._x_semidim = x_semidim
        self._y_semidim = y_semidim
        self._dim_p = 2
        self._dim_c = dim_c
        self._dt = dt
        self._substeps = substeps
        self._sub_dt = self._dt / self._substeps
        self._drag = drag
        self._gravity = torch.tensor(gravity, device=self.device, dtype=torch.float32)
        self._linear_friction = linear_friction
        self._angular_friction = angular_friction
        self._collision_force = collision_force
        self._joint_force = joint_force
        self._contact_margin = contact_margin
        self._torque_constraint_force = torque_constraint_force
        self._joints = {}
        # graph mode's sink for asserts on device tensors inside the step (None: assert eagerly)
        self._assert_sink = None
        # graph mode's sink for host code that waits on the device inside the step (the spawn
        # sampler; None: run it inline)
        self._hole_sink = None
        self._deferred_sink = None  # (graph capture) launches whose host side runs after each replay
        self._collidable_pairs = [
            {Sphere, Sphere},
            {Sphere, Box},
            {Sphere, Line},
            {Line, Line},
            {Line, Box},
            {Box, Box},
        ]
        self.entity_index_map = {}
        self.broadphase = "batch"
        # World.forces_dict / torques_dict (core.py:1975-1992): the step exports each dynamic
        # entity's last-substep totals (12 B per entity and env).  On by default for CPU worlds
        # (the reference's behaviour); opt-in on GPU worlds, where the exporting kernel keeps 3
        # more live registers per entity (balance C2: k_world 34.4 -> 38.3 us, profiles/r03/
        # run4_bisect).  VMAS_EXPORT_FORCES=0/1 overrides the default.
        env_default = os.environ.get("VMAS_EXPORT_FORCES")
        self.export_forces = (env_default != "0") if env_default is not None else torch.device(device).type == "cpu"
        self._forces_dict = None
        self._torques_dict = None
        self._force_buf = None
        self._engine = None

    def add_agent(self, agent: Agent):
        """Only way to add agents to the world"""
        agent.batch_dim = self._batch_dim
        agent.to(self._device)
        agent._spawn(dim_c=self._dim_c, dim_p=self.dim_p)
        self._agents.append(agent)
        STATIC_VERSION[0] += 1

    def add_landmark(self, landmark: Landmark):
        """Only way to add landmarks to the world"""
        landmark.batch_dim = self._batch_dim
        landmark.to(self._device)
        landmark._spawn(dim_c=self.dim_c, dim_p=self.dim_p)
        self._landmarks.append(landmark)
        STATIC_VERSION[0] += 1

    def add_joint(self, joint: Joint):
        assert self._substeps > 1, "For joints, world substeps needs to be more than 1"
        if joint.landmark is not None:
            self.add_landmark(joint.landmark)
        for constraint in joint.joint_constraints:
            self._joints.update({frozenset({constraint.entity_a.name, constraint.entity_b.name}): constraint})
        STATIC_VERSION[0] += 1

    def reset(self, env_index: int):
        for e in self.entities:
            e._reset(env_index)

    def zero_grad(self):
        for e in self.entities:
            e.zero_grad()

    @property
    def agents(self) -> List[Agent]:
        return self._agents

    @property
    def landmarks(self) -> List[Landmark]:
        return self._landmarks

    @property
    def x_semidim(self):
        return self._x_semidim

    @property
    def dt(self):
        return self._dt

    @property
    def y_semidim(self):
        return self._y_semidim

    @property
    def dim_p(self):
        return self._dim_p

    @property
    def dim_c(self):
        return self._dim_c

    @property
    def joints(self):
        return self._joints.values()

    @property
    def entities(self) -> List[Entity]:
        return self._landmarks + self._agents

    @property
    def policy_agents(self) -> List[Agent]:
        return [agent for agent in self._agents if agent.action_script is None]

    @property
    def scripted_agents(self) -> List[Agent]:
        return [agent for agent in self._agents if agent.action_script is not None]

    # ---- engine ---------------------------------------------------------------------------------
    @property
    def engine(self):
        if self._engine is None:
            from ._engine import PhysicsEngine

            self._engine = PhysicsEngine(self)
        return self._engine

    # ---- ray casting (core.py:1627-1785) ---------------------------------------------------------
    def cast_ray(self, entity: Entity, angles: Tensor, max_range: float,
                 entity_filter: Callable[[Entity], bool] = lambda _: False):
        pos = entity.state.pos
        assert pos.ndim == 2 and angles.ndim == 1
        assert pos.shape[0] == angles.shape[0]
        return self.engine.cast_rays(entity, angles.unsqueeze(-1), max_range, entity_filter).squeeze(-1)

    def cast_rays(self, entity: Entity, angles: Tensor, max_range: float,
                  entity_filter: Callable[[Entity], bool] = lambda _: False):
        return self.engine.cast_rays(entity, angles, max_range, entity_filter)

    # ---- distance queries (core.py:1787-1968) ----------------------------------------------------
    def get_distance_from_point(self, entity: Entity, test_point_pos, env_index: int = None):
        self._check_batch_index(env_index)
        value = self.engine.distance_from_point(entity, test_point_pos)
        return value[env_index] if env_index is not None else value

    def get_distance(self, entity_a: Entity, entity_b: Entity, env_index: int = None):
        self._check_batch_index(env_index)
        value = self.engine.distance(entity_a, entity_b)
        a_shape, b_shape = entity_a.shape, entity_b.shape
        # the reference indexes by env_index only in its sphere/line/box-sphere branches
        point_based = isinstance(a_shape, Sphere) or isinstance(b_shape, Sphere)
        return value[env_index] if (env_index is not None and point_based) else value

    def is_overlapping(self, entity_a: Entity, entity_b: Entity, env_index: int = None):
        self._check_batch_index(env_index)
        value = self.engine.overlap(entity_a, entity_b)
        if env_index is None:
            return value
        # indexed only in the sphere branches, as core.py:1931 returns get_distance(...) < 0 directly
        point_based = isinstance(entity_a.shape, Sphere) or isinstance(entity_b.shape, Sphere)
        return value[env_index] if point_based else value

    # ---- the step (core.py:1970-2014) -------------------------------------------------------------
    @property
    def forces_dict(self):
        """{entity: [B, 2]} force totals of the last step's last substep (core.py:1975-2198), as the
        reference leaves them after every step.  The step writes them into one buffer (the
        kernels' last-substep totals, ``export_forces``, on by default); the dict of views is
        built on first read."""
        if self._forces_dict is None:
            self._build_force_dicts()
        return self._forces_dict

    @property
    def torques_dict(self):
        """{entity: [B, 1]} torque totals of the last step's last substep (core.py:1984-2198)."""
        if self._torques_dict is None:
            self._build_force_dicts()
        return self._torques_dict

    def _build_force_dicts(self):
        buf = getattr(self, "_force_buf", None)
        if buf is None:
            raise AttributeError("forces_dict: no step has exported force totals yet (world.export_forces "
                                 "was False at the last step, or no step ran)")
        fd, B, engine, done = buf
        self._forces_dict, self._torques_dict = engine.force_dicts(fd, B, done)

    def step(self):
        self.entity_index_map = {e: i for i, e in enumerate(self.entities)}
        self.engine.step()
        if self._dim_c > 0:
            for agent in self._agents:
                self._update_comm_state(agent)

    def collides(self, a: Entity, b: Entity) -> bool:
        """Static part of World.collides (core.py:2787-2795) plus the batch-any range test."""
        if not self._collides_static(a, b):
            return False
        return bool(
            (
                torch.linalg.vector_norm(a.state.pos - b.state.pos, dim=-1)
                <= a.shape.circumscribed_radius() + b.shape.circumscribed_radius()
            ).any()
        )

    def _collides_static(self, a: Entity, b: Entity) -> bool:
        if (not a.collides(b)) or (not b.collides(a)) or a is b:
            return False
        if not a.movable and not a.rotatable and not b.movable and not b.rotatable:
            return False
        if not {a.shape.__class__, b.shape.__class__} in self._collidable_pairs:
            return False
        return True

    def _update_comm_state(self, agent):
        if not agent.silent:
            agent.state.c = agent.action.c

    @override(TorchVectorizedObject)
    def to(self, device: torch.device):
        super().to(device)
        for e in self.entities:
            e.to(device)
        self._engine = None
