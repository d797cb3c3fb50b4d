# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Joints (restates vmas/simulator/joints.py).

``Joint`` is an observer that owns an optional "joint landmark" (a Line or Box of length
``dist``) and the ``JointConstraint`` s that the physics step enforces (core.py:2200-2291).  The
constraint geometry (anchor deltas, rotate flag, fixed rotation) is read by the engine when it
builds its tables; a per-env ``fixed_rotation`` tensor (set by ``notify``) is read every step.
"""
from __future__ import annotations

from typing import Optional, Tuple, TYPE_CHECKING

import torch

from .utils import Color, Observer, TorchUtils, X, Y

if TYPE_CHECKING:
    from .core import Entity


class Joint(Observer):
    def __init__(
        self,
        entity_a: "Entity",
        entity_b: "Entity",
        anchor_a: Tuple[float, float] = (0.0, 0.0),
        anchor_b: Tuple[float, float] = (0.0, 0.0),
        rotate_a: bool = True,
        rotate_b: bool = True,
        dist: float = 0.0,
        collidable: bool = False,
        width: float = 0.0,
        mass: float = 1.0,
        fixed_rotation_a: Optional[float] = None,
        fixed_rotation_b: Optional[float] = None,
    ):
        from .core import Box, Landmark, Line

        assert entity_a != entity_b, "Cannot join same entity"
        for anchor in (anchor_a, anchor_b):
            assert max(anchor) <= 1 and min(anchor) >= -1, (
                f"Joint anchor points should be between -1 and 1, got {anchor}"
            )
        assert dist >= 0, f"Joint dist must be >= 0, got {dist}"
        if dist == 0:
            assert not collidable, "Cannot have collidable joint with dist 0"
            assert width == 0, "Cannot have width for joint with dist 0"
            assert fixed_rotation_a == fixed_rotation_b, (
                "If dist is 0, fixed_rotation_a and fixed_rotation_b should be the same"
            )
        if fixed_rotation_a is not None:
            assert not rotate_a, "If you provide a fixed rotation for a, rotate_a should be False"
        if fixed_rotation_b is not None:
            assert not rotate_b, "If you provide a fixed rotation for b, rotate_b should be False"
        if width > 0:
            assert collidable

        self.entity_a = entity_a
        self.entity_b = entity_b
        self.rotate_a = rotate_a
        self.rotate_b = rotate_b
        self.fixed_rotation_a = fixed_rotation_a
        self.fixed_rotation_b = fixed_rotation_b
        self.landmark = None
        self.joint_constraints = []

        if dist == 0:
            self.joint_constraints.append(
                JointConstraint(
                    entity_a, entity_b, anchor_a=anchor_a, anchor_b=anchor_b, dist=dist,
                    rotate=rotate_a and rotate_b, fixed_rotation=fixed_rotation_a,
                )
            )
        else:
            entity_a.subscribe(self)
            entity_b.subscribe(self)
            self.landmark = Landmark(
                name=f"joint {entity_a.name} {entity_b.name}",
                collide=collidable,
                movable=True,
                rotatable=True,
                mass=mass,
                shape=(Box(length=dist, width=width) if width != 0 else Line(length=dist)),
                color=Color.BLACK,
                is_joint=True,
            )
            self.joint_constraints += [
                JointConstraint(
                    self.landmark, entity_a, anchor_a=(-1, 0), anchor_b=anchor_a, dist=0.0,
                    rotate=rotate_a, fixed_rotation=fixed_rotation_a,
                ),
                JointConstraint(
                    self.landmark, entity_b, anchor_a=(1, 0), anchor_b=anchor_b, dist=0.0,
                    rotate=rotate_b, fixed_rotation=fixed_rotation_b,
                ),
            ]

    def notify(self, observable, *args, **kwargs):
        # joints.py:119-143: re-centre the joint landmark between the two anchors
        pos_a = self.joint_constraints[0].pos_point(self.entity_a)
        pos_b = self.joint_constraints[1].pos_point(self.entity_b)
        self.landmark.set_pos((pos_a + pos_b) / 2, batch_index=None)
        angle = torch.atan2(pos_b[:, Y] - pos_a[:, Y], pos_b[:, X] - pos_a[:, X]).unsqueeze(-1)
        self.landmark.set_rot(angle, batch_index=None)
        if not self.rotate_a and self.fixed_rotation_a is None:
            self.joint_constraints[0].fixed_rotation = angle - self.entity_a.state.rot
        if not self.rotate_b and self.fixed_rotation_b is None:
            self.joint_constraints[1].fixed_rotation = angle - self.entity_b.state.rot


class JointConstraint:
    """Uncollidable constraint binding two entities at anchor points at a distance (joints.py:147)."""
    def __setattr__(self, name, value):
        object.__setattr__(self, name, value)
        if name in ("dist", "rotate", "fixed_rotation"):  # (read by the engine's signature)
            from . import core

            core.STATIC_VERSION[0] += 1


    def __init__(
        self,
        entity_a: "Entity",
        entity_b: "Entity",
        anchor_a: Tuple[float, float] = (0.0, 0.0),
        anchor_b: Tuple[float, float] = (0.0, 0.0),
        dist: float = 0.0,
        rotate: bool = True,
        fixed_rotation: Optional[float] = None,
    ):
        assert entity_a != entity_b, "Cannot join same entity"
        for anchor in (anchor_a, anchor_b):
            assert max(anchor) <= 1 and min(anchor) >= -1, (
                f"Joint anchor points should be between -1 and 1, got {anchor}"
            )
        assert dist >= 0, f"Joint dist must be >= 0, got {dist}"
        if fixed_rotation is not None:
            assert not rotate, "If fixed rotation is provided, rotate should be False"
        if rotate:
            assert fixed_rotation is None, "If you provide a fixed rotation, rotate should be False"
            fixed_rotation = 0.0
        self.entity_a = entity_a
        self.entity_b = entity_b
        self.anchor_a = anchor_a
        self.anchor_b = anchor_b
        self.dist = dist
        self.fixed_rotation = fixed_rotation
        self.rotate = rotate

    def delta_anchor(self, entity: "Entity") -> Tuple[float, float]:
        if entity is self.entity_a:
            anchor = self.anchor_a
        elif entity is self.entity_b:
            anchor = self.anchor_b
        else:
            raise AssertionError()
        return entity.shape.get_delta_from_anchor(anchor)

    def get_delta_anchor(self, entity: "Entity"):
        d = torch.tensor(self.delta_anchor(entity), device=entity.state.pos.device)
        return TorchUtils.rotate_vector(d.unsqueeze(0).expand(entity.state.pos.shape), entity.state.rot)

    def pos_point(self, entity: "Entity"):
        return entity.state.pos + self.get_delta_anchor(entity)
