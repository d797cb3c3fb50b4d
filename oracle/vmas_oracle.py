# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""ORACLE -- test infrastructure only (never imported by the product package).

A PyTorch-CPU restatement of the reference's tensor programs for the hot path:
  * World.step                (vmas/simulator/core.py:1970-2912, incl. the batch-global
                               broadphase World.collides core.py:2787-2802)
  * World.cast_rays / cast_ray (core.py:1233-1785)
  * distance queries           (core.py:1787-1968)
  * closest-point geometry     (vmas/simulator/physics.py:12-428)
Each function follows the reference's op sequence (class-batched stacks, the same python-scalar
/ fp32-tensor mixes, the same torch reductions), so that it is both the checker for the native
engine and the "reference PyTorch-CPU" baseline timed by bench.py.

Parity status: the reference itself may not be run in this environment (SURVEY.md §8c records
the refusal) and holds no numeric golden vectors, so this oracle is pinned by analytic
known-answer tests (tests/test_oracle_kat.py) and the reference's behavioural pins restated in
tests/ -- not by reference outputs ("parity partially pinned").

It works on any World object with the reference's attribute names (the product's
``vectorizedmultiagentsimulator_amd.simulator.core.World`` has them), reading entity parameters
from it and state from an explicit snapshot, so one-step teacher-forced comparisons are easy:
``compare_one_step(world)``.
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch
from torch import Tensor

LINE_MIN_DIST = 4 / 6e2  # utils.py:27
X, Y = 0, 1
CPU = torch.device("cpu")


# ------------------------------------------------------------------------------------------------
# TorchUtils (utils.py:166-201)
def clamp_with_norm(tensor: Tensor, max_norm: float):
    norm = torch.linalg.vector_norm(tensor, dim=-1)
    new_tensor = (tensor / norm.unsqueeze(-1)) * max_norm
    cond = (norm > max_norm).unsqueeze(-1).expand(tensor.shape)
    return torch.where(cond, new_tensor, tensor)


def rotate_vector(vector: Tensor, angle: Tensor):
    if len(angle.shape) == len(vector.shape):
        angle = angle.squeeze(-1)
    cos = torch.cos(angle)
    sin = torch.sin(angle)
    return torch.stack([vector[..., X] * cos - vector[..., Y] * sin, vector[..., X] * sin + vector[..., Y] * cos], dim=-1)


def cross(a: Tensor, b: Tensor):
    return (a[..., X] * b[..., Y] - a[..., Y] * b[..., X]).unsqueeze(-1)


def compute_torque(f: Tensor, r: Tensor):
    return cross(r, f)


# ------------------------------------------------------------------------------------------------
# physics.py
def get_inner_point_box(outside_point, surface_point, box_pos):  # physics.py:12-22
    v = surface_point - outside_point
    u = box_pos - surface_point
    v_norm = torch.linalg.vector_norm(v, dim=-1).unsqueeze(-1)
    x_magnitude = (v * u).sum(-1).unsqueeze(-1) / v_norm
    x = (v / v_norm) * x_magnitude
    cond = v_norm == 0
    x = torch.where(cond.expand(x.shape), surface_point, x)
    x_magnitude = torch.where(cond, 0, x_magnitude)
    return surface_point + x, torch.abs(x_magnitude.squeeze(-1))


def _as_len(v, like):
    if not isinstance(v, Tensor):
        v = torch.tensor(v, dtype=torch.float32).expand(like.shape[0])
    return v


def get_closest_box_box(box_pos, box_rot, box_width, box_length, box2_pos, box2_rot, box2_width, box2_length):
    box_width, box_length = _as_len(box_width, box_pos), _as_len(box_length, box_pos)
    box2_width, box2_length = _as_len(box2_width, box2_pos), _as_len(box2_length, box2_pos)
    lines_pos, lines_rot, lines_length = get_all_lines_box(
        torch.stack([box_pos, box2_pos], dim=0),
        torch.stack([box_rot, box2_rot], dim=0),
        torch.stack([box_width, box2_width], dim=0),
        torch.stack([box_length, box2_length], dim=0),
    )
    lines_a_pos, lines_b_pos = lines_pos.unbind(1)
    lines_a_rot, lines_b_rot = lines_rot.unbind(1)
    lines_a_length, lines_b_length = lines_length.unbind(1)
    points_first, points_second = get_closest_line_box(
        torch.stack([box2_pos.unsqueeze(0).expand(lines_a_pos.shape), box_pos.unsqueeze(0).expand(lines_b_pos.shape)], dim=0),
        torch.stack([box2_rot.unsqueeze(0).expand(lines_a_rot.shape), box_rot.unsqueeze(0).expand(lines_b_rot.shape)], dim=0),
        torch.stack([box2_width.unsqueeze(0).expand(lines_a_length.shape), box_width.unsqueeze(0).expand(lines_b_length.shape)], dim=0),
        torch.stack([box2_length.unsqueeze(0).expand(lines_a_length.shape), box_length.unsqueeze(0).expand(lines_b_length.shape)], dim=0),
        torch.stack([lines_a_pos, lines_b_pos], dim=0),
        torch.stack([lines_a_rot, lines_b_rot], dim=0),
        torch.stack([lines_a_length, lines_b_length], dim=0),
    )
    points_box2_a, points_box_b = points_first.unbind(0)
    points_box_a, points_box2_b = points_second.unbind(0)
    p1s = points_box_a.unbind(0) + points_box_b.unbind(0)
    p2s = points_box2_a.unbind(0) + points_box2_b.unbind(0)
    closest_point_1 = torch.full(box_pos.shape, float("inf"), dtype=torch.float32)
    closest_point_2 = torch.full(box_pos.shape, float("inf"), dtype=torch.float32)
    distance = torch.full(box_pos.shape[:-1], float("inf"), dtype=torch.float32)
    for p1, p2 in zip(p1s, p2s):
        d = torch.linalg.vector_norm(p1 - p2, dim=-1)
        is_closest = d < distance
        is_closest_exp = is_closest.unsqueeze(-1).expand(p1.shape)
        closest_point_1 = torch.where(is_closest_exp, p1, closest_point_1)
        closest_point_2 = torch.where(is_closest_exp, p2, closest_point_2)
        distance = torch.where(is_closest, d, distance)
    return closest_point_1, closest_point_2


def get_line_extrema(line_pos, line_rot, line_length):  # physics.py:131-140
    line_length = line_length.view(line_rot.shape)
    x = (line_length / 2) * torch.cos(line_rot)
    y = (line_length / 2) * torch.sin(line_rot)
    xy = torch.cat([x, y], dim=-1)
    return line_pos + xy, line_pos - xy


def get_closest_points_line_line(line_pos, line_rot, line_length, line2_pos, line2_rot, line2_length):
    line_length = _as_len(line_length, line_pos)
    line2_length = _as_len(line2_length, line_pos)
    points_a, points_b = get_line_extrema(
        torch.stack([line_pos, line2_pos], dim=0),
        torch.stack([line_rot, line2_rot], dim=0),
        torch.stack([line_length, line2_length], dim=0),
    )
    point_a1, point_b1 = points_a.unbind(0)
    point_a2, point_b2 = points_b.unbind(0)
    point_i, d_i = get_intersection_point_line_line(point_a1, point_a2, point_b1, point_b2)
    (point_a1_line_b, point_a2_line_b, point_b1_line_a, point_b2_line_a) = get_closest_point_line(
        torch.stack([line2_pos, line2_pos, line_pos, line_pos], dim=0),
        torch.stack([line2_rot, line2_rot, line_rot, line_rot], dim=0),
        torch.stack([line2_length, line2_length, line_length, line_length], dim=0),
        torch.stack([point_a1, point_a2, point_b1, point_b2], dim=0),
    ).unbind(0)
    point_pairs = (
        (point_a1, point_a1_line_b),
        (point_a2, point_a2_line_b),
        (point_b1_line_a, point_b1),
        (point_b2_line_a, point_b2),
    )
    closest_point_1 = torch.full(line_pos.shape, float("inf"), dtype=torch.float32)
    closest_point_2 = torch.full(line_pos.shape, float("inf"), dtype=torch.float32)
    min_distance = torch.full(line_pos.shape[:-1], float("inf"), dtype=torch.float32)
    for p1, p2 in point_pairs:
        d = torch.linalg.vector_norm(p1 - p2, dim=-1)
        is_closest = d < min_distance
        is_closest_exp = is_closest.unsqueeze(-1).expand(p1.shape)
        closest_point_1 = torch.where(is_closest_exp, p1, closest_point_1)
        closest_point_2 = torch.where(is_closest_exp, p2, closest_point_2)
        min_distance = torch.where(is_closest, d, min_distance)
    cond = (d_i == 0).unsqueeze(-1).expand(point_i.shape)
    closest_point_1 = torch.where(cond, point_i, closest_point_1)
    closest_point_2 = torch.where(cond, point_i, closest_point_2)
    return closest_point_1, closest_point_2


def get_intersection_point_line_line(point_a1, point_a2, point_b1, point_b2):  # physics.py:221-259
    r = point_a2 - point_a1
    s = point_b2 - point_b1
    p = point_a1
    q = point_b1
    cross_q_minus_p_r = cross(q - p, r)
    cross_q_minus_p_s = cross(q - p, s)
    cross_r_s = cross(r, s)
    u = cross_q_minus_p_r / cross_r_s
    t = cross_q_minus_p_s / cross_r_s
    t_in_range = (0 <= t) * (t <= 1)
    u_in_range = (0 <= u) * (u <= 1)
    cross_r_s_is_zero = cross_r_s == 0
    distance = torch.full(point_a1.shape[:-1], float("inf"), dtype=torch.float32)
    point = torch.full(point_a1.shape, float("inf"), dtype=torch.float32)
    condition = ~cross_r_s_is_zero * u_in_range * t_in_range
    point = torch.where(condition.expand(point.shape), p + t * r, point)
    distance = torch.where(condition.squeeze(-1), 0.0, distance)
    return point, distance


def get_closest_point_box(box_pos, box_rot, box_width, box_length, test_point_pos):  # physics.py:262-294
    box_width, box_length = _as_len(box_width, box_pos), _as_len(box_length, box_pos)
    closest_points = get_all_points_box(box_pos, box_rot, box_width, box_length, test_point_pos)
    closest_point = torch.full(box_pos.shape, float("inf"), dtype=torch.float32)
    distance = torch.full(box_pos.shape[:-1], float("inf"), dtype=torch.float32)
    for p in closest_points:
        d = torch.linalg.vector_norm(test_point_pos - p, dim=-1)
        is_closest = d < distance
        closest_point = torch.where(is_closest.unsqueeze(-1).expand(p.shape), p, closest_point)
        distance = torch.where(is_closest, d, distance)
    return closest_point


def get_all_lines_box(box_pos, box_rot, box_width, box_length):  # physics.py:297-324
    rotated_vector = torch.cat([box_rot.cos(), box_rot.sin()], dim=-1)
    rot_2 = box_rot + torch.pi / 2
    rotated_vector2 = torch.cat([rot_2.cos(), rot_2.sin()], dim=-1)
    expanded_half_box_length = box_length.unsqueeze(-1).expand(rotated_vector.shape) / 2
    expanded_half_box_width = box_width.unsqueeze(-1).expand(rotated_vector.shape) / 2
    p1 = box_pos + rotated_vector * expanded_half_box_length
    p2 = box_pos - rotated_vector * expanded_half_box_length
    p3 = box_pos + rotated_vector2 * expanded_half_box_width
    p4 = box_pos - rotated_vector2 * expanded_half_box_width
    ps, rots, lengths = [], [], []
    for i, p in enumerate([p1, p2, p3, p4]):
        ps.append(p)
        rots.append(box_rot + torch.pi / 2 if i <= 1 else box_rot)
        lengths.append(box_width if i <= 1 else box_length)
    return torch.stack(ps, dim=0), torch.stack(rots, dim=0), torch.stack(lengths, dim=0)


def get_closest_line_box(box_pos, box_rot, box_width, box_length, line_pos, line_rot, line_length):
    box_width, box_length = _as_len(box_width, box_pos), _as_len(box_length, box_pos)
    line_length = _as_len(line_length, line_pos)
    lines_pos, lines_rot, lines_length = get_all_lines_box(box_pos, box_rot, box_width, box_length)
    closest_point_1 = torch.full(box_pos.shape, float("inf"), dtype=torch.float32)
    closest_point_2 = torch.full(box_pos.shape, float("inf"), dtype=torch.float32)
    distance = torch.full(box_pos.shape[:-1], float("inf"), dtype=torch.float32)
    ps_box, ps_line = get_closest_points_line_line(
        lines_pos, lines_rot, lines_length,
        line_pos.unsqueeze(0).expand(lines_pos.shape),
        line_rot.unsqueeze(0).expand(lines_rot.shape),
        line_length.unsqueeze(0).expand(lines_length.shape),
    )
    for p_box, p_line in zip(ps_box.unbind(0), ps_line.unbind(0)):
        d = torch.linalg.vector_norm(p_box - p_line, dim=-1)
        is_closest = d < distance
        is_closest_exp = is_closest.unsqueeze(-1).expand(closest_point_1.shape)
        closest_point_1 = torch.where(is_closest_exp, p_box, closest_point_1)
        closest_point_2 = torch.where(is_closest_exp, p_line, closest_point_2)
        distance = torch.where(is_closest, d, distance)
    return closest_point_1, closest_point_2


def get_all_points_box(box_pos, box_rot, box_width, box_length, test_point_pos):
    lines_pos, lines_rot, lines_length = get_all_lines_box(box_pos, box_rot, box_width, box_length)
    return get_closest_point_line(
        lines_pos, lines_rot, lines_length, test_point_pos.unsqueeze(0).expand(lines_pos.shape)
    ).unbind(0)


def get_closest_point_line(line_pos, line_rot, line_length, test_point_pos, limit_to_line_length=True):
    assert line_rot.shape[-1] == 1
    if not isinstance(line_length, Tensor):
        line_length = torch.tensor(line_length, dtype=torch.float32).expand(line_rot.shape)
    rotated_vector = torch.cat([line_rot.cos(), line_rot.sin()], dim=-1)
    delta_pos = line_pos - test_point_pos
    dot_p = (delta_pos * rotated_vector).sum(-1).unsqueeze(-1)
    sign = torch.sign(dot_p)
    distance_from_line_center = (
        torch.minimum(torch.abs(dot_p), (line_length / 2).view(dot_p.shape))
        if limit_to_line_length
        else torch.abs(dot_p)
    )
    return line_pos - sign * distance_from_line_center * rotated_vector


# ------------------------------------------------------------------------------------------------
# snapshots
def _kind(shape) -> str:
    return type(shape).__name__  # "Sphere" / "Box" / "Line"


def _cpu(t):
    return None if t is None else t.detach().to(CPU, torch.float32).clone()


def snapshot(world) -> Dict[int, dict]:
    """CPU copy of every entity's state (+ agent force/torque), keyed by entity index."""
    snap = {}
    for i, e in enumerate(world.entities):
        s = e.state
        d = {"pos": _cpu(s.pos), "vel": _cpu(s.vel), "rot": _cpu(s.rot), "ang_vel": _cpu(s.ang_vel)}
        if hasattr(s, "force"):
            d["force"] = _cpu(s.force)
            d["torque"] = _cpu(s.torque)
        snap[i] = d
    return snap


class _Ent:
    """Minimal stand-in exposing entity params + snapshot state, so the restated code reads
    exactly like the reference (``entity.state.pos``, ``entity.mass``...)."""

    class _S:
        pass

    def __init__(self, e, st):
        self.e = e
        self.state = _Ent._S()
        for k, v in st.items():
            setattr(self.state, k, v)
        self.shape = e.shape
        self.name = e.name
        self.movable = e.movable
        self.rotatable = e.rotatable
        self.mass = e.mass
        self.moment_of_inertia = e.moment_of_inertia
        self.drag = e.drag
        self.linear_friction = e.linear_friction
        self.angular_friction = e.angular_friction
        self.gravity = _cpu(e.gravity) if isinstance(e.gravity, Tensor) else e.gravity
        self.max_speed = e.max_speed
        self.v_range = e.v_range
        self.is_agent = hasattr(st, "__contains__") and "force" in st
        self.max_f = getattr(e, "max_f", None)
        self.f_range = getattr(e, "f_range", None)
        self.max_t = getattr(e, "max_t", None)
        self.t_range = getattr(e, "t_range", None)

    def collides(self, other: "_Ent"):
        return self.e.collides(other.e)


class OracleWorld:
    """The reference World.step / cast_rays / distance programs on CPU tensors."""

    def __init__(self, world, snap: Dict[int, dict], broadphase: str = "batch", grad_safe: bool = False):
        self.w = world
        # the reference's ray casts write max_range into a norm's output in place (core.py:1277,
        # 1370, 1537-1540), which torch.autograd refuses to differentiate; grad_safe restates those
        # writes as torch.where (the same values) so tests can take the oracle's ray gradients
        self.grad_safe = grad_safe
        self.ents: List[_Ent] = [_Ent(e, snap[i]) for i, e in enumerate(world.entities)]
        self.by_obj = {id(e): self.ents[i] for i, e in enumerate(world.entities)}
        self.batch_dim = world.batch_dim
        self._substeps = world._substeps
        self._sub_dt = world._sub_dt  # the attribute itself (ref core.py:2068, 2870), not dt/substeps
        self._drag = world._drag
        self._gravity = _cpu(world._gravity)
        self._linear_friction = world._linear_friction
        self._angular_friction = world._angular_friction
        self._collision_force = world._collision_force
        self._joint_force = world._joint_force
        self._contact_margin = world._contact_margin
        self._torque_constraint_force = world._torque_constraint_force
        self._x_semidim = world._x_semidim
        self._y_semidim = world._y_semidim
        self._collidable_pairs = world._collidable_pairs
        self.broadphase = broadphase
        self.active_log = []  # per substep: list of (class, a name, b name)
        # per env: the smallest |dist - cut-off| of any soft-contact evaluation of the step (the
        # force switches on/off discontinuously there: dist > dist_min, dist < 1e-6)
        self.cutoff_margin = torch.full((self.batch_dim,), float("inf"))

    # ---- step (core.py:1970-2014) ---------------------------------------------------------------
    def step(self):
        for substep in range(self._substeps):
            self.forces_dict = {e: torch.zeros(self.batch_dim, 2, dtype=torch.float32) for e in self.ents}
            self.torques_dict = {e: torch.zeros(self.batch_dim, 1, dtype=torch.float32) for e in self.ents}
            for entity in self.ents:
                if entity.is_agent:
                    self._apply_action_force(entity)
                    self._apply_action_torque(entity)
                self._apply_friction_force(entity)
                self._apply_gravity(entity)
            self._apply_vectorized_enviornment_force()
            for entity in self.ents:
                self._integrate_state(entity, substep)

    def _apply_action_force(self, agent):  # core.py:2017-2027
        if agent.movable:
            if agent.max_f is not None:
                agent.state.force = clamp_with_norm(agent.state.force, agent.max_f)
            if agent.f_range is not None:
                agent.state.force = torch.clamp(agent.state.force, -agent.f_range, agent.f_range)
            self.forces_dict[agent] = self.forces_dict[agent] + agent.state.force

    def _apply_action_torque(self, agent):  # core.py:2029-2040
        if agent.rotatable:
            if agent.max_t is not None:
                agent.state.torque = clamp_with_norm(agent.state.torque, agent.max_t)
            if agent.t_range is not None:
                agent.state.torque = torch.clamp(agent.state.torque, -agent.t_range, agent.t_range)
            self.torques_dict[agent] = self.torques_dict[agent] + agent.state.torque

    def _apply_gravity(self, entity):  # core.py:2042-2051
        if entity.movable:
            if not (self._gravity == 0.0).all():
                self.forces_dict[entity] = self.forces_dict[entity] + entity.mass * self._gravity
            if entity.gravity is not None:
                self.forces_dict[entity] = self.forces_dict[entity] + entity.mass * entity.gravity

    def _apply_friction_force(self, entity):  # core.py:2053-2101
        def get_friction_force(vel, coeff, force, mass):
            speed = torch.linalg.vector_norm(vel, dim=-1)
            static = speed == 0
            static_exp = static.unsqueeze(-1).expand(vel.shape)
            if not isinstance(coeff, Tensor):
                coeff = torch.full_like(force, coeff)
            coeff = coeff.expand(force.shape)
            friction_force_constant = coeff * mass
            friction_force = -(vel / torch.where(static, 1e-8, speed).unsqueeze(-1)) * torch.minimum(
                friction_force_constant, (vel.abs() / self._sub_dt) * mass
            )
            return torch.where(static_exp, 0.0, friction_force)

        if entity.linear_friction is not None:
            self.forces_dict[entity] = self.forces_dict[entity] + get_friction_force(
                entity.state.vel, entity.linear_friction, self.forces_dict[entity], entity.mass)
        elif self._linear_friction > 0:
            self.forces_dict[entity] = self.forces_dict[entity] + get_friction_force(
                entity.state.vel, self._linear_friction, self.forces_dict[entity], entity.mass)
        if entity.angular_friction is not None:
            self.torques_dict[entity] = self.torques_dict[entity] + get_friction_force(
                entity.state.ang_vel, entity.angular_friction, self.torques_dict[entity], entity.moment_of_inertia)
        elif self._angular_friction > 0:
            self.torques_dict[entity] = self.torques_dict[entity] + get_friction_force(
                entity.state.ang_vel, self._angular_friction, self.torques_dict[entity], entity.moment_of_inertia)

    def collides(self, a, b) -> bool:  # core.py:2787-2802
        if (not a.collides(b)) or (not b.collides(a)) or a is b:
            return False
        if not a.movable and not a.rotatable and not b.movable and not b.rotatable:
            return False
        if not {a.shape.__class__, b.shape.__class__} in self._collidable_pairs:
            return False
        if self.broadphase == "batch" and not (
            torch.linalg.vector_norm(a.state.pos - b.state.pos, dim=-1)
            <= a.shape.circumscribed_radius() + b.shape.circumscribed_radius()
        ).any():
            return False
        return True

    def _apply_vectorized_enviornment_force(self):  # core.py:2103-2188
        s_s, l_s, b_s, l_l, b_l, b_b, joints = [], [], [], [], [], [], []
        jmap = self.w._joints
        for a, entity_a in enumerate(self.ents):
            for b, entity_b in enumerate(self.ents):
                if b <= a:
                    continue
                joint = jmap.get(frozenset({entity_a.name, entity_b.name}), None)
                if joint is not None:
                    joints.append(joint)
                    if joint.dist == 0:
                        continue
                if not self.collides(entity_a, entity_b):
                    continue
                ka, kb = _kind(entity_a.shape), _kind(entity_b.shape)
                if ka == "Sphere" and kb == "Sphere":
                    s_s.append((entity_a, entity_b))
                elif {ka, kb} == {"Line", "Sphere"}:
                    l_s.append((entity_a, entity_b) if kb == "Sphere" else (entity_b, entity_a))
                elif ka == "Line" and kb == "Line":
                    l_l.append((entity_a, entity_b))
                elif {ka, kb} == {"Box", "Sphere"}:
                    b_s.append((entity_a, entity_b) if kb == "Sphere" else (entity_b, entity_a))
                elif {ka, kb} == {"Box", "Line"}:
                    b_l.append((entity_a, entity_b) if kb == "Line" else (entity_b, entity_a))
                elif ka == "Box" and kb == "Box":
                    b_b.append((entity_a, entity_b))
                else:
                    raise AssertionError()
        self.active_log.append([(c, x.name, y.name) for c, lst in
                                (("ss", s_s), ("ls", l_s), ("ll", l_l), ("bs", b_s), ("bl", b_l), ("bb", b_b))
                                for x, y in lst])
        self._vectorized_joint_constraints(joints)
        self._sphere_sphere(s_s)
        self._sphere_line(l_s)
        self._line_line(l_l)
        self._box_sphere(b_s)
        self._box_line(b_l)
        self._box_box(b_b)

    def update_env_forces(self, entity_a, f_a, t_a, entity_b, f_b, t_b):  # core.py:2190-2198
        if entity_a.movable:
            self.forces_dict[entity_a] = self.forces_dict[entity_a] + f_a
        if entity_a.rotatable:
            self.torques_dict[entity_a] = self.torques_dict[entity_a] + t_a
        if entity_b.movable:
            self.forces_dict[entity_b] = self.forces_dict[entity_b] + f_b
        if entity_b.rotatable:
            self.torques_dict[entity_b] = self.torques_dict[entity_b] + t_b

    def _t(self, values):
        """[B, P] tensor of per-pair python floats (torch.tensor(...) stack + expand)."""
        return torch.stack([torch.tensor(v) for v in values], dim=-1).unsqueeze(0).expand(self.batch_dim, -1)

    def _vectorized_joint_constraints(self, joints):  # core.py:2200-2291
        if not len(joints):
            return
        E = lambda ent: self.by_obj[id(ent)]  # noqa: E731
        pos_a, pos_b, pos_joint_a, pos_joint_b, dist, rotate, rot_a, rot_b, joint_rot = ([] for _ in range(9))
        for joint in joints:
            ea, eb = E(joint.entity_a), E(joint.entity_b)
            for ent, lst in ((ea, pos_joint_a), (eb, pos_joint_b)):
                d = torch.tensor(joint.delta_anchor(ent.e)).unsqueeze(0).expand(ent.state.pos.shape)
                lst.append(ent.state.pos + rotate_vector(d, ent.state.rot))
            pos_a.append(ea.state.pos)
            pos_b.append(eb.state.pos)
            dist.append(torch.tensor(joint.dist))
            rotate.append(torch.tensor(joint.rotate))
            rot_a.append(ea.state.rot)
            rot_b.append(eb.state.rot)
            fr = joint.fixed_rotation
            joint_rot.append(
                torch.tensor(fr).unsqueeze(-1).expand(self.batch_dim, 1) if not isinstance(fr, Tensor) else _cpu(fr)
            )
        pos_a, pos_b = torch.stack(pos_a, dim=-2), torch.stack(pos_b, dim=-2)
        pos_joint_a, pos_joint_b = torch.stack(pos_joint_a, dim=-2), torch.stack(pos_joint_b, dim=-2)
        rot_a, rot_b = torch.stack(rot_a, dim=-2), torch.stack(rot_b, dim=-2)
        dist = torch.stack(dist, dim=-1).unsqueeze(0).expand(self.batch_dim, -1)
        rotate = torch.stack(rotate, dim=-1).unsqueeze(0).expand(self.batch_dim, -1).unsqueeze(-1)
        joint_rot = torch.stack(joint_rot, dim=-2)
        fa_att, fb_att = self._get_constraint_forces(pos_joint_a, pos_joint_b, dist_min=dist, attractive=True,
                                                     force_multiplier=self._joint_force)
        fa_rep, fb_rep = self._get_constraint_forces(pos_joint_a, pos_joint_b, dist_min=dist, attractive=False,
                                                     force_multiplier=self._joint_force)
        force_a = fa_att + fa_rep
        force_b = fb_att + fb_rep
        torque_a_rotate = compute_torque(force_a, pos_joint_a - pos_a)
        torque_b_rotate = compute_torque(force_b, pos_joint_b - pos_b)
        torque_a_fixed, torque_b_fixed = self._get_constraint_torques(
            rot_a, rot_b + joint_rot, force_multiplier=self._torque_constraint_force)
        torque_a = torch.where(rotate, torque_a_rotate, torque_a_rotate + torque_a_fixed)
        torque_b = torch.where(rotate, torque_b_rotate, torque_b_rotate + torque_b_fixed)
        for i, joint in enumerate(joints):
            self.update_env_forces(E(joint.entity_a), force_a[:, i], torque_a[:, i],
                                   E(joint.entity_b), force_b[:, i], torque_b[:, i])

    def _sphere_sphere(self, s_s):  # core.py:2293-2338
        if not len(s_s):
            return
        pos_a = torch.stack([a.state.pos for a, _ in s_s], dim=-2)
        pos_b = torch.stack([b.state.pos for _, b in s_s], dim=-2)
        ra = self._t([a.shape.radius for a, _ in s_s])
        rb = self._t([b.shape.radius for _, b in s_s])
        force_a, force_b = self._get_constraint_forces(pos_a, pos_b, dist_min=ra + rb,
                                                       force_multiplier=self._collision_force)
        for i, (a, b) in enumerate(s_s):
            self.update_env_forces(a, force_a[:, i], 0, b, force_b[:, i], 0)

    def _sphere_line(self, l_s):  # core.py:2340-2391
        if not len(l_s):
            return
        pos_l = torch.stack([l.state.pos for l, _ in l_s], dim=-2)
        pos_s = torch.stack([s.state.pos for _, s in l_s], dim=-2)
        rot_l = torch.stack([l.state.rot for l, _ in l_s], dim=-2)
        radius_s = self._t([s.shape.radius for _, s in l_s])
        length_l = self._t([l.shape.length for l, _ in l_s])
        closest_point = get_closest_point_line(pos_l, rot_l, length_l, pos_s)
        force_sphere, force_line = self._get_constraint_forces(
            pos_s, closest_point, dist_min=radius_s + LINE_MIN_DIST, force_multiplier=self._collision_force)
        torque_line = compute_torque(force_line, closest_point - pos_l)
        for i, (l, s) in enumerate(l_s):
            self.update_env_forces(l, force_line[:, i], torque_line[:, i], s, force_sphere[:, i], 0)

    def _line_line(self, l_l):  # core.py:2393-2456
        if not len(l_l):
            return
        pos_a = torch.stack([a.state.pos for a, _ in l_l], dim=-2)
        pos_b = torch.stack([b.state.pos for _, b in l_l], dim=-2)
        rot_a = torch.stack([a.state.rot for a, _ in l_l], dim=-2)
        rot_b = torch.stack([b.state.rot for _, b in l_l], dim=-2)
        len_a = self._t([a.shape.length for a, _ in l_l])
        len_b = self._t([b.shape.length for _, b in l_l])
        point_a, point_b = get_closest_points_line_line(pos_a, rot_a, len_a, pos_b, rot_b, len_b)
        force_a, force_b = self._get_constraint_forces(point_a, point_b, dist_min=LINE_MIN_DIST,
                                                       force_multiplier=self._collision_force)
        torque_a = compute_torque(force_a, point_a - pos_a)
        torque_b = compute_torque(force_b, point_b - pos_b)
        for i, (a, b) in enumerate(l_l):
            self.update_env_forces(a, force_a[:, i], torque_a[:, i], b, force_b[:, i], torque_b[:, i])

    def _box_sphere(self, b_s):  # core.py:2458-2551
        if not len(b_s):
            return
        pos_box = torch.stack([b.state.pos for b, _ in b_s], dim=-2)
        pos_sphere = torch.stack([s.state.pos for _, s in b_s], dim=-2)
        rot_box = torch.stack([b.state.rot for b, _ in b_s], dim=-2)
        length_box = self._t([b.shape.length for b, _ in b_s])
        width_box = self._t([b.shape.width for b, _ in b_s])
        not_hollow_prior = torch.stack([torch.tensor(not b.shape.hollow) for b, _ in b_s], dim=-1)
        not_hollow = not_hollow_prior.unsqueeze(0).expand(self.batch_dim, -1)
        radius_sphere = self._t([s.shape.radius for _, s in b_s])
        closest_point_box = get_closest_point_box(pos_box, rot_box, width_box, length_box, pos_sphere)
        inner_point_box = closest_point_box
        d = torch.zeros_like(radius_sphere, dtype=torch.float)
        if not_hollow_prior.any():
            inner_hollow, d_hollow = get_inner_point_box(pos_sphere, closest_point_box, pos_box)
            cond = not_hollow.unsqueeze(-1).expand(inner_point_box.shape)
            inner_point_box = torch.where(cond, inner_hollow, inner_point_box)
            d = torch.where(not_hollow, d_hollow, d)
        force_sphere, force_box = self._get_constraint_forces(
            pos_sphere, inner_point_box, dist_min=radius_sphere + LINE_MIN_DIST + d,
            force_multiplier=self._collision_force)
        torque_box = compute_torque(force_box, closest_point_box - pos_box)
        for i, (b, s) in enumerate(b_s):
            self.update_env_forces(b, force_box[:, i], torque_box[:, i], s, force_sphere[:, i], 0)

    def _box_line(self, b_l):  # core.py:2553-2652
        if not len(b_l):
            return
        pos_box = torch.stack([b.state.pos for b, _ in b_l], dim=-2)
        pos_line = torch.stack([l.state.pos for _, l in b_l], dim=-2)
        rot_box = torch.stack([b.state.rot for b, _ in b_l], dim=-2)
        rot_line = torch.stack([l.state.rot for _, l in b_l], dim=-2)
        length_box = self._t([b.shape.length for b, _ in b_l])
        width_box = self._t([b.shape.width for b, _ in b_l])
        not_hollow_prior = torch.stack([torch.tensor(not b.shape.hollow) for b, _ in b_l], dim=-1)
        not_hollow = not_hollow_prior.unsqueeze(0).expand(self.batch_dim, -1)
        length_line = self._t([l.shape.length for _, l in b_l])
        point_box, point_line = get_closest_line_box(pos_box, rot_box, width_box, length_box, pos_line, rot_line,
                                                     length_line)
        inner_point_box = point_box
        d = torch.zeros_like(length_line, dtype=torch.float)
        if not_hollow_prior.any():
            inner_hollow, d_hollow = get_inner_point_box(point_line, point_box, pos_box)
            cond = not_hollow.unsqueeze(-1).expand(inner_point_box.shape)
            inner_point_box = torch.where(cond, inner_hollow, inner_point_box)
            d = torch.where(not_hollow, d_hollow, d)
        force_box, force_line = self._get_constraint_forces(
            inner_point_box, point_line, dist_min=LINE_MIN_DIST + d, force_multiplier=self._collision_force)
        torque_box = compute_torque(force_box, point_box - pos_box)
        torque_line = compute_torque(force_line, point_line - pos_line)
        for i, (b, l) in enumerate(b_l):
            self.update_env_forces(b, force_box[:, i], torque_box[:, i], l, force_line[:, i], torque_line[:, i])

    def _box_box(self, b_b):  # core.py:2654-2785
        if not len(b_b):
            return
        pos_box = torch.stack([a.state.pos for a, _ in b_b], dim=-2)
        rot_box = torch.stack([a.state.rot for a, _ in b_b], dim=-2)
        length_box = self._t([a.shape.length for a, _ in b_b])
        width_box = self._t([a.shape.width for a, _ in b_b])
        nh_prior = torch.stack([torch.tensor(not a.shape.hollow) for a, _ in b_b], dim=-1)
        nh = nh_prior.unsqueeze(0).expand(self.batch_dim, -1)
        pos_box2 = torch.stack([b.state.pos for _, b in b_b], dim=-2)
        rot_box2 = torch.stack([b.state.rot for _, b in b_b], dim=-2)
        length_box2 = self._t([b.shape.length for _, b in b_b])
        width_box2 = self._t([b.shape.width for _, b in b_b])
        nh2_prior = torch.stack([torch.tensor(not b.shape.hollow) for _, b in b_b], dim=-1)
        nh2 = nh2_prior.unsqueeze(0).expand(self.batch_dim, -1)
        point_a, point_b = get_closest_box_box(pos_box, rot_box, width_box, length_box, pos_box2, rot_box2,
                                               width_box2, length_box2)
        inner_a, d_a = point_a, torch.zeros_like(length_box, dtype=torch.float)
        if nh_prior.any():
            ih, dh = get_inner_point_box(point_b, point_a, pos_box)
            inner_a = torch.where(nh.unsqueeze(-1).expand(inner_a.shape), ih, inner_a)
            d_a = torch.where(nh, dh, d_a)
        inner_b, d_b = point_b, torch.zeros_like(length_box2, dtype=torch.float)
        if nh2_prior.any():
            ih2, dh2 = get_inner_point_box(point_a, point_b, pos_box2)
            inner_b = torch.where(nh2.unsqueeze(-1).expand(inner_b.shape), ih2, inner_b)
            d_b = torch.where(nh2, dh2, d_b)
        force_a, force_b = self._get_constraint_forces(inner_a, inner_b, dist_min=d_a + d_b + LINE_MIN_DIST,
                                                       force_multiplier=self._collision_force)
        torque_a = compute_torque(force_a, point_a - pos_box)
        torque_b = compute_torque(force_b, point_b - pos_box2)
        for i, (a, b) in enumerate(b_b):
            self.update_env_forces(a, force_a[:, i], torque_a[:, i], b, force_b[:, i], torque_b[:, i])

    def _get_constraint_forces(self, pos_a, pos_b, dist_min, force_multiplier, attractive=False):  # 2804-2838
        min_dist = 1e-6
        delta_pos = pos_a - pos_b
        dist = torch.linalg.vector_norm(delta_pos, dim=-1)
        sign = -1 if attractive else 1
        k = self._contact_margin
        penetration = torch.logaddexp(torch.tensor(0.0, dtype=torch.float32), (dist_min - dist) * sign / k) * k
        force = sign * force_multiplier * delta_pos / torch.where(dist > 0, dist, 1e-8).unsqueeze(-1) * penetration.unsqueeze(-1)
        force = torch.where((dist < min_dist).unsqueeze(-1), 0.0, force)
        with torch.no_grad():
            m = torch.minimum((dist - dist_min).abs(), (dist - min_dist).abs()).reshape(dist.shape[0], -1)
            self.cutoff_margin = torch.minimum(self.cutoff_margin, m.amin(-1).nan_to_num(float("inf")))
        if not attractive:
            force = torch.where((dist > dist_min).unsqueeze(-1), 0.0, force)
        else:
            force = torch.where((dist < dist_min).unsqueeze(-1), 0.0, force)
        return force, -force

    def _get_constraint_torques(self, rot_a, rot_b, force_multiplier):  # core.py:2840-2857
        min_delta_rot = 1e-9
        delta_rot = rot_a - rot_b
        abs_delta_rot = torch.linalg.vector_norm(delta_rot, dim=-1).unsqueeze(-1)
        k = 1
        penetration = k * (torch.exp(abs_delta_rot / k) - 1)
        torque = force_multiplier * delta_rot.sign() * penetration
        torque = torch.where((abs_delta_rot < min_delta_rot), 0.0, torque)
        return -torque, torque

    def _integrate_state(self, entity, substep):  # core.py:2859-2907
        if entity.movable:
            if substep == 0:
                drag = entity.drag if entity.drag is not None else self._drag
                entity.state.vel = entity.state.vel * (1 - drag)
            accel = self.forces_dict[entity] / entity.mass
            entity.state.vel = entity.state.vel + accel * self._sub_dt
            if entity.max_speed is not None:
                entity.state.vel = clamp_with_norm(entity.state.vel, entity.max_speed)
            if entity.v_range is not None:
                entity.state.vel = entity.state.vel.clamp(-entity.v_range, entity.v_range)
            new_pos = entity.state.pos + entity.state.vel * self._sub_dt
            entity.state.pos = torch.stack(
                [
                    new_pos[..., X].clamp(-self._x_semidim, self._x_semidim) if self._x_semidim is not None else new_pos[..., X],
                    new_pos[..., Y].clamp(-self._y_semidim, self._y_semidim) if self._y_semidim is not None else new_pos[..., Y],
                ],
                dim=-1,
            )
        if entity.rotatable:
            if substep == 0:
                drag = entity.drag if entity.drag is not None else self._drag
                entity.state.ang_vel = entity.state.ang_vel * (1 - drag)
            entity.state.ang_vel = entity.state.ang_vel + (self.torques_dict[entity] / entity.moment_of_inertia) * self._sub_dt
            entity.state.rot = entity.state.rot + entity.state.ang_vel * self._sub_dt

    def result(self) -> Dict[int, dict]:
        out = {}
        for i, e in enumerate(self.ents):
            out[i] = {k: getattr(e.state, k) for k in ("pos", "vel", "rot", "ang_vel", "force", "torque")
                      if hasattr(e.state, k)}
        return out

    # ---- ray casting (core.py:1280-1785) ---------------------------------------------------------
    def _cast_rays_to_box(self, box_pos, box_rot, box_length, box_width, ray_origin, ray_direction, max_range):
        batch_size = ray_origin.shape[:-1]
        num_angles = ray_direction.shape[-1]
        n_boxes = box_pos.shape[-2]
        ray_origin = ray_origin.unsqueeze(-2).unsqueeze(-2).expand(*batch_size, n_boxes, num_angles, 2)
        box_pos_expanded = box_pos.unsqueeze(-2).expand(*batch_size, n_boxes, num_angles, 2)
        ray_direction = ray_direction.unsqueeze(-2).expand(*batch_size, n_boxes, num_angles)
        box_rot_expanded = box_rot.unsqueeze(-1).expand(*batch_size, n_boxes, num_angles)
        box_width_expanded = box_width.unsqueeze(-1).expand(*batch_size, n_boxes, num_angles)
        box_length_expanded = box_length.unsqueeze(-1).expand(*batch_size, n_boxes, num_angles)
        pos_origin = ray_origin - box_pos_expanded
        pos_aabb = rotate_vector(pos_origin, -box_rot_expanded)
        ray_dir_world = torch.stack([torch.cos(ray_direction), torch.sin(ray_direction)], dim=-1)
        ray_dir_aabb = rotate_vector(ray_dir_world, -box_rot_expanded)
        tx1 = (-box_length_expanded / 2 - pos_aabb[..., X]) / ray_dir_aabb[..., X]
        tx2 = (box_length_expanded / 2 - pos_aabb[..., X]) / ray_dir_aabb[..., X]
        tx = torch.stack([tx1, tx2], dim=-1)
        tmin, _ = torch.min(tx, dim=-1)
        tmax, _ = torch.max(tx, dim=-1)
        ty1 = (-box_width_expanded / 2 - pos_aabb[..., Y]) / ray_dir_aabb[..., Y]
        ty2 = (box_width_expanded / 2 - pos_aabb[..., Y]) / ray_dir_aabb[..., Y]
        ty = torch.stack([ty1, ty2], dim=-1)
        tymin, _ = torch.min(ty, dim=-1)
        tymax, _ = torch.max(ty, dim=-1)
        tmin, _ = torch.max(torch.stack([tmin, tymin], dim=-1), dim=-1)
        tmax, _ = torch.min(torch.stack([tmax, tymax], dim=-1), dim=-1)
        intersect_aabb = tmin.unsqueeze(-1) * ray_dir_aabb + pos_aabb
        intersect_world = rotate_vector(intersect_aabb, box_rot_expanded) + box_pos_expanded
        collision = (tmax >= tmin) & (tmin > 0.0)
        dist = torch.linalg.norm(ray_origin - intersect_world, dim=-1)
        return self._miss(dist, ~collision, max_range)

    def _cast_rays_to_sphere(self, sphere_pos, sphere_radius, ray_origin, ray_direction, max_range):
        batch_size = ray_origin.shape[:-1]
        num_angles = ray_direction.shape[-1]
        n_spheres = sphere_pos.shape[-2]
        ray_origin = ray_origin.unsqueeze(-2).unsqueeze(-2).expand(*batch_size, n_spheres, num_angles, 2)
        sphere_pos_expanded = sphere_pos.unsqueeze(-2).expand(*batch_size, n_spheres, num_angles, 2)
        ray_direction = ray_direction.unsqueeze(-2).expand(*batch_size, n_spheres, num_angles)
        sphere_radius_expanded = sphere_radius.unsqueeze(-1).expand(*batch_size, n_spheres, num_angles)
        ray_dir_world = torch.stack([torch.cos(ray_direction), torch.sin(ray_direction)], dim=-1)
        line_rot = ray_direction.unsqueeze(-1)
        line_length = max_range
        line_pos = ray_origin + ray_dir_world * (line_length / 2)
        closest_point = get_closest_point_line(line_pos, line_rot, line_length, sphere_pos_expanded,
                                               limit_to_line_length=False)
        d = sphere_pos_expanded - closest_point
        d_norm = torch.linalg.vector_norm(d, dim=-1)
        ray_intersects = d_norm < sphere_radius_expanded
        a = sphere_radius_expanded**2 - d_norm**2
        m = torch.sqrt(torch.where(a > 0, a, 1e-8))
        u = sphere_pos_expanded - ray_origin
        u1 = closest_point - ray_origin
        u_dot_ray = (u * ray_dir_world).sum(-1)
        sphere_is_in_front = u_dot_ray > 0.0
        dist = torch.linalg.vector_norm(u1, dim=-1) - m
        return self._miss(dist, ~(ray_intersects & sphere_is_in_front), max_range)

    def _cast_rays_to_line(self, line_pos, line_rot, line_length, ray_origin, ray_direction, max_range):
        batch_size = ray_origin.shape[:-1]
        num_angles = ray_direction.shape[-1]
        n_lines = line_pos.shape[-2]
        ray_origin = ray_origin.unsqueeze(-2).unsqueeze(-2).expand(*batch_size, n_lines, num_angles, 2)
        line_pos_expanded = line_pos.unsqueeze(-2).expand(*batch_size, n_lines, num_angles, 2)
        ray_direction = ray_direction.unsqueeze(-2).expand(*batch_size, n_lines, num_angles)
        line_rot_expanded = line_rot.unsqueeze(-1).expand(*batch_size, n_lines, num_angles)
        line_length_expanded = line_length.unsqueeze(-1).expand(*batch_size, n_lines, num_angles)
        r = torch.stack([torch.cos(line_rot_expanded), torch.sin(line_rot_expanded)], dim=-1) * line_length_expanded.unsqueeze(-1)
        q = ray_origin
        s = torch.stack([torch.cos(ray_direction), torch.sin(ray_direction)], dim=-1)
        rxs = cross(r, s)
        t = cross(q - line_pos_expanded, s / rxs)
        u = cross(q - line_pos_expanded, r / rxs)
        d = torch.linalg.norm(u * s, dim=-1)
        for miss in ((rxs == 0.0), (t > 0.5), (t < -0.5), (u < 0.0)):
            d = self._miss(d, miss.squeeze(-1), max_range)
        return d

    def _miss(self, d, miss, max_range):
        """``d[miss] = max_range`` (the reference's in-place write), or its torch.where form."""
        if self.grad_safe:
            return torch.where(miss, torch.tensor(max_range, dtype=d.dtype), d)
        d[miss] = max_range
        return d

    def cast_rays(self, entity_index: int, angles: Tensor, max_range: float, entity_filter):
        entity = self.ents[entity_index]
        pos = entity.state.pos
        dists = torch.full_like(angles, fill_value=max_range).unsqueeze(-1)
        boxes, spheres, lines = [], [], []
        for e in self.ents:
            if entity is e or not entity_filter(e.e):
                continue
            k = _kind(e.shape)
            (boxes if k == "Box" else spheres if k == "Sphere" else lines).append(e)
        B = self.batch_dim
        if len(boxes):
            d = self._cast_rays_to_box(
                torch.stack([b.state.pos for b in boxes], dim=-2), torch.stack([b.state.rot for b in boxes], dim=-2).squeeze(-1),
                torch.stack([torch.tensor(b.shape.length) for b in boxes], dim=-1).unsqueeze(0).expand(B, -1),
                torch.stack([torch.tensor(b.shape.width) for b in boxes], dim=-1).unsqueeze(0).expand(B, -1),
                pos, angles, max_range)
            dists = torch.cat([dists, d.transpose(-1, -2)], dim=-1)
        if len(spheres):
            d = self._cast_rays_to_sphere(
                torch.stack([s.state.pos for s in spheres], dim=-2),
                torch.stack([torch.tensor(s.shape.radius) for s in spheres], dim=-1).unsqueeze(0).expand(B, -1),
                pos, angles, max_range)
            dists = torch.cat([dists, d.transpose(-1, -2)], dim=-1)
        if len(lines):
            d = self._cast_rays_to_line(
                torch.stack([l.state.pos for l in lines], dim=-2), torch.stack([l.state.rot for l in lines], dim=-2).squeeze(-1),
                torch.stack([torch.tensor(l.shape.length) for l in lines], dim=-1).unsqueeze(0).expand(B, -1),
                pos, angles, max_range)
            dists = torch.cat([dists, d.transpose(-1, -2)], dim=-1)
        dist, _ = torch.min(dists, dim=-1)
        return dist

    # ---- distance queries (core.py:1787-1968) ----------------------------------------------------
    def get_distance_from_point(self, entity, test_point_pos):
        k = _kind(entity.shape)
        if k == "Sphere":
            return torch.linalg.vector_norm(entity.state.pos - test_point_pos, dim=-1) - entity.shape.radius
        if k == "Box":
            cp = get_closest_point_box(entity.state.pos, entity.state.rot, entity.shape.width, entity.shape.length,
                                       test_point_pos)
            return torch.linalg.vector_norm(test_point_pos - cp, dim=-1) - LINE_MIN_DIST
        cp = get_closest_point_line(entity.state.pos, entity.state.rot, entity.shape.length, test_point_pos)
        return torch.linalg.vector_norm(test_point_pos - cp, dim=-1) - LINE_MIN_DIST

    def get_distance(self, a, b):
        ka, kb = _kind(a.shape), _kind(b.shape)
        if ka == "Sphere" and kb == "Sphere":
            return self.get_distance_from_point(a, b.state.pos) - b.shape.radius
        if {ka, kb} == {"Box", "Sphere"}:
            box, sphere = (a, b) if kb == "Sphere" else (b, a)
            rv = self.get_distance_from_point(box, sphere.state.pos) - sphere.shape.radius
            rv[self.is_overlapping(a, b)] = -1
            return rv
        if {ka, kb} == {"Line", "Sphere"}:
            line, sphere = (a, b) if kb == "Sphere" else (b, a)
            return self.get_distance_from_point(line, sphere.state.pos) - sphere.shape.radius
        if ka == "Line" and kb == "Line":
            pa, pb = get_closest_points_line_line(a.state.pos, a.state.rot, a.shape.length, b.state.pos, b.state.rot,
                                                  b.shape.length)
            return torch.linalg.vector_norm(pa - pb, dim=1) - LINE_MIN_DIST
        if {ka, kb} == {"Box", "Line"}:
            box, line = (a, b) if kb == "Line" else (b, a)
            pb_, pl = get_closest_line_box(box.state.pos, box.state.rot, box.shape.width, box.shape.length,
                                           line.state.pos, line.state.rot, line.shape.length)
            return torch.linalg.vector_norm(pb_ - pl, dim=1) - LINE_MIN_DIST
        pa, pb = get_closest_box_box(a.state.pos, a.state.rot, a.shape.width, a.shape.length, b.state.pos,
                                     b.state.rot, b.shape.width, b.shape.length)
        return torch.linalg.vector_norm(pa - pb, dim=-1) - LINE_MIN_DIST

    def is_overlapping(self, a, b):
        ka, kb = _kind(a.shape), _kind(b.shape)
        if {ka, kb} == {"Box", "Sphere"}:
            box, sphere = (a, b) if kb == "Sphere" else (b, a)
            cp = get_closest_point_box(box.state.pos, box.state.rot, box.shape.width, box.shape.length,
                                       sphere.state.pos)
            d_sc = torch.linalg.vector_norm(sphere.state.pos - cp, dim=-1)
            d_sb = torch.linalg.vector_norm(sphere.state.pos - box.state.pos, dim=-1)
            d_cb = torch.linalg.vector_norm(box.state.pos - cp, dim=-1)
            return (d_sb < d_cb) + (d_sc < sphere.shape.radius + LINE_MIN_DIST)
        return self.get_distance(a, b) < 0


# ------------------------------------------------------------------------------------------------
# conveniences for tests / smoke / bench
def oracle_step(world, snap=None, broadphase: str = "batch"):
    """Reference World.step on CPU copies of ``world``'s state; returns (new_snap, OracleWorld)."""
    if snap is None:
        snap = snapshot(world)
    ow = OracleWorld(world, {i: {k: v.clone() for k, v in d.items()} for i, d in snap.items()}, broadphase)
    ow.step()
    return ow.result(), ow


def load_snapshot(world, snap: Dict[int, dict]) -> None:
    """Teacher forcing: write a snapshot into ``world``'s entities (on the world's device)."""
    dev = world.device
    for i, e in enumerate(world.entities):
        s = e.state
        for k, v in snap[i].items():
            setattr(s, "_" + k, v.to(dev).clone())


def sensitivity_band(world, snap, expected, broadphase="batch", n=2, eps=1.2e-7, seed=1234):
    """Per-element fp32 conditioning of one step: max |oracle(perturbed) - oracle| over ``n``
    random relative input perturbations of ~1 ulp (eps = 2**-23).  A stiff system (joints, tiny
    inertias) amplifies last-bit differences; the parity tolerance must include that band."""
    g = torch.Generator().manual_seed(seed)
    band = {i: {k: torch.zeros_like(v) for k, v in d.items()} for i, d in expected.items()}
    for _ in range(n):
        pert = {i: {k: v * (1 + eps * torch.randn(v.shape, generator=g)) for k, v in d.items()}
                for i, d in snap.items()}
        out, _ = oracle_step(world, pert, broadphase)
        for i in band:
            for k in band[i]:
                band[i][k] = torch.maximum(band[i][k], (out[i][k] - expected[i][k]).abs().nan_to_num(0.0))
    return band


# Stated fp32 tolerance of one teacher-forced step: |got - expected| <=
#   atol (1e-5 on pos/rot, 1e-4 on vel/ang_vel/force/torque) + rtol 1e-4 * |expected|
#   + 4 x the oracle's own 1-ulp sensitivity band (when provided)
# An environment outside it passes only when it is CERTIFIED to sit on a contact cut-off: the
# soft contact force is discontinuous at dist == dist_min (and dist == 1e-6), so a last-bit
# difference in dist switches a force of ~c * k * log 2 on or off.  ``cutoff`` is the oracle's
# per-env smallest |dist - cut-off| over every contact evaluation of the step
# (OracleWorld.cutoff_margin); an env is certified when it is <= ``cutoff_tol``: 4e-6, i.e.
# a few tens of fp32 ulps at the configs' contact distances (0.05-0.3), which covers the
# last-bit state drift of up to 10 substeps before the crossing.  A certified env's error is
# still BOUNDED (``cutoff_bound``): by what contact switches can change in one step -- each of an
# entity's (E - 1) pairs toggling a force of c * k * log 2 (the soft force at dist == dist_min)
# in each of the S substeps, twice over:
#   vel     <= 2 S (E-1) c k log2 sub_dt / m_min          pos <= vel bound * dt
#   ang_vel <= 2 S (E-1) c k log2 lever sub_dt / I_min    rot <= ang_vel bound * dt
# (lever = the largest circumscribed radius; agent force / torque: no contact term, tolerance
# only).  ``max_bad_frac`` (default 0) additionally allows uncertified envs (kept for callers
# that opt in; no test does).
CUTOFF_TOL = 4e-6
BAND_RETRY_N = 16  # perturbations of the second band estimate (compare_one_step)


def cutoff_bound(world) -> Dict[str, float]:
    """Per-field bound of a certified cut-off env's error (see CUTOFF_TOL)."""
    ents = world.entities
    dyn = [e for e in ents if e.movable or e.rotatable]
    if not dyn:
        return {}
    f_jump = float(world._collision_force) * float(world._contact_margin) * math.log(2.0)
    S, sdt = int(world._substeps), float(world._sub_dt)
    dt = S * sdt
    pairs = max(len(ents) - 1, 1)
    m_min = min(float(e.mass) for e in dyn)
    rot = [e for e in ents if e.rotatable]
    i_min = min(float(e.moment_of_inertia) for e in rot) if rot else 1.0
    lever = max(float(_circ_radius(e.shape)) for e in ents)
    v = 2 * S * pairs * f_jump * sdt / m_min
    w = 2 * S * pairs * f_jump * lever * sdt / i_min
    return {"vel": v, "pos": v * dt, "ang_vel": w, "rot": w * dt, "force": 0.0, "torque": 0.0}


def _circ_radius(shape) -> float:
    k = _kind(shape)
    if k == "Sphere":
        return shape.radius
    if k == "Box":
        return math.sqrt((shape.length / 2) ** 2 + (shape.width / 2) ** 2)
    return shape.length / 2


def compare(a: Dict[int, dict], b: Dict[int, dict], world=None, atol_pos=1e-5, atol_vel=1e-4, rtol=1e-4,
            band=None, band_factor=4.0, max_bad_frac=0.0, cutoff=None, cutoff_tol=CUTOFF_TOL):
    """Engine result ``a`` vs oracle result ``b`` under the stated tolerance (see CUTOFF_TOL).
    ``cutoff`` (per-env margins) enables certification; a certified env must still stay within
    ``cutoff_bound(world)`` + the tolerance.  The report carries the numbers a reader needs:
    bad / uncertified envs, the largest cut-off margin among certified envs, the largest error of
    a certified env as a fraction of its bound, max |diff| and the band's max per field."""
    worst, band_max = {}, {}
    env_err: Dict[str, torch.Tensor] = {}  # per field: per-env max |diff| over entities / components
    bad_envs = None
    excess = []  # per field: (diff - tol) / bound per env, for the certification bound
    bound = cutoff_bound(world) if (world is not None and cutoff is not None) else {}
    for i in a:
        for k, va in a[i].items():
            vb = b[i][k].to(va.device)
            diff = (va - vb).abs()
            if diff.numel():
                e = diff.nan_to_num(float("inf")).reshape(diff.shape[0], -1).amax(-1)
                env_err[k] = e if k not in env_err else torch.maximum(env_err[k], e)
            tol = (atol_pos if k in ("pos", "rot") else atol_vel) + rtol * vb.abs()
            if band is not None:
                tol = tol + band_factor * band[i][k]
                band_max[k] = max(band_max.get(k, 0.0), float(band[i][k].max()) if band[i][k].numel() else 0.0)
            nan_mis = torch.isnan(va).ne(torch.isnan(vb))
            bad = (diff > tol) | nan_mis
            bad = bad.reshape(bad.shape[0], -1).any(-1)
            bad_envs = bad if bad_envs is None else (bad_envs | bad)
            if bound:
                over = (diff - tol).clamp_min(0.0).nan_to_num(float("inf"))
                over = torch.where(nan_mis, torch.full_like(over, float("inf")), over)
                over = over.reshape(over.shape[0], -1).amax(-1)
                bk = bound.get(k, 0.0)
                excess.append(over / bk if bk > 0 else torch.where(over > 0, float("inf"), 0.0))
            m = float(diff.nan_to_num(0.0).max()) if diff.numel() else 0.0
            name = world.entities[i].name if world is not None else str(i)
            if m > worst.get(k, (0.0, ""))[0]:
                worst[k] = (m, name)
    n_bad = int(bad_envs.sum()) if bad_envs is not None else 0
    n_env = int(bad_envs.numel()) if bad_envs is not None else 1
    rep = {"bad_envs": n_bad, "n_envs": n_env}
    uncertified = n_bad
    rep["certified_envs"] = 0
    if n_bad and cutoff is not None:
        idx = bad_envs.nonzero().flatten()
        margins = cutoff[idx]
        frac = torch.stack(excess).amax(0)[idx] if excess else torch.zeros(len(idx))
        cert = (margins <= cutoff_tol) & (frac <= 1.0)
        uncertified = int((~cert).sum())
        rep["certified_envs"] = int(cert.sum())
        rep["bad_env_cutoff_margins"] = [(int(i), float(m)) for i, m in zip(idx[:16], margins[:16])]
        if bool(cert.any()):
            rep["certified_max_margin"] = float(margins[cert].max())
            rep["certified_max_bound_frac"] = float(frac[cert].max())
    rep["uncertified_envs"] = uncertified
    rep["ok"] = uncertified <= max_bad_frac * n_env
    rep["max_abs"] = {k: v[0] for k, v in worst.items()}
    rep["where"] = {k: v[1] for k, v in worst.items()}
    # aggregate error over envs (a systematic error moves these; a chaotic contact env moves only
    # the max): the 99.9th percentile and the mean of the per-env max |diff|, per field
    rep["p999_abs"] = {k: float(torch.quantile(e.double(), 0.999)) for k, e in env_err.items()}
    rep["mean_abs"] = {k: float(e.double().mean()) for k, e in env_err.items()}
    if band_max:
        rep["band_max"] = band_max
    return rep


def compare_one_step(world, broadphase: str = "batch", with_band: bool = True, certify: bool = True, **tol):
    """Teacher-forced one-step parity: native engine vs this oracle from the same state.
    certify=False: no cut-off certification (a strict run: every env must be within tolerance)."""
    snap = snapshot(world)
    expected, ow = oracle_step(world, snap, broadphase)
    band = sensitivity_band(world, snap, expected, broadphase) if with_band else None
    world.broadphase = broadphase
    world.step()
    got = snapshot(world)
    rep = compare(got, expected, world, band=band, cutoff=ow.cutoff_margin if certify else None, **tol)
    if band is not None and rep["uncertified_envs"]:
        # two random 1-ulp perturbations can miss a stiff env's sensitivity: before calling an
        # env bad, estimate the oracle's band again from BAND_RETRY_N more (the band is a property
        # of the oracle at this state, not of the engine) and compare once more
        more = sensitivity_band(world, snap, expected, broadphase, n=BAND_RETRY_N, seed=98765)
        band = {i: {k: torch.maximum(band[i][k], more[i][k]) for k in band[i]} for i in band}
        rep = compare(got, expected, world, band=band, cutoff=ow.cutoff_margin if certify else None, **tol)
        rep["band_retry"] = BAND_RETRY_N
    rep["iterations"] = getattr(world.engine, "last_iterations", None)
    rep["active_pairs_per_substep"] = [len(x) for x in ow.active_log]
    return rep


def install(world) -> None:
    """Route ``world.step`` through the oracle (CPU baseline / reference-semantics runs)."""

    def step():
        world.entity_index_map = {e: i for i, e in enumerate(world.entities)}
        new, _ = oracle_step(world, snapshot(world), getattr(world, "broadphase", "batch"))
        for i, e in enumerate(world.entities):
            s = e.state
            for k, v in new[i].items():
                setattr(s, "_" + k, v)

    world.step = step


# ------------------------------------------------------------------------------------------------
# ScenarioUtils.find_random_pos_for_entity (reference vmas/simulator/utils.py:272-319), the
# reference's per-try loop (torch.cdist + torch.any host sync), for the spawn-sampler parity tests.
def find_random_pos_for_entity(occupied_positions, batch_size, device, min_dist_between_entities, x_bounds, y_bounds):
    pos = None
    while True:
        proposed_pos = torch.cat(
            [
                torch.empty((batch_size, 1, 1), device=device, dtype=torch.float32).uniform_(*x_bounds),
                torch.empty((batch_size, 1, 1), device=device, dtype=torch.float32).uniform_(*y_bounds),
            ],
            dim=2,
        )
        if pos is None:
            pos = proposed_pos
        if occupied_positions.shape[1] == 0:
            break
        dist = torch.cdist(occupied_positions, pos)
        overlaps = torch.any((dist < min_dist_between_entities).squeeze(2), dim=1)
        if torch.any(overlaps, dim=0):
            pos[overlaps] = proposed_pos[overlaps]
        else:
            break
    return pos
