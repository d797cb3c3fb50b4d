"""Bridge between the Python World and the native engine (``libvmas_mi355x.so``).

Per world it builds the static tables of the C ABI (entities, candidate pairs in the reference's
accumulation order, joints) and re-creates them whenever the world's configuration signature
changes.  Per ``World.step`` it gathers the current state tensors of every entity as raw pointers
+ strides (so views, user-replaced and in-place-mutated tensors are all read where they live),
allocates ONE fresh output buffer, calls ``vmas_world_step`` and re-points the integrated fields
of the entities at views of that buffer -- the reference's "integration creates new tensors"
semantics (core.py:2866-2907) without any copy.

Device ``cuda:i`` (ROCm) -> gfx950 kernels on the current torch stream; device ``cpu`` -> the
host backend of the same library (same arithmetic).  There is no PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import operator
import os
from typing import Callable, List

import numpy as np
import torch

from .. import _native as N
from .utils import LINE_MIN_DIST

_LMD32 = np.float32(LINE_MIN_DIST)


def _f32(x) -> float:
    return float(np.float32(x))


_SHAPE_CODES = {}  # shape type -> VMAS_* code (isinstance resolved once per type)


def _shape_code(shape) -> int:
    code = _SHAPE_CODES.get(type(shape))
    if code is not None:
        return code
    from .core import Box, Line, Sphere

    if isinstance(shape, Sphere):
        code = N.VMAS_SPHERE
    elif isinstance(shape, Box):
        code = N.VMAS_BOX
    elif isinstance(shape, Line):
        code = N.VMAS_LINE
    else:
        raise RuntimeError(f"Shape {shape} currently not handled by the engine")
    _SHAPE_CODES[type(shape)] = code
    return code


def _shape_dims(shape, code):
    if code == N.VMAS_SPHERE:
        return (shape.radius,)
    if code == N.VMAS_BOX:
        return (shape.length, shape.width)
    return (shape.length,)


_GRAD_OK = False  # the step's autograd Function is filling the tables (tensors may require grad)


def _check_grad(tensors) -> None:
    if torch.is_grad_enabled() and not _GRAD_OK:
        for t in tensors:
            if t is not None and t.requires_grad:
                raise NotImplementedError(
                    "The MI355X engine has no backward pass: World.step / cast_rays / distance "
                    "queries cannot run on tensors that require grad (grad_enabled=True)."
                )


_DEFERRED: list = []  # (destroy function, handle) of engines collected during a stream capture


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def drain_deferred() -> None:
    """Destroys the engines whose collection fell into a stream capture (call outside one)."""
    while _DEFERRED and not _capturing():
        f, h = _DEFERRED.pop()
        f(h)


class PhysicsEngine:
    def __init__(self, world):
        self.world = world
        self.lib = N.load_library()
        self._sig = None
        self._handle = None
        self._jit = None
        self._sig_cache = None  # (STATIC_VERSION, signature)
        self.jit_error = None
        self.kernel_name = "k_step"
        self._dev_index = -1
        self._qrefs = {}  # distance-query shape references, see _ref
        self._ray_tables = {}  # LIDAR target tables, see _ray_table
        self._last_iterations = 0
        self.steps = 0

    @property
    def last_iterations(self) -> int:
        """Broadphase fixed-point passes of the last step.  The specialised kernel runs them on
        the device without a host wait, so reading this waits for the step (and raises a
        device-side fixed-point failure)."""
        if self._last_iterations == 0 and self._jit is not None and self.steps:
            n = ctypes.c_int32(0)
            N.check_jit(self.lib.vmas_jit_world_passes(self._jit, ctypes.byref(n)), "vmas_jit_world_passes")
            self._last_iterations = n.value
        return self._last_iterations

    @property
    def jit_grid(self) -> int:
        """Relay grid of the specialised kernel (negative: plain launches; 0: host-driven loop)."""
        return self.lib.vmas_jit_world_grid(self._jit) if self._jit is not None else 0

    def __del__(self):
        try:
            handles = [(self.lib.vmas_world_destroy, self._handle), (self.lib.vmas_jit_world_destroy, self._jit)]
            handles = [(f, h) for f, h in handles if h is not None]
            if handles and _capturing():
                # the garbage collector can run this while a graph-mode step is being captured:
                # freeing device memory then aborts the process, so it waits for drain_deferred()
                _DEFERRED.extend(handles)
                return
            for f, h in handles:
                f(h)
        except Exception:
            pass

    # ---- device helpers ---------------------------------------------------------------------------
    def _device(self) -> torch.device:
        dev = torch.device(self.world.device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        return dev

    def _native_device(self, dev: torch.device) -> int:
        if dev.type == "cpu":
            return -1
        if dev.type == "cuda":
            return dev.index
        raise RuntimeError(f"device {dev} is not supported by the MI355X engine")

    def _stream(self, dev: torch.device):
        if dev.type == "cuda":
            return N.stream_ptr(dev.index if dev.index is not None else torch.cuda.current_device())
        return None

    def _prep(self, t: torch.Tensor, dev: torch.device) -> torch.Tensor:
        if t.device != dev or t.dtype != torch.float32:
            t = t.to(device=dev, dtype=torch.float32)
        return t

    # ---- static tables ----------------------------------------------------------------------------
    # entity attributes the static tables are built from (compared every step; any change
    # rebuilds the tables).  Gravity enters only as "has one" (its values are read per step).
    _ENTITY_SIG = operator.attrgetter(
        "_shape", "_movable", "_rotatable", "_collide", "_collision_filter", "_mass", "_drag",
        "_linear_friction", "_angular_friction", "_max_speed", "_v_range",
    )
    _AGENT_SIG = operator.attrgetter("_max_f", "_f_range", "_max_t", "_t_range")

    def _signature(self):
        # (recomputed only after an assignment to an attribute it reads: core.STATIC_VERSION)
        from . import core

        v = core.STATIC_VERSION[0]
        c = self._sig_cache
        if c is not None and c[0] == v:
            return c[1]
        sig = self._signature_now()
        self._sig_cache = (v, sig)
        return sig

    def _signature_now(self):
        w = self.world
        es = []
        for e in w.entities:
            shape = e._shape
            es.append((e, self._ENTITY_SIG(e), getattr(shape, "hollow", None), e._gravity is None,
                       self._AGENT_SIG(e) if hasattr(e, "_max_f") else None))
        js = []
        for j in w._joints.values():
            fr = j.fixed_rotation
            js.append((j, j.dist, j.rotate, fr if not isinstance(fr, torch.Tensor) else "tensor"))
        return (
            tuple(es), tuple(js), w._drag, w._linear_friction, w._angular_friction, w._x_semidim,
            w._y_semidim, w._collision_force, w._joint_force, w._torque_constraint_force,
            w._contact_margin, id(w._gravity), id(w._collidable_pairs), w.batch_dim, str(w.device),
            bool(w.export_forces),
        )

    def _build(self, sig, max_substeps: int):
        w = self.world
        dev = self._device()
        self._dev = dev
        self._dev_index = self._native_device(dev)
        ents = list(w.entities)
        E = len(ents)
        index = {id(e): i for i, e in enumerate(ents)}
        agents = [e for e in ents if hasattr(e, "_action")]
        agent_index = {id(a): i for i, a in enumerate(agents)}

        # --- candidate pairs in the reference's order (core.py:2103-2188)
        joints, ss, ls, ll, bs, bl, bb = [], [], [], [], [], [], []
        for a in range(E):
            ea = ents[a]
            for b in range(a + 1, E):
                eb = ents[b]
                jc = w._joints.get(frozenset({ea.name, eb.name}), None)
                if jc is not None:
                    joints.append(jc)
                    if jc.dist == 0:
                        continue
                if not w._collides_static(ea, eb):
                    continue
                ca, cb = _shape_code(ea.shape), _shape_code(eb.shape)
                S, B_, L = N.VMAS_SPHERE, N.VMAS_BOX, N.VMAS_LINE
                if ca == S and cb == S:
                    ss.append((ea, eb))
                elif {ca, cb} == {L, S}:
                    ls.append((ea, eb) if cb == S else (eb, ea))
                elif ca == L and cb == L:
                    ll.append((ea, eb))
                elif {ca, cb} == {B_, S}:
                    bs.append((ea, eb) if cb == S else (eb, ea))
                elif {ca, cb} == {B_, L}:
                    bl.append((ea, eb) if cb == L else (eb, ea))
                elif ca == B_ and cb == B_:
                    bb.append((ea, eb))
                else:
                    raise AssertionError()
        self.joint_list = joints
        pairs = []
        for ji, jc in enumerate(joints):
            pairs.append((N.VMAS_PAIR_JOINT, jc.entity_a, jc.entity_b, ji, 0.0, _f32(jc.dist)))

        def cr(e):
            return e.shape.circumscribed_radius()

        for ea, eb in ss:
            pairs.append((N.VMAS_PAIR_SS, ea, eb, -1, _f32(cr(ea) + cr(eb)),
                          float(np.float32(ea.shape.radius) + np.float32(eb.shape.radius))))
        for ea, eb in ls:
            pairs.append((N.VMAS_PAIR_LS, ea, eb, -1, _f32(cr(ea) + cr(eb)),
                          float(np.float32(eb.shape.radius) + _LMD32)))
        for ea, eb in ll:
            pairs.append((N.VMAS_PAIR_LL, ea, eb, -1, _f32(cr(ea) + cr(eb)), float(_LMD32)))
        for ea, eb in bs:
            pairs.append((N.VMAS_PAIR_BS, ea, eb, -1, _f32(cr(ea) + cr(eb)),
                          float(np.float32(eb.shape.radius) + _LMD32)))
        for ea, eb in bl:
            pairs.append((N.VMAS_PAIR_BL, ea, eb, -1, _f32(cr(ea) + cr(eb)), float(_LMD32)))
        for ea, eb in bb:
            pairs.append((N.VMAS_PAIR_BB, ea, eb, -1, _f32(cr(ea) + cr(eb)), float(_LMD32)))
        P = len(pairs)
        pd = (N.VmasPairDesc * max(P, 1))()
        for i, (cls, ea, eb, ji, bpr, dmin) in enumerate(pairs):
            pd[i].cls, pd[i].ea, pd[i].eb, pd[i].joint = cls, index[id(ea)], index[id(eb)], ji
            pd[i].bp_radius, pd[i].dmin = bpr, dmin
        self.pairs = pairs

        # --- joints
        jd = (N.VmasJointDesc * max(len(joints), 1))()
        for i, jc in enumerate(joints):
            da = jc.delta_anchor(jc.entity_a)
            db = jc.delta_anchor(jc.entity_b)
            jd[i].delta_a_x, jd[i].delta_a_y = _f32(da[0]), _f32(da[1])
            jd[i].delta_b_x, jd[i].delta_b_y = _f32(db[0]), _f32(db[1])
            jd[i].dist = _f32(jc.dist)
            jd[i].rotate = int(bool(jc.rotate))
            fr = jc.fixed_rotation
            if fr is None:
                raise RuntimeError("JointConstraint.fixed_rotation is None (Joint.notify never ran)")
            jd[i].fixed_rotation = 0.0 if isinstance(fr, torch.Tensor) else _f32(fr)

        # --- entities
        ed = (N.VmasEntityDesc * max(E, 1))()
        n_lin = n_rot = n_force = n_torque = 0
        self.lin_slots, self.rot_slots, self.force_slots, self.torque_slots = [], [], [], []
        for i, e in enumerate(ents):
            d = ed[i]
            d.shape = _shape_code(e.shape)
            flags = 0
            if e.movable:
                flags |= N.F_MOVABLE
            if e.rotatable:
                flags |= N.F_ROTATABLE
            if d.shape == N.VMAS_BOX and e.shape.hollow:
                flags |= N.F_HOLLOW
            is_agent = id(e) in agent_index
            d.agent_index = agent_index[id(e)] if is_agent else -1
            d.out_lin = d.out_rot = d.out_force = d.out_torque = -1
            if e.movable:
                d.out_lin = n_lin
                self.lin_slots.append(e)
                n_lin += 1
            if e.rotatable:
                d.out_rot = n_rot
                self.rot_slots.append(e)
                n_rot += 1
            if is_agent:
                flags |= N.F_AGENT
                if e.movable and (e.max_f is not None or e.f_range is not None):
                    d.out_force = n_force
                    self.force_slots.append(e)
                    n_force += 1
                if e.rotatable and (e.max_t is not None or e.t_range is not None):
                    d.out_torque = n_torque
                    self.torque_slots.append(e)
                    n_torque += 1
                if e.max_f is not None:
                    flags |= N.F_MAX_F
                    d.max_f = _f32(e.max_f)
                if e.f_range is not None:
                    flags |= N.F_F_RANGE
                    d.f_range = _f32(e.f_range)
                if e.max_t is not None:
                    flags |= N.F_MAX_T
                    d.max_t = _f32(e.max_t)
                if e.t_range is not None:
                    flags |= N.F_T_RANGE
                    d.t_range = _f32(e.t_range)
            if d.shape == N.VMAS_SPHERE:
                d.radius = _f32(e.shape.radius)
            else:
                d.half_length = float(np.float32(e.shape.length) / np.float32(2))
                if d.shape == N.VMAS_BOX:
                    d.half_width = float(np.float32(e.shape.width) / np.float32(2))
            d.mass = _f32(e.mass)
            d.inertia = _f32(e.moment_of_inertia)
            drag = e.drag if e.drag is not None else w._drag
            d.one_minus_drag = _f32(1 - drag)
            if e.linear_friction is not None:
                flags |= N.F_LIN_FRIC
                d.lin_fric = _f32(e.linear_friction)
            elif w._linear_friction > 0:
                flags |= N.F_LIN_FRIC
                d.lin_fric = _f32(w._linear_friction)
            if e.angular_friction is not None:
                flags |= N.F_ANG_FRIC
                d.ang_fric = _f32(e.angular_friction)
            elif w._angular_friction > 0:
                flags |= N.F_ANG_FRIC
                d.ang_fric = _f32(w._angular_friction)
            if e.max_speed is not None:
                flags |= N.F_MAX_SPEED
                d.max_speed = _f32(e.max_speed)
            if e.v_range is not None:
                flags |= N.F_V_RANGE
                d.v_range = _f32(e.v_range)
            if e.gravity is not None:
                flags |= N.F_GRAVITY
            d.flags = flags

        cfg = N.VmasWorldConfig()
        cfg.n_entities, cfg.n_agents, cfg.n_pairs, cfg.n_joints = E, len(agents), P, len(joints)
        cfg.batch = w.batch_dim
        cfg.device = self._dev_index
        cfg.n_out_lin, cfg.n_out_rot, cfg.n_out_force, cfg.n_out_torque = n_lin, n_rot, n_force, n_torque
        cfg.contact_margin = _f32(w._contact_margin)
        cfg.collision_force = _f32(w._collision_force)
        cfg.joint_force = _f32(w._joint_force)
        cfg.torque_constraint_force = _f32(w._torque_constraint_force)
        g = w._gravity.detach().to("cpu", torch.float32).reshape(-1).tolist()
        cfg.gravity_x, cfg.gravity_y = g[0], g[1]
        cfg.has_world_gravity = int(not (g[0] == 0.0 and g[1] == 0.0))
        cfg.has_x_semidim = int(w._x_semidim is not None)
        cfg.has_y_semidim = int(w._y_semidim is not None)
        cfg.x_semidim = _f32(w._x_semidim) if w._x_semidim is not None else 0.0
        cfg.y_semidim = _f32(w._y_semidim) if w._y_semidim is not None else 0.0
        cfg.max_substeps = max_substeps
        cfg.export_forces = int(bool(w.export_forces))
        # a scenario program the world module also compiles (its own kernel + k_world's epilogue;
        # set by the scenario's make_world, e.g. balance)
        # (VMAS_JIT_EPILOGUE=0: none, an A/B knob)
        cfg.epilogue = (int(getattr(w, "_jit_epilogue", N.EPILOGUE_NONE))
                        if os.environ.get("VMAS_JIT_EPILOGUE", "1") != "0" else N.EPILOGUE_NONE)
        handle = ctypes.c_void_p()
        N.check(self.lib.vmas_world_create(ctypes.byref(cfg), ed, pd, jd, ctypes.byref(handle)),
                "vmas_world_create")
        if self._handle is not None:
            self.lib.vmas_world_destroy(self._handle)
        self._handle = handle
        # GPU worlds: the world-specialised kernel (csrc/vmas_jit.hip) when it applies, with the
        # generic k_step as the fallback (both native; VMAS_JIT=0 forces the generic kernel).
        # Only parameter VALUES changed (a mass re-rolled at reset, het_mass.py:48-54; a drag, a
        # limit): the world kernel takes them as arguments -- no new code object, no compile.
        keep_jit = (self._jit is not None and max_substeps == self._max_substeps and
                    self.lib.vmas_jit_world_set_params(self._jit, ctypes.byref(cfg), ed, pd, jd) == 0)
        if self._jit is not None and not keep_jit:
            self.lib.vmas_jit_world_destroy(self._jit)
            self._jit = None
        if not keep_jit:
            self.jit_error = None
        if keep_jit:
            pass
        elif self._dev_index >= 0 and os.environ.get("VMAS_JIT", "1") != "0":
            jh = ctypes.c_void_p()
            rc = self.lib.vmas_jit_world_create(ctypes.byref(cfg), ed, pd, jd, ctypes.byref(jh))
            if rc == 0:
                self._jit = jh
            else:
                self.jit_error = self.lib.vmas_jit_last_error().decode(errors="replace")
        self.kernel_name = "k_world" if self._jit is not None else "k_step"
        self._tables = (ed, pd, jd)
        self._cfg = cfg
        self._max_substeps = max_substeps
        self.entities = ents
        self.agents = agents
        self.n_out = (n_lin, n_rot, n_force, n_torque)
        self._eio = np.zeros(E, dtype=N.ENTITY_IO_DTYPE)
        self._eio_f = {k: self._eio[k] for k in N.ENTITY_IO_DTYPE.names}  # field views
        # per entity: the state tensors last seen ([pos, vel, rot, ang_vel, gravity], identity
        # checked every step) and the converted tensors its pointer-table row points at
        self._ent_seen = [None] * E
        self._ent_keep = [None] * E
        self._agent_seen = [None] * len(agents)
        self._agent_keep = [None] * len(agents)
        B = w.batch_dim
        # one output buffer per step: every (B, 2) field first ([pos x n_lin | vel x n_lin |
        # force x n_force]), then every (B, 1) field ([rot x n_rot | ang_vel x n_rot | torque x
        # n_torque]), so two strided views + unbind give all the new state tensors
        n2, n1 = 2 * n_lin + n_force, 2 * n_rot + n_torque
        self._n2, self._n1 = n2, n1
        self._out_numel = max(n2 * B * 2 + n1 * B, 1)
        self._out_off = (0, n_lin * B * 2, n2 * B * 2, n2 * B * 2 + n_rot * B, 2 * n_lin * B * 2,
                         n2 * B * 2 + 2 * n_rot * B)  # floats: pos, vel, rot, ang, force, torque
        self._lin_rows = np.array([index[id(e)] for e in self.lin_slots], dtype=np.int64)
        self._rot_rows = np.array([index[id(e)] for e in self.rot_slots], dtype=np.int64)
        self._lin_slot_bytes = np.arange(len(self.lin_slots), dtype=np.uint64) * np.uint64(8 * B)
        self._rot_slot_bytes = np.arange(len(self.rot_slots), dtype=np.uint64) * np.uint64(4 * B)
        self._lin_idx = [index[id(e)] for e in self.lin_slots]
        self._rot_idx = [index[id(e)] for e in self.rot_slots]
        self._aio = np.zeros(max(len(agents), 1), dtype=N.AGENT_IO_DTYPE)
        self._aio_f = {k: self._aio[k] for k in N.AGENT_IO_DTYPE.names}
        self._jio = np.zeros(max(len(joints), 1), dtype=N.JOINT_IO_DTYPE)
        self._io = N.VmasStepIO()
        self._io.entities, self._io.agents, self._io.joints = (
            self._eio.ctypes.data, self._aio.ctypes.data, self._jio.ctypes.data)
        self._step_params = None
        self._sig = sig

    # ---- kernel timing (bench.py roofline) --------------------------------------------------------
    def set_timing(self, enable: bool) -> None:
        self._ensure()
        self._timing = bool(enable)
        self._apply_timing()

    def _apply_timing(self):
        on = int(getattr(self, "_timing", False))
        N.check(self.lib.vmas_world_set_timing(self._handle, on), "vmas_world_set_timing")
        if self._jit is not None:
            N.check_jit(self.lib.vmas_jit_world_set_timing(self._jit, on), "vmas_jit_world_set_timing")

    def device_timing(self, reset: bool = True, with_clock: bool = False):
        """(milliseconds, launches[, shader clock GHz]) of the specialised step kernel from its
        in-kernel device timer (vmas_jit_world_device_timing): the timer of launches replayed from
        a HIP graph, and the clock the chip held inside the kernel."""
        ms = ctypes.c_double(0.0)
        n = ctypes.c_int64(0)
        ghz = ctypes.c_double(0.0)
        if self._jit is not None:
            N.check_jit(self.lib.vmas_jit_world_device_timing(self._jit, int(reset), ctypes.byref(ms),
                                                              ctypes.byref(n), ctypes.byref(ghz)),
                        "vmas_jit_world_device_timing")
        return (ms.value, n.value, ghz.value) if with_clock else (ms.value, n.value)

    def check_device_errors(self) -> None:
        """Raise a device-side fixed-point failure reported by any launch so far, without waiting
        (graph replays do not pass through vmas_jit_world_step's own check)."""
        if self._jit is not None:
            N.check_jit(self.lib.vmas_jit_world_check(self._jit), "vmas_jit_world_check")

    def graph_token(self):
        """What a captured step depends on besides tensor contents: the static tables (entity /
        joint / world parameters), the kernel object and the step parameters."""
        w = self.world
        return (self._signature(), int(w._substeps), w._sub_dt, w.broadphase, id(self._jit), id(self._handle))

    def get_timing(self, reset: bool = True):
        """(milliseconds, launches) of the step kernel (k_world or k_step) since the last reset."""
        ms = ctypes.c_double(0.0)
        n = ctypes.c_int64(0)
        if self._jit is not None:
            N.check_jit(self.lib.vmas_jit_world_get_timing(self._jit, int(reset), ctypes.byref(ms), ctypes.byref(n)),
                        "vmas_jit_world_get_timing")
        else:
            N.check(self.lib.vmas_world_get_timing(self._handle, int(reset), ctypes.byref(ms), ctypes.byref(n)),
                    "vmas_world_get_timing")
        return ms.value, n.value

    def jit_source(self) -> str:
        """Generated source of the world-specialised kernel ('' when the generic kernel runs)."""
        self._ensure()
        if self._jit is None:
            return ""
        n = self.lib.vmas_jit_world_source(self._jit, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        self.lib.vmas_jit_world_source(self._jit, buf, n + 1)
        return buf.value.decode()

    def jit_profile(self):
        """Phase timestamps [max_substeps*4 + 2, 16 wave columns] of the profiled workgroup
        (VMAS_JIT_PROFILE); columns past the kernel's wave count stay 0."""
        if self._jit is None:
            return None
        n = self.lib.vmas_jit_world_profile(self._jit, None, 0)
        N.check_jit(n, "vmas_jit_world_profile")
        if n == 0:
            return None
        out = np.zeros(n, dtype=np.uint64)
        N.check_jit(self.lib.vmas_jit_world_profile(self._jit, out.ctypes.data, n), "vmas_jit_world_profile")
        return out.reshape(-1, 16)

    def jit_program(self, kind: int):
        """The world module's handle when it was compiled with scenario program `kind`
        (N.EPILOGUE_*; csrc/vmas_jit.hip), else None (no module, a CPU world, another program)."""
        if self._dev_index < 0:
            return None
        self._ensure()
        if self._jit is None or self.lib.vmas_jit_world_epilogue(self._jit) != kind:
            return None
        return self._jit

    def jit_compile_check(self) -> str:
        """Generate and hipRTC-compile this world's specialised kernel without a device (build
        check on CPU machines); returns the generated source, raises on failure."""
        self._ensure()
        ed, pd, jd = self._tables
        n = self.lib.vmas_jit_compile_check(ctypes.byref(self._cfg), ed, pd, jd, None, 0)
        N.check_jit(n, "vmas_jit_compile_check")
        buf = ctypes.create_string_buffer(n + 1)
        self.lib.vmas_jit_compile_check(ctypes.byref(self._cfg), ed, pd, jd, buf, n + 1)
        return buf.value.decode()

    def _ensure(self):
        sub = int(self.world._substeps)
        sig = self._signature()
        if sig != self._sig or self._handle is None or sub > self._max_substeps:
            self._build(sig, max(sub, 16))
            if getattr(self, "_timing", False):
                self._apply_timing()

    # ---- the step ---------------------------------------------------------------------------------
    def _fill_entity_row(self, i, e, dev, B):
        """(Re)read entity i's state tensors into its pointer-table row; remember them by identity."""
        st = e._state
        orig = [st._pos, st._vel, st._rot, st._ang_vel, e._gravity]
        _check_grad(orig[:4])
        pos, vel, rot, ang = (self._prep(t, dev) for t in orig[:4])
        f = self._eio_f
        ps, vs = pos.stride(), vel.stride()
        f["pos"][i], f["vel"][i], f["rot"][i], f["ang"][i] = pos.data_ptr(), vel.data_ptr(), rot.data_ptr(), ang.data_ptr()
        f["pos_s0"][i], f["pos_s1"][i], f["vel_s0"][i], f["vel_s1"][i] = ps[0], ps[1], vs[0], vs[1]
        f["rot_s0"][i], f["ang_s0"][i] = rot.stride(0), ang.stride(0)
        g = orig[4]
        if g is not None:
            g = self._prep(g, dev).expand(B, 2)
            f["grav"][i] = g.data_ptr()
            f["grav_s0"][i], f["grav_s1"][i] = g.stride(0), g.stride(1)
        else:
            f["grav"][i] = 0
        # keep the converted tensors alive as long as the row points at them
        self._ent_seen[i] = orig
        self._ent_keep[i] = [pos, vel, rot, ang, g]

    def _fill_agent_row(self, i, a, dev):
        st = a._state
        force, torque = st._force, st._torque
        if force.requires_grad or torque.requires_grad:
            _check_grad((force, torque))
        f = force if (force.dtype is torch.float32 and force.device == dev) else self._prep(force, dev)
        t = torque if (torque.dtype is torch.float32 and torque.device == dev) else self._prep(torque, dev)
        fs = f.stride()
        af = self._aio_f
        af["force"][i], af["torque"][i] = f.data_ptr(), t.data_ptr()
        af["force_s0"][i], af["force_s1"][i], af["torque_s0"][i] = fs[0], fs[1], t.stride(0)
        self._agent_seen[i] = (force, torque)
        self._agent_keep[i] = (f, t)

    def _needs_grad(self) -> bool:
        if not torch.is_grad_enabled():
            return False
        for e in self.world.entities:
            st = e._state
            if st._pos.requires_grad or st._vel.requires_grad or st._rot.requires_grad or st._ang_vel.requires_grad:
                return True
        for a in self.world.agents:
            st = a._state
            if st._force.requires_grad or st._torque.requires_grad:
                return True
        return False

    def step(self):
        self._ensure()
        if self._needs_grad():
            # autograd through the step: the forward is the native step, the backward the native
            # vector-Jacobian product (csrc/vmas_grad.hip); the new state tensors are views of the
            # autograd Function's output
            inputs = []
            for e in self.entities:
                st = e._state
                inputs += [st._pos, st._vel, st._rot, st._ang_vel]
            for a in self.agents:
                inputs += [a._state._force, a._state._torque]
            out = _StepFn.apply(self, *inputs)
            self._repoint(out)
            return
        out = self._launch()
        self._repoint(out)

    def _launch(self, grad_ok: bool = False) -> torch.Tensor:
        """Fill the pointer tables from the current state tensors and run the native step into a
        fresh output buffer (returned)."""
        global _GRAD_OK
        w = self.world
        dev = self._dev
        B = w.batch_dim
        _GRAD_OK = grad_ok
        try:
            return self._launch_body(w, dev, B)
        finally:
            _GRAD_OK = False

    def _launch_body(self, w, dev, B) -> torch.Tensor:
        # pointer tables: only tensors that are not the objects seen last step are re-read
        seen = self._ent_seen
        for i, e in enumerate(self.entities):
            c = seen[i]
            st = e._state
            if (c is None or st._pos is not c[0] or st._vel is not c[1] or st._rot is not c[2]
                    or st._ang_vel is not c[3] or e._gravity is not c[4]):
                self._fill_entity_row(i, e, dev, B)
        aseen = self._agent_seen
        for i, a in enumerate(self.agents):
            c = aseen[i]
            st = a._state
            if c is None or st._force is not c[0] or st._torque is not c[1]:
                self._fill_agent_row(i, a, dev)
        jio = self._jio
        keep = []
        for i, jc in enumerate(self.joint_list):
            fr = jc.fixed_rotation
            if isinstance(fr, torch.Tensor):
                fr = self._prep(fr, dev)
                if fr.dim() == 0 or fr.shape[0] != B:
                    fr = fr.reshape(-1)[:1].expand(B, 1) if fr.numel() == 1 else fr.expand(B, 1)
                keep.append(fr)
                jio[i]["fixed_rotation"] = fr.data_ptr()
                jio[i]["s0"] = fr.stride(0)
            else:
                jio[i]["fixed_rotation"] = 0

        # one fresh output buffer (layout: see _build)
        out = torch.empty(self._out_numel, device=dev, dtype=torch.float32)
        base = out.data_ptr()
        o_pos, o_vel, o_rot, o_ang, o_force, o_torque = self._out_off
        io = self._io
        io.out_pos, io.out_vel, io.out_rot = base + 4 * o_pos, base + 4 * o_vel, base + 4 * o_rot
        io.out_ang_vel, io.out_force, io.out_torque = base + 4 * o_ang, base + 4 * o_force, base + 4 * o_torque
        # the substep loop runs w._substeps times with the world's own w._sub_dt attribute, as
        # ref core.py:1977 / 2068 / 2870 / 2879 / 2905 / 2907 read them (two independent
        # attributes: setting one does not update the other)
        params = (w._substeps, w._sub_dt, w.broadphase)
        if params != self._step_params:
            io.substeps = int(w._substeps)
            io.sub_dt = _f32(w._sub_dt)
            io.broadphase = N.BROADPHASE_BATCH if w.broadphase == "batch" else N.BROADPHASE_ENV
            self._step_params = params
        fd = None
        if self._cfg.export_forces:
            # World.forces_dict / torques_dict rows ([E][B][2] | [E][B]); entities that neither move
            # nor rotate are not written by the kernels (their rows are set when the dicts are
            # first read: zeros, or their friction -- _static_forces)
            E = len(self.entities)
            fd = torch.empty(E * B * 3, device=dev, dtype=torch.float32)
            io.out_fdict, io.out_tdict = fd.data_ptr(), fd.data_ptr() + 4 * E * B * 2
        else:
            io.out_fdict = io.out_tdict = 0
        iters = ctypes.c_int32(0)
        if self._jit is not None:
            N.check_jit(self.lib.vmas_jit_world_step(self._jit, ctypes.byref(io), self._stream(dev),
                                                     ctypes.byref(iters)), "vmas_jit_world_step")
        else:
            N.check(self.lib.vmas_world_step(self._handle, ctypes.byref(io), self._stream(dev),
                                             ctypes.byref(iters)), "vmas_world_step")
        self._last_iterations = iters.value
        # the dicts are built from the buffer when first read (World.forces_dict); a step that did
        # not export leaves none (stale dicts of an earlier step must not be read as this one's).
        # Rows of entities that neither move nor rotate: zeros, set on first read, except where
        # friction acts on their (constant) velocity -- computed here, from the state and
        # coefficients of this step (a read after a later change must see this step's values)
        done = ()
        if fd is not None:
            done = self._static_friction_rows(fd, B, w)
        w._force_buf = (fd, B, self, done) if fd is not None else None
        w._forces_dict = w._torques_dict = None
        self.steps += 1
        self._last_keep = keep
        return out

    def _static_friction_rows(self, fd: torch.Tensor, B: int, w):
        """Step time: the rows of static entities on which friction acts (see force_dicts);
        returns their entity indices."""
        done = []
        for i, e in enumerate(self.entities):
            if e.movable or e.rotatable:
                continue
            lin = e.linear_friction is not None or w._linear_friction > 0
            ang = e.angular_friction is not None or w._angular_friction > 0
            if lin or ang:
                E = len(self.entities)
                f2 = fd[: E * B * 2].view(E, B, 2)
                f1 = fd[E * B * 2:].view(E, B, 1)
                f2[i].zero_()
                f1[i].zero_()
                self._static_forces(e, f2[i], f1[i], w)
                done.append(i)
        return tuple(done)

    def force_dicts(self, fd: torch.Tensor, B: int, done=()):
        """World.forces_dict / torques_dict (ref core.py:1975-1992) of the step that wrote ``fd``:
        per entity, views of its last-substep force [B,2] and torque [B,1] totals.  Rows of
        entities that neither move nor rotate (the kernels do not write them): friction rows
        (``done``) were set at step time, the others are zeros, set here."""
        E = len(self.entities)
        f2 = fd[: E * B * 2].view(E, B, 2)
        f1 = fd[E * B * 2:].view(E, B, 1)
        forces, torques = {}, {}
        for i, e in enumerate(self.entities):
            forces[e], torques[e] = f2[i], f1[i]
            if not (e.movable or e.rotatable) and i not in done:
                f2[i].zero_()
                f1[i].zero_()
        return forces, torques

    @staticmethod
    def _static_forces(e, f, t, w) -> None:
        """An entity that neither moves nor rotates only receives friction from its (constant)
        velocity (ref core.py:2053-2101; contacts and gravity need movable / rotatable)."""

        def friction(vel, coeff, mass):  # get_friction_force (ref core.py:2054-2072)
            speed = torch.linalg.vector_norm(vel, dim=-1)
            static = speed == 0
            ff = -(vel / torch.where(static, 1e-8, speed).unsqueeze(-1)) * torch.minimum(
                torch.full_like(vel, coeff) * mass, (vel.abs() / w._sub_dt) * mass)
            return torch.where(static.unsqueeze(-1).expand(vel.shape), 0.0, ff)

        lin = e.linear_friction if e.linear_friction is not None else (
            w._linear_friction if w._linear_friction > 0 else None)
        ang = e.angular_friction if e.angular_friction is not None else (
            w._angular_friction if w._angular_friction > 0 else None)
        if lin is not None:
            f.copy_(friction(e.state.vel.to(f.dtype), lin, e.mass))
        if ang is not None:
            t.copy_(friction(e.state.ang_vel.to(t.dtype), ang, e.moment_of_inertia))

    def _repoint(self, out: torch.Tensor) -> None:
        """Re-point the integrated fields at views of the fresh buffer (new tensor objects, as the
        reference) and update their pointer-table rows in bulk."""
        w = self.world
        B = w.batch_dim
        base = out.data_ptr()
        o_pos, o_vel, o_rot, o_ang, o_force, o_torque = self._out_off
        seen = self._ent_seen
        n_lin, n_rot, n_force, n_torque = self.n_out
        n2, n1 = self._n2, self._n1
        two = out.as_strided((n2, B, 2), (2 * B, 2, 1)).unbind(0) if n2 else ()
        one = out.as_strided((n1, B, 1), (B, 1, 1), 2 * B * n2).unbind(0) if n1 else ()
        f = self._eio_f
        ekeep = self._ent_keep
        if n_lin:
            rows = self._lin_rows
            f["pos"][rows] = np.uint64(base + 4 * o_pos) + self._lin_slot_bytes
            f["vel"][rows] = np.uint64(base + 4 * o_vel) + self._lin_slot_bytes
            f["pos_s0"][rows], f["pos_s1"][rows] = 2, 1
            f["vel_s0"][rows], f["vel_s1"][rows] = 2, 1
            for k, i in enumerate(self._lin_idx):
                st = self.entities[i]._state
                p, v = two[k], two[n_lin + k]
                st._pos, st._vel = p, v
                c, kc = seen[i], ekeep[i]
                c[0] = kc[0] = p
                c[1] = kc[1] = v
        if n_rot:
            rows = self._rot_rows
            f["rot"][rows] = np.uint64(base + 4 * o_rot) + self._rot_slot_bytes
            f["ang"][rows] = np.uint64(base + 4 * o_ang) + self._rot_slot_bytes
            f["rot_s0"][rows], f["ang_s0"][rows] = 1, 1
            for k, i in enumerate(self._rot_idx):
                st = self.entities[i]._state
                r, av = one[k], one[n_rot + k]
                st._rot, st._ang_vel = r, av
                c, kc = seen[i], ekeep[i]
                c[2] = kc[2] = r
                c[3] = kc[3] = av
        for k, a in enumerate(self.force_slots):
            a._state._force = two[2 * n_lin + k]
        for k, a in enumerate(self.torque_slots):
            a._state._torque = one[2 * n_rot + k]

    # ---- ray casting ------------------------------------------------------------------------------
    def cast_rays(self, entity, angles: torch.Tensor, max_range: float,
                  entity_filter: Callable, rot_offset: torch.Tensor = None) -> torch.Tensor:
        if torch.is_grad_enabled():
            targets = [e for e in self.world.entities if e is not entity and entity_filter(e)]
            ins = [entity.state.pos, angles, rot_offset]
            for e in targets:
                ins += [e.state.pos, e.state.rot]
            if any(t is not None and t.requires_grad for t in ins):
                return _RaysFn.apply(self, entity, max_range, entity_filter, len(targets), *ins)
        return self._cast_rays_native(entity, angles, max_range, entity_filter, rot_offset)

    def _cast_rays_native(self, entity, angles: torch.Tensor, max_range: float,
                          entity_filter: Callable, rot_offset: torch.Tensor = None) -> torch.Tensor:
        w = self.world
        dev = self._device()
        B = w.batch_dim
        targets: List = []
        for e in w.entities:
            if entity is e or not entity_filter(e):
                continue
            assert e.collides(entity) and entity.collides(e), "Rays are only casted among collidables"
            targets.append(e)
        keep = []
        origin = self._prep(entity.state.pos, dev)
        ang = self._prep(angles, dev)
        _check_grad((origin, ang, rot_offset))
        if ang.dim() == 1:
            ang = ang.unsqueeze(-1)
        R = ang.shape[-1]
        assert ang.shape[0] == B
        tg = self._ray_table(targets)
        if targets:
            ps = [self._prep(e.state.pos, dev) for e in targets]
            rs = [self._prep(e.state.rot, dev) for e in targets]
            _check_grad(ps)
            _check_grad(rs)
            keep += ps + rs
            # the per-call fields, one vectorised write each (the shape fields are cached)
            tg["pos"] = [p.data_ptr() for p in ps]
            tg["rot"] = [r.data_ptr() for r in rs]
            tg["pos_s0"] = [p.stride(0) for p in ps]
            tg["pos_s1"] = [p.stride(1) for p in ps]
            tg["rot_s0"] = [r.stride(0) for r in rs]
        out = torch.empty((B, R), device=dev, dtype=torch.float32)
        rot_ptr, rot_s0 = None, 0
        if rot_offset is not None:
            ro = self._prep(rot_offset, dev)
            keep.append(ro)
            rot_ptr, rot_s0 = ro.data_ptr(), ro.stride(0)
        N.check(
            self.lib.vmas_cast_rays(
                self._native_device(dev), B, R, origin.data_ptr(), origin.stride(0), origin.stride(1),
                ang.data_ptr(), ang.stride(0), ang.stride(1), rot_ptr, rot_s0, tg.ctypes.data,
                len(targets), _f32(max_range), out.data_ptr(), self._stream(dev),
            ),
            "vmas_cast_rays",
        )
        return out

    def _ray_table(self, targets) -> np.ndarray:
        """The VmasRayTarget rows of a target list with their shape fields filled; cached per
        list of (entity, shape object, dimensions) -- the state pointers are written per call."""
        sig = tuple((e, e.shape, _shape_dims(e.shape, _shape_code(e.shape))) for e in targets)
        key = tuple(id(e) for e in targets)
        c = self._ray_tables.get(key)
        if c is not None and len(c[0]) == len(sig) and all(
                a[0] is b[0] and a[1] is b[1] and a[2] == b[2] for a, b in zip(c[0], sig)):
            return c[1]
        tg = np.zeros(max(len(targets), 1), dtype=N.RAY_TARGET_DTYPE)
        for i, (e, shape, dims) in enumerate(sig):
            code = _shape_code(shape)
            row = tg[i]
            row["shape"] = code
            if code == N.VMAS_SPHERE:
                row["radius"] = _f32(dims[0])
            else:
                row["length"] = _f32(dims[0])
                row["width"] = _f32(dims[1]) if code == N.VMAS_BOX else 0.0
        if len(self._ray_tables) > 64:
            self._ray_tables.clear()
        self._ray_tables[key] = (sig, tg)
        return tg

    # ---- distance queries -------------------------------------------------------------------------
    def _ref(self, e, dev, keep, slot=0) -> N.VmasShapeRef:
        """Shape + state reference of one entity.  The shape part is cached per entity (rebuilt
        when the shape object or its dimensions change); the state pointers are read per call."""
        shape = e.shape
        code = _shape_code(shape)
        dims = _shape_dims(shape, code)
        key = (id(e), slot)
        c = self._qrefs.get(key)
        if c is None or c[0] is not e or c[1] is not shape or c[2] != dims:
            r = N.VmasShapeRef()
            r.shape = code
            if code == N.VMAS_SPHERE:
                r.radius = _f32(dims[0])
                r.radius_lmd = _f32(dims[0] + LINE_MIN_DIST)
            else:
                r.length = _f32(dims[0])
                if code == N.VMAS_BOX:
                    r.width = _f32(dims[1])
            c = self._qrefs[key] = (e, shape, dims, r)
        r = c[3]
        st = e._state
        return self._fill_ref(r, st._pos, st._rot, dev, keep)

    def _ref_from(self, e, p, rot, dev, keep, slot=0) -> N.VmasShapeRef:
        """_ref with explicit (saved) pos / rot tensors (the distance query's backward)."""
        r = self._ref(e, dev, [], slot)
        return self._fill_ref(r, p.detach(), rot.detach(), dev, keep)

    def _fill_ref(self, r, p, rot, dev, keep) -> N.VmasShapeRef:
        if p.dtype is not torch.float32 or p.device != dev:
            p = p.to(device=dev, dtype=torch.float32)
        if rot.dtype is not torch.float32 or rot.device != dev:
            rot = rot.to(device=dev, dtype=torch.float32)
        if p.requires_grad or rot.requires_grad:
            _check_grad((p, rot))
        keep.append(p)
        keep.append(rot)
        ps = p.stride()
        r.pos, r.rot = p.data_ptr(), rot.data_ptr()
        r.pos_s0, r.pos_s1, r.rot_s0 = ps[0], ps[1], rot.stride(0)
        return r

    def _query(self, kind, a, b=None, tp=None):
        global _GRAD_OK
        if kind == N.OVERLAP_PAIR:  # a bool result: nothing to differentiate
            prev, _GRAD_OK = _GRAD_OK, True
            try:
                return self._query_native(kind, a, b, tp)
            finally:
                _GRAD_OK = prev
        if torch.is_grad_enabled():
            ins = [a._state._pos, a._state._rot]
            ins += [b._state._pos, b._state._rot] if b is not None else [None, None]
            tpt = torch.as_tensor(tp) if tp is not None else None
            ins.append(tpt)
            if any(t is not None and t.requires_grad for t in ins):
                return _DistFn.apply(self, kind, a, b, *ins)
        return self._query_native(kind, a, b, tp)

    def _query_native(self, kind, a, b=None, tp=None):
        w = self.world
        dev = self._device()
        B = w.batch_dim
        keep = []
        ra = self._ref(a, dev, keep, 0)
        rb = self._ref(b, dev, keep, 1) if b is not None else None
        tptr, t0, t1 = None, 0, 0
        if tp is not None:
            tp = self._prep(torch.as_tensor(tp), dev)
            _check_grad((tp,))
            if tp.dim() == 1:
                tp = tp.unsqueeze(0)
            tp = tp.expand(B, 2)
            keep.append(tp)
            tptr, t0, t1 = tp.data_ptr(), tp.stride(0), tp.stride(1)
        out = torch.empty(B, device=dev, dtype=torch.bool if kind == N.OVERLAP_PAIR else torch.float32)
        N.check(
            self.lib.vmas_distance(
                self._native_device(dev), B, kind, ctypes.byref(ra),
                ctypes.byref(rb) if rb is not None else None, tptr, t0, t1, out.data_ptr(),
                self._stream(dev),
            ),
            "vmas_distance",
        )
        return out

    @staticmethod
    def _canonical(a, b):
        """Order a pair as the reference's distance branches do (box/line first, sphere last)."""
        ca, cb = _shape_code(a.shape), _shape_code(b.shape)
        S, B_, L = N.VMAS_SPHERE, N.VMAS_BOX, N.VMAS_LINE
        if ca == S and cb != S:
            return b, a
        if ca == L and cb == B_:
            return b, a
        return a, b

    def distance_from_point(self, entity, test_point):
        return self._query(N.DIST_POINT, entity, tp=test_point)

    def distance(self, a, b):
        a, b = self._canonical(a, b)
        return self._query(N.DIST_PAIR, a, b)

    def overlap(self, a, b):
        a, b = self._canonical(a, b)
        return self._query(N.OVERLAP_PAIR, a, b)


class _StepFn(torch.autograd.Function):
    """World.step with autograd: forward = the native step (k_world / k_step / host backend),
    backward = vmas_world_step_vjp (forward-mode duals through the same physics, contracted
    with the output gradient; csrc/vmas_grad.hip).  Inputs: every entity's pos / vel / rot /
    ang_vel, then every agent's force / torque; output: the step's output buffer."""

    @staticmethod
    def forward(ctx, eng, *inputs):
        out = eng._launch(grad_ok=True)
        # the backward reads the inputs through a snapshot of this step's pointer tables
        ctx.eng = eng
        ctx.tables = (eng._eio.copy(), eng._aio.copy(), eng._jio.copy(), eng._io.substeps, eng._io.sub_dt,
                      eng._io.broadphase)
        # the world tables of THIS forward (a parameter or entity change before the backward
        # rebuilds the engine's own; the VJP must differentiate the step that ran)
        ctx.world_tables = (eng._cfg, eng._tables, eng._out_off, list(eng.entities), list(eng.agents))
        ctx.keep = ([list(k) if k is not None else None for k in eng._ent_keep],
                    [tuple(k) if k is not None else None for k in eng._agent_keep], eng._last_keep)
        # the backward re-runs the step on the forward's input values: inputs that require grad
        # are saved (autograd checks their versions), the others are copied (a scenario may edit
        # them in place after the step, e.g. discovery's target respawn)
        ctx.grad_mask = [x.requires_grad for x in inputs]
        ctx.consts = [None if x.requires_grad else x.detach().clone() for x in inputs]
        ctx.save_for_backward(*[x if x.requires_grad else None for x in inputs])
        return out

    @staticmethod
    def backward(ctx, gout):
        eng = ctx.eng
        saved = ctx.saved_tensors
        inputs = [s if s is not None else c for s, c in zip(saved, ctx.consts)]
        eio, aio, jio, substeps, sub_dt, bp = ctx.tables
        cfg, (ed, pd, jd), out_off, entities, agents = ctx.world_tables
        eio, aio = eio.copy(), aio.copy()
        dev = eng._dev
        B = eng.world.batch_dim
        keep = []
        for i in range(len(entities)):  # the rows point at the forward's input values
            pos, vel, rot, ang = (eng._prep(t.detach(), dev) for t in inputs[4 * i: 4 * i + 4])
            keep += [pos, vel, rot, ang]
            eio["pos"][i], eio["vel"][i], eio["rot"][i], eio["ang"][i] = pos.data_ptr(), vel.data_ptr(), rot.data_ptr(), ang.data_ptr()
            eio["pos_s0"][i], eio["pos_s1"][i] = pos.stride()
            eio["vel_s0"][i], eio["vel_s1"][i] = vel.stride()
            eio["rot_s0"][i], eio["ang_s0"][i] = rot.stride(0), ang.stride(0)
        off = 4 * len(entities)
        for i in range(len(agents)):
            f, t = (eng._prep(x.detach(), dev) for x in inputs[off + 2 * i: off + 2 * i + 2])
            keep += [f, t]
            aio["force"][i], aio["torque"][i] = f.data_ptr(), t.data_ptr()
            aio["force_s0"][i], aio["force_s1"][i] = f.stride()
            aio["torque_s0"][i] = t.stride(0)
        io = N.VmasStepIO()
        io.entities, io.agents, io.joints = eio.ctypes.data, aio.ctypes.data, jio.ctypes.data
        io.substeps, io.sub_dt, io.broadphase = substeps, sub_dt, bp
        g = gout.to(device=dev, dtype=torch.float32).contiguous()
        base = g.data_ptr()
        go = N.VmasStepIO()
        o_pos, o_vel, o_rot, o_ang, o_force, o_torque = out_off
        go.out_pos, go.out_vel, go.out_rot = base + 4 * o_pos, base + 4 * o_vel, base + 4 * o_rot
        go.out_ang_vel, go.out_force, go.out_torque = base + 4 * o_ang, base + 4 * o_force, base + 4 * o_torque
        E, A = len(entities), len(agents)
        grads = []
        ptrs = {k: (ctypes.c_void_p * max(E, 1))() for k in ("pos", "vel", "rot", "ang")}
        ptrs.update({k: (ctypes.c_void_p * max(A, 1))() for k in ("force", "torque")})
        for i in range(E):
            for k, w2, key in ((0, 2, "pos"), (1, 2, "vel"), (2, 1, "rot"), (3, 1, "ang")):
                t = torch.zeros(B, w2, device=dev, dtype=torch.float32)
                grads.append(t)
                ptrs[key][i] = t.data_ptr()
        for i in range(A):
            for w2, key in ((2, "force"), (1, "torque")):
                t = torch.zeros(B, w2, device=dev, dtype=torch.float32)
                grads.append(t)
                ptrs[key][i] = t.data_ptr()
        gio = N.VmasGradIO(*(ctypes.cast(ptrs[k], ctypes.c_void_p) for k in ("pos", "vel", "rot", "ang", "force", "torque")))
        N.check_aux(eng.lib.vmas_world_step_vjp(ctypes.byref(cfg), ed, pd, jd, ctypes.byref(io), ctypes.byref(go),
                                                ctypes.byref(gio), eng._stream(dev) if eng._dev_index >= 0 else None),
                    "vmas_world_step_vjp")
        out = []
        for t, x, needs in zip(grads, inputs, ctx.grad_mask):
            out.append(t.reshape(x.shape).to(dtype=x.dtype, device=x.device) if needs else None)
        return (None, *out)


class _DistFn(torch.autograd.Function):
    """get_distance / get_distance_from_point with autograd: forward = vmas_distance, backward =
    vmas_distance_vjp (dual numbers through the same closest-point functions)."""

    @staticmethod
    def forward(ctx, eng, kind, a, b, pa, ra, pb, rb, tp):
        global _GRAD_OK
        prev, _GRAD_OK = _GRAD_OK, True
        try:
            out = eng._query_native(kind, a, b, tp)
        finally:
            _GRAD_OK = prev
        ctx.eng, ctx.kind, ctx.a, ctx.b = eng, kind, a, b
        ctx.save_for_backward(pa, ra, pb if pb is not None else torch.empty(0), rb if rb is not None else torch.empty(0),
                              tp if tp is not None else torch.empty(0))
        ctx.has_b, ctx.has_tp = pb is not None, tp is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        eng, kind = ctx.eng, ctx.kind
        pa, ra, pb, rb, tp = ctx.saved_tensors
        dev = eng._device()
        B = eng.world.batch_dim
        keep = []
        refa = N.VmasShapeRef()
        ctypes.memmove(ctypes.byref(refa), ctypes.byref(eng._ref_from(ctx.a, pa, ra, dev, keep, 0)), ctypes.sizeof(refa))
        refb = None
        if ctx.has_b:
            refb = N.VmasShapeRef()
            ctypes.memmove(ctypes.byref(refb), ctypes.byref(eng._ref_from(ctx.b, pb, rb, dev, keep, 1)), ctypes.sizeof(refb))
        tptr, t0, t1 = None, 0, 0
        if ctx.has_tp:
            t = eng._prep(tp.detach(), dev)
            if t.dim() == 1:
                t = t.unsqueeze(0)
            t = t.expand(B, 2)
            keep.append(t)
            tptr, t0, t1 = t.data_ptr(), t.stride(0), t.stride(1)
        g = gout.detach().to(device=dev, dtype=torch.float32).contiguous()
        z = lambda n: torch.zeros(B, n, device=dev, dtype=torch.float32)  # noqa: E731
        ga_p, ga_r, gb_p, gb_r, gt = z(2), z(1), z(2), z(1), z(2)
        N.check_aux(eng.lib.vmas_distance_vjp(
            eng._native_device(dev), B, kind, ctypes.byref(refa), ctypes.byref(refb) if refb is not None else None,
            tptr, t0, t1, g.data_ptr(), ga_p.data_ptr(), ga_r.data_ptr(), gb_p.data_ptr(), gb_r.data_ptr(),
            gt.data_ptr(), eng._stream(dev)), "vmas_distance_vjp")
        if eng._native_device(dev) >= 0:
            torch.cuda.current_stream(dev).synchronize()

        def fit(gr, x):
            if x is None or x.numel() == 0 or not x.requires_grad:
                return None
            return gr.reshape(x.shape).to(dtype=x.dtype, device=x.device) if gr.numel() == x.numel() else \
                gr.sum(0).reshape(x.shape).to(dtype=x.dtype, device=x.device)

        return (None, None, None, None, fit(ga_p, pa), fit(ga_r, ra), fit(gb_p, pb) if ctx.has_b else None,
                fit(gb_r, rb) if ctx.has_b else None, fit(gt, tp) if ctx.has_tp else None)


class _RaysFn(torch.autograd.Function):
    """World.cast_rays with autograd: forward = vmas_cast_rays, backward = vmas_cast_rays_vjp."""

    @staticmethod
    def forward(ctx, eng, entity, max_range, entity_filter, n_targets, origin, angles, rot_offset, *tpr):
        global _GRAD_OK
        prev, _GRAD_OK = _GRAD_OK, True
        try:
            out = eng._cast_rays_native(entity, angles, max_range, entity_filter, rot_offset)
        finally:
            _GRAD_OK = prev
        ctx.eng, ctx.max_range, ctx.nt = eng, max_range, n_targets
        ctx.targets = [e for e in eng.world.entities if e is not entity and entity_filter(e)]
        ctx.has_rot = rot_offset is not None
        ctx.save_for_backward(origin, angles, rot_offset if rot_offset is not None else torch.empty(0), *tpr)
        return out

    @staticmethod
    def backward(ctx, gout):
        eng = ctx.eng
        saved = ctx.saved_tensors
        origin, angles, rot = saved[0], saved[1], saved[2]
        tpr = saved[3:]
        dev = eng._device()
        B = eng.world.batch_dim
        keep = []
        o = eng._prep(origin.detach(), dev)
        ang = eng._prep(angles.detach(), dev)
        if ang.dim() == 1:
            ang = ang.unsqueeze(-1)
        R = ang.shape[-1]
        rptr, rs0 = None, 0
        if ctx.has_rot:
            r = eng._prep(rot.detach(), dev)
            keep.append(r)
            rptr, rs0 = r.data_ptr(), r.stride(0)
        tg = eng._ray_table(ctx.targets).copy()
        ps = [eng._prep(tpr[2 * i].detach(), dev) for i in range(ctx.nt)]
        rs = [eng._prep(tpr[2 * i + 1].detach(), dev) for i in range(ctx.nt)]
        keep += ps + rs + [o, ang]
        if ctx.nt:
            tg["pos"] = [p.data_ptr() for p in ps]
            tg["rot"] = [x.data_ptr() for x in rs]
            tg["pos_s0"] = [p.stride(0) for p in ps]
            tg["pos_s1"] = [p.stride(1) for p in ps]
            tg["rot_s0"] = [x.stride(0) for x in rs]
        g = gout.detach().to(device=dev, dtype=torch.float32).contiguous()
        z = lambda *shape: torch.zeros(*shape, device=dev, dtype=torch.float32)  # noqa: E731
        g_o, g_r, g_a = z(B, 2), z(B, 1), z(B, R)
        g_tp = [z(B, 2) for _ in range(ctx.nt)]
        g_tr = [z(B, 1) for _ in range(ctx.nt)]
        arr_p = (ctypes.c_void_p * max(ctx.nt, 1))(*[t.data_ptr() for t in g_tp])
        arr_r = (ctypes.c_void_p * max(ctx.nt, 1))(*[t.data_ptr() for t in g_tr])
        N.check_aux(eng.lib.vmas_cast_rays_vjp(
            eng._native_device(dev), B, R, o.data_ptr(), o.stride(0), o.stride(1), ang.data_ptr(), ang.stride(0),
            ang.stride(1), rptr, rs0, tg.ctypes.data, ctx.nt, _f32(ctx.max_range), g.data_ptr(), g_o.data_ptr(),
            g_r.data_ptr(), g_a.data_ptr(), arr_p, arr_r, eng._stream(dev)), "vmas_cast_rays_vjp")

        def fit(gr, x):
            if x is None or x.numel() == 0 or not x.requires_grad:
                return None
            if gr.numel() != x.numel():
                gr = gr.sum(0)
            return gr.reshape(x.shape).to(dtype=x.dtype, device=x.device)

        out = [None, None, None, None, None, fit(g_o, origin), fit(g_a, angles), fit(g_r, rot) if ctx.has_rot else None]
        for i in range(ctx.nt):
            out += [fit(g_tp[i], tpr[2 * i]), fit(g_tr[i], tpr[2 * i + 1])]
        return tuple(out)
