"""ctypes binding of the C ABI declared in ``include/vmas_mi355x.h``.

The shared library ``libvmas_mi355x.so`` is built in-tree by ``__graft_entry__.build()`` (hipcc,
``--offload-arch=gfx950``).  It contains both the gfx950 kernels and the host (``device == -1``)
backend compiled from the same ``csrc/vmas_physics.hpp``.  There is no Python fallback: if the
library is missing, importing the simulator raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

LIB_NAME = "libvmas_mi355x.so"
# VMAS_LIB_PATH: another build of the same sources (tools/asan_host.sh: the host-sanitized one)
LIB_PATH = Path(os.environ.get("VMAS_LIB_PATH") or Path(__file__).resolve().parent / LIB_NAME)

# ------------------------------------------------------------------------------------------------
# constants mirrored from include/vmas_mi355x.h
VMAS_ABI_VERSION = 6
VMAS_SPHERE, VMAS_BOX, VMAS_LINE = 0, 1, 2
(
    VMAS_PAIR_JOINT,
    VMAS_PAIR_SS,
    VMAS_PAIR_LS,
    VMAS_PAIR_LL,
    VMAS_PAIR_BS,
    VMAS_PAIR_BL,
    VMAS_PAIR_BB,
) = range(7)
F_MOVABLE = 1 << 0
F_ROTATABLE = 1 << 1
F_HOLLOW = 1 << 2
F_AGENT = 1 << 3
F_MAX_F = 1 << 4
F_F_RANGE = 1 << 5
F_MAX_T = 1 << 6
F_T_RANGE = 1 << 7
F_MAX_SPEED = 1 << 8
F_V_RANGE = 1 << 9
F_LIN_FRIC = 1 << 10
F_ANG_FRIC = 1 << 11
F_GRAVITY = 1 << 12
BROADPHASE_BATCH = 0
BROADPHASE_ENV = 1
DIST_POINT, DIST_PAIR, OVERLAP_PAIR = 0, 1, 2
EPILOGUE_NONE, EPILOGUE_BALANCE, EPILOGUE_TRANSPORT = 0, 1, 2  # VmasWorldConfig.epilogue

# exported symbols (tests check the library exports every one of them)
EXPORTED_SYMBOLS = (
    "vmas_abi_version",
    "vmas_device_count",
    "vmas_last_error",
    "vmas_stream_abort_capture",
    "vmas_graph_launch",
    "vmas_graph_chain_build",
    "vmas_graph_chain_launch",
    "vmas_graph_chain_free",
    "vmas_graph_chain_nodes",
    "vmas_graph_chain_fused",
    "vmas_graph_chain_set_writeback",
    "vmas_graph_chain_launch_wb",
    "vmas_jit_world_epilogue",
    "vmas_jit_program_outputs",
    "vmas_host_waits",
    "vmas_test_hold",
    "vmas_balance_outputs",
    "vmas_test_exact_math",
    "vmas_test_fast_trig",
    "vmas_copy_spans",
    "vmas_spawn_targets",
    "vmas_spawn_scratch_words",
    "vmas_spawn_channel_create",
    "vmas_spawn_channel_destroy",
    "vmas_spawn_channel_arm",
    "vmas_spawn_channel_in",
    "vmas_spawn_channel_wait",
    "vmas_spawn_profile",
    "vmas_world_step_vjp",
    "vmas_distance_vjp",
    "vmas_cast_rays_vjp",
    "vmas_flocking_outputs",
    "vmas_flocking_target_action",
    "vmas_assert_publish_range",
    "vmas_transport_outputs",
    "vmas_discovery_outputs",
    "vmas_world_create",
    "vmas_world_destroy",
    "vmas_world_step",
    "vmas_world_set_timing",
    "vmas_world_get_timing",
    "vmas_cast_rays",
    "vmas_distance",
    "vmas_check_actions",
    "vmas_apply_actions",
    "vmas_apply_actions_launch",
    "vmas_apply_actions_flags",
    "vmas_uniform_columns",
    "vmas_uniform_columns_snap",
    "vmas_copy_spans_draw",
    "vmas_graph_chain_launch_tail",
    "vmas_test_tail_draw",
    "vmas_assert_create",
    "vmas_assert_destroy",
    "vmas_assert_publish",
    "vmas_assert_wait",
    "vmas_spawn_resolve",
    "vmas_aux_last_error",
    "vmas_jit_world_create",
    "vmas_jit_world_destroy",
    "vmas_jit_world_step",
    "vmas_jit_world_set_timing",
    "vmas_jit_world_get_timing",
    "vmas_jit_world_device_timing",
    "vmas_jit_world_source",
    "vmas_jit_compile_check",
    "vmas_jit_world_profile",
    "vmas_jit_world_passes",
    "vmas_jit_world_check",
    "vmas_jit_world_grid",
    "vmas_jit_world_set_params",
    "vmas_jit_stats",
    "vmas_jit_last_error",
)

_i32 = ctypes.c_int32
_u32 = ctypes.c_uint32
_f32 = ctypes.c_float
_vp = ctypes.c_void_p


class VmasEntityDesc(ctypes.Structure):
    _fields_ = [
        ("shape", _i32),
        ("flags", _u32),
        ("agent_index", _i32),
        ("out_lin", _i32),
        ("out_rot", _i32),
        ("out_force", _i32),
        ("out_torque", _i32),
        ("radius", _f32),
        ("half_length", _f32),
        ("half_width", _f32),
        ("mass", _f32),
        ("inertia", _f32),
        ("one_minus_drag", _f32),
        ("lin_fric", _f32),
        ("ang_fric", _f32),
        ("max_speed", _f32),
        ("v_range", _f32),
        ("max_f", _f32),
        ("f_range", _f32),
        ("max_t", _f32),
        ("t_range", _f32),
    ]


class VmasPairDesc(ctypes.Structure):
    _fields_ = [
        ("cls", _i32),
        ("ea", _i32),
        ("eb", _i32),
        ("joint", _i32),
        ("bp_radius", _f32),
        ("dmin", _f32),
    ]


class VmasJointDesc(ctypes.Structure):
    _fields_ = [
        ("delta_a_x", _f32),
        ("delta_a_y", _f32),
        ("delta_b_x", _f32),
        ("delta_b_y", _f32),
        ("dist", _f32),
        ("rotate", _i32),
        ("fixed_rotation", _f32),
        ("pad", _i32),
    ]


class VmasWorldConfig(ctypes.Structure):
    _fields_ = [
        ("n_entities", _i32),
        ("n_agents", _i32),
        ("n_pairs", _i32),
        ("n_joints", _i32),
        ("batch", _i32),
        ("device", _i32),
        ("n_out_lin", _i32),
        ("n_out_rot", _i32),
        ("n_out_force", _i32),
        ("n_out_torque", _i32),
        ("contact_margin", _f32),
        ("collision_force", _f32),
        ("joint_force", _f32),
        ("torque_constraint_force", _f32),
        ("gravity_x", _f32),
        ("gravity_y", _f32),
        ("has_world_gravity", _i32),
        ("x_semidim", _f32),
        ("y_semidim", _f32),
        ("has_x_semidim", _i32),
        ("has_y_semidim", _i32),
        ("max_substeps", _i32),
        ("export_forces", _i32),
        ("epilogue", _i32),
        ("pad_cfg", _i32),
    ]


class VmasStepIO(ctypes.Structure):
    _fields_ = [
        ("entities", _vp),
        ("agents", _vp),
        ("joints", _vp),
        ("out_pos", _vp),
        ("out_vel", _vp),
        ("out_rot", _vp),
        ("out_ang_vel", _vp),
        ("out_force", _vp),
        ("out_torque", _vp),
        ("substeps", _i32),
        ("sub_dt", _f32),
        ("broadphase", _i32),
        ("pad", _i32),
        ("out_fdict", _vp),
        ("out_tdict", _vp),
    ]


class VmasShapeRef(ctypes.Structure):
    _fields_ = [
        ("shape", _i32),
        ("pad0", _i32),
        ("radius", _f32),
        ("length", _f32),
        ("width", _f32),
        ("radius_lmd", _f32),
        ("pos", _vp),
        ("rot", _vp),
        ("pos_s0", _i32),
        ("pos_s1", _i32),
        ("rot_s0", _i32),
        ("pad", _i32),
    ]


VMAS_COPY_MAX_SPANS = 160


class VmasCopySpan(ctypes.Structure):
    _fields_ = [("src", _vp), ("dst", _vp), ("nbytes", ctypes.c_int64)]


def copy_raw(device_index: int, spans, stream) -> None:
    """One native launch (vmas_copy_spans) for every (src_ptr, dst_ptr, nbytes) span."""
    n = len(spans)
    if not n:
        return
    arr = (VmasCopySpan * n)()
    for i, (src, dst, nb) in enumerate(spans):
        arr[i].src, arr[i].dst, arr[i].nbytes = src, dst, nb
    check_aux(load_library().vmas_copy_spans(device_index, arr, n, stream), "vmas_copy_spans")


VMAS_SPAWN_MAX_TARGETS = 16
VMAS_SPAWN_MAX_TRIES = 65536


VMAS_SPAWN_ERR_WORD = 64
VMAS_SPAWN_OFF_END_WORD = 36  # (u64: the generator offset after a call through a channel)
VMAS_SPAWN_RNG_WORD = 40  # (where a channel's seed / offset / seq are staged)


def spawn_words(n_targets: int) -> int:  # VMAS_SPAWN_WORDS
    return 96 + 32 * n_targets + 32 * 32


class VmasSpawnTargetsIO(ctypes.Structure):
    _fields_ = [
        ("batch", _i32), ("n_agents", _i32), ("n_targets", _i32), ("mode", _i32),
        ("agents", _vp), ("ag_s0", _i32), ("ag_s1", _i32), ("ag_s2", _i32), ("max_tries", _i32),
        ("pos", _vp * VMAS_SPAWN_MAX_TARGETS), ("pos_s0", _i32 * VMAS_SPAWN_MAX_TARGETS),
        ("pos_s1", _i32 * VMAS_SPAWN_MAX_TARGETS),
        ("covered", _vp), ("cov_s0", _i32), ("cov_s1", _i32),
        ("min_dist", _f32), ("x_lo", _f32), ("x_hi", _f32), ("y_lo", _f32), ("y_hi", _f32), ("pad1", _f32),
        ("seed", ctypes.c_uint64), ("offset", ctypes.c_uint64), ("max_accepted", _vp), ("channel", _vp),
        ("backup", _vp), ("scratch", _vp), ("scratch_words", ctypes.c_int64), ("prestaged", _i32), ("pad2", _i32),
    ]


COPY_SPAN_DTYPE = np.dtype([("src", np.uint64), ("dst", np.uint64), ("nbytes", np.int64)])  # VmasCopySpan
VMAS_COPY_STORE64 = -8  # (a span storing the 8-byte value src at dst)


def stream_ptr(index: int) -> int:
    """The raw hipStream_t of torch's current stream on device `index` (what
    torch.cuda.current_stream(index).cuda_stream returns, without building a Stream object: the
    host path of a step asks for it several times)."""
    return _raw_stream(index)


def _raw_stream(index):
    import torch

    return torch._C._cuda_getCurrentRawStream(index)


def copy_table(device_index: int, table: np.ndarray, lo: int, hi: int, stream) -> None:
    """One native launch (vmas_copy_spans) for rows lo..hi of a COPY_SPAN_DTYPE table."""
    copy_table_at(device_index, table.ctypes.data, lo, hi, stream)


def copy_table_at(device_index: int, table_addr: int, lo: int, hi: int, stream) -> None:
    """copy_table with the table's address (ndarray.ctypes.data, taken once by a caller that keeps
    the table: each access of .ctypes builds a helper object)."""
    if hi > lo:
        rc = (_copy_fn or _bind_copy())(device_index, table_addr + lo * COPY_SPAN_DTYPE.itemsize, hi - lo, stream)
        if rc:
            check_aux(rc, "vmas_copy_spans")


_copy_fn = None


def _bind_copy():
    global _copy_fn
    _copy_fn = load_library().vmas_copy_spans
    return _copy_fn


def copy_spans(device_index: int, pairs, stream) -> None:
    """dst.copy_(src) for every (dst, src) pair of same-size contiguous device tensors, all in one
    native launch (vmas_copy_spans; any dtype: bytes are copied)."""
    copy_raw(device_index, [(s.data_ptr(), d.data_ptr(), d.numel() * d.element_size()) for d, s in pairs], stream)


class VmasGradIO(ctypes.Structure):
    _fields_ = [("pos", _vp), ("vel", _vp), ("rot", _vp), ("ang_vel", _vp), ("force", _vp), ("torque", _vp)]


class VmasVec(ctypes.Structure):
    _fields_ = [("p", _vp), ("s0", _i32), ("s1", _i32)]


VMAS_SCN_MAX_AGENTS = 32
VMAS_SCN_REWARD, VMAS_SCN_OBS, VMAS_SCN_DONE = 1, 2, 4


class VmasBalanceIO(ctypes.Structure):
    _fields_ = [
        ("batch", _i32), ("n_agents", _i32), ("what", _i32), ("pad0", _i32),
        ("shaping_factor", _f32), ("fall_reward", _f32), ("pi", _f32), ("pad1", _f32),
        ("package", VmasShapeRef), ("goal", VmasShapeRef), ("line", VmasShapeRef), ("floor", VmasShapeRef),
        ("package_vel", VmasVec), ("line_vel", VmasVec), ("line_ang_vel", VmasVec),
        ("agent_pos", VmasVec * VMAS_SCN_MAX_AGENTS), ("agent_vel", VmasVec * VMAS_SCN_MAX_AGENTS),
        ("global_shaping", _vp), ("gs_s0", _i32), ("pad2", _i32),
        ("global_shaping_out", _vp), ("package_dist", _vp), ("pos_rew", _vp), ("ground_rew", _vp),
        ("on_the_ground", _vp),
        ("rewards", _vp * VMAS_SCN_MAX_AGENTS), ("obs", _vp * VMAS_SCN_MAX_AGENTS),
        ("done", _vp), ("pos_rew_prev", _vp),
        ("out_delta", _vp),  # (graph mode's direct outputs: [obs, rewards, done] byte offsets)
    ]


class VmasRayTarget(ctypes.Structure):
    _fields_ = [("shape", _i32), ("radius", _f32), ("length", _f32), ("width", _f32), ("pos", _vp), ("rot", _vp),
                ("pos_s0", _i32), ("pos_s1", _i32), ("rot_s0", _i32), ("pad", _i32)]


VMAS_SCN_MAX_RAY_TARGETS = 16
VMAS_FLOCK_MAX_AGENTS = 16
_FA = VMAS_FLOCK_MAX_AGENTS


class VmasFlockingIO(ctypes.Structure):
    _fields_ = [
        ("batch", _i32), ("n_all", _i32), ("n_policy", _i32), ("what", _i32),
        ("target", _i32), ("n_rays", _i32), ("n_ray_targets", _i32), ("sum_mode", _i32),
        ("min_collision_distance", _f32), ("collision_reward", _f32), ("desired_distance", _f32),
        ("dist_shaping_factor", _f32), ("max_range", _f32), ("pad0", _f32),
        ("collide_reward_on", _i32), ("fast_lidar", _i32),
        ("agents", VmasShapeRef * _FA), ("scripted", _i32 * _FA), ("policy", _i32 * _FA),
        ("vel", VmasVec * _FA), ("rot", VmasVec * _FA), ("angles", _vp * _FA),
        ("ang_s0", _i32 * _FA), ("ang_s1", _i32 * _FA),
        ("ray_targets", VmasRayTarget * VMAS_SCN_MAX_RAY_TARGETS),
        ("t", _vp),
        ("shaping_in", _vp * _FA), ("shaping_out", _vp * _FA), ("dist_rew", _vp * _FA),
        ("collision_rew", _vp * _FA), ("rewards", _vp * _FA), ("obs", _vp * _FA), ("lidar", _vp * _FA),
        ("out_delta", _vp),  # (graph mode's direct outputs: [obs, rewards, done] byte offsets)
    ]


VMAS_TRANSPORT_MAX_PACKAGES = 8
VMAS_TRANSPORT_MAX_AGENTS = 16
_TP, _TA = VMAS_TRANSPORT_MAX_PACKAGES, VMAS_TRANSPORT_MAX_AGENTS


class VmasTransportIO(ctypes.Structure):
    _fields_ = [
        ("batch", _i32), ("n_agents", _i32), ("n_packages", _i32), ("what", _i32),
        ("shaping_factor", _f32), ("red", _f32 * 3), ("green", _f32 * 3), ("pad0", _f32),
        ("package", VmasShapeRef * _TP), ("goal", VmasShapeRef * _TP), ("package_vel", VmasVec * _TP),
        ("agent_pos", VmasVec * _TA), ("agent_vel", VmasVec * _TA),
        ("global_shaping", _vp * _TP), ("gs_s0", _i32 * _TP), ("global_shaping_out", _vp * _TP),
        ("dist_to_goal", _vp * _TP), ("on_goal", _vp * _TP), ("color", _vp * _TP), ("on_goal_in", _vp * _TP),
        ("rew", _vp), ("obs", _vp * _TA), ("done", _vp),
        ("out_delta", _vp),  # (graph mode's direct outputs: [obs, rewards, done] byte offsets)
    ]


VMAS_DISC_MAX_AGENTS, VMAS_DISC_MAX_TARGETS, VMAS_DISC_MAX_ENTITIES, VMAS_DISC_MAX_LIDARS = 16, 16, 32, 2
_DA, _DT, _DE, _DL = VMAS_DISC_MAX_AGENTS, VMAS_DISC_MAX_TARGETS, VMAS_DISC_MAX_ENTITIES, VMAS_DISC_MAX_LIDARS


class VmasDiscoveryIO(ctypes.Structure):
    _fields_ = [
        ("batch", _i32), ("n_agents", _i32), ("n_targets", _i32), ("what", _i32),
        ("covering_range", _f32), ("covering_rew_coeff", _f32), ("time_penalty", _f32),
        ("agents_per_target", _i32), ("shared_reward", _i32), ("n_entities", _i32), ("n_lidars", _i32),
        ("time_int", _i32), ("fast_lidar", _i32), ("time_penalty_i", ctypes.c_int64),
        ("agent_entity", _i32 * _DA), ("target_entity", _i32 * _DT),
        ("pos", VmasVec * _DE), ("radius", _f32 * _DE), ("vel", VmasVec * _DA), ("rot", VmasVec * _DA),
        ("n_rays", _i32 * _DL), ("max_range", _f32 * _DL), ("mask", ctypes.c_uint32 * _DL),
        ("angles", (_vp * _DA) * _DL), ("ang_s0", (_i32 * _DA) * _DL), ("ang_s1", (_i32 * _DA) * _DL),
        ("lidar", (_vp * _DA) * _DL), ("obs", _vp * _DA),
        ("agents_pos", _vp), ("targets_pos", _vp), ("dists", _vp), ("per_target", _vp), ("covered", _vp),
        ("time_rew", _vp), ("shared", _vp), ("covering", _vp * _DA), ("collision", _vp * _DA),
        ("rewards", _vp * _DA),
        ("covered_count", _vp), ("all_time", _vp), ("done", _vp),
        ("out_delta", _vp),  # (graph mode's direct outputs: [obs, rewards, done] byte offsets)
        ("stage_in", _vp), ("stage_out", _vp),  # (a spawn channel's words staged for the step's respawn)
    ]


# Per-call pointer tables are built as numpy structured arrays (one row per entity/agent/joint);
# their layouts must match VmasEntityIO / VmasAgentIO / VmasJointIO / VmasRayTarget.
ENTITY_IO_DTYPE = np.dtype(
    [
        ("pos", "<u8"),
        ("vel", "<u8"),
        ("rot", "<u8"),
        ("ang", "<u8"),
        ("grav", "<u8"),
        ("pos_s0", "<i4"),
        ("pos_s1", "<i4"),
        ("vel_s0", "<i4"),
        ("vel_s1", "<i4"),
        ("rot_s0", "<i4"),
        ("ang_s0", "<i4"),
        ("grav_s0", "<i4"),
        ("grav_s1", "<i4"),
    ]
)
AGENT_IO_DTYPE = np.dtype(
    [
        ("force", "<u8"),
        ("torque", "<u8"),
        ("force_s0", "<i4"),
        ("force_s1", "<i4"),
        ("torque_s0", "<i4"),
        ("pad", "<i4"),
    ]
)
JOINT_IO_DTYPE = np.dtype([("fixed_rotation", "<u8"), ("s0", "<i4"), ("pad", "<i4")])
RAY_TARGET_DTYPE = np.dtype(
    [
        ("shape", "<i4"),
        ("radius", "<f4"),
        ("length", "<f4"),
        ("width", "<f4"),
        ("pos", "<u8"),
        ("rot", "<u8"),
        ("pos_s0", "<i4"),
        ("pos_s1", "<i4"),
        ("rot_s0", "<i4"),
        ("pad", "<i4"),
    ]
)
ACTION_REF_DTYPE = np.dtype(
    [
        ("u", "<u8"),
        ("u_range", "<u8"),
        ("s0", "<i4"),
        ("s1", "<i4"),
        ("n_cols", "<i4"),
        ("n_phys", "<i4"),
        ("clamp", "<i4"),
        ("pad", "<i4"),
    ]
)
ACTION_APPLY_REF_DTYPE = np.dtype(
    [
        ("u", "<u8"),
        ("u_range", "<u8"),
        ("u_mult", "<u8"),
        ("out_offset", "<i8"),
        ("s0", "<i4"),
        ("s1", "<i4"),
        ("n_cols", "<i4"),
        ("n_phys", "<i4"),
        ("clamp", "<i4"),
        ("pad", "<i4"),
    ]
)
UNIFORM_COLUMN_DTYPE = np.dtype([("out", "<u8"), ("stride", "<i8"), ("from_", "<f4"), ("to", "<f4"), ("offset", "<u8"),
                                 ("u_out", "<u8"), ("u_stride", "<i8"), ("u_range", "<f4"), ("u_mult", "<f4"),
                                 ("u_clamp", "<i4"), ("pad", "<i4")])
assert UNIFORM_COLUMN_DTYPE.itemsize == 64
assert ACTION_REF_DTYPE.itemsize == 40
assert ACTION_APPLY_REF_DTYPE.itemsize == 56
assert ENTITY_IO_DTYPE.itemsize == 72
assert AGENT_IO_DTYPE.itemsize == 32
assert JOINT_IO_DTYPE.itemsize == 16
assert RAY_TARGET_DTYPE.itemsize == 48 and ctypes.sizeof(VmasRayTarget) == 48
assert ctypes.sizeof(VmasEntityDesc) == 84
assert ctypes.sizeof(VmasShapeRef) == 56


class NativeLibraryError(RuntimeError):
    pass


_lib = None


def load_library(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load (once) and return the native library.  Raises NativeLibraryError if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise NativeLibraryError(
            f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the MI355X engine has no Python fallback)"
        )
    lib = ctypes.CDLL(str(p))
    lib.vmas_abi_version.restype = _i32
    lib.vmas_device_count.restype = _i32
    lib.vmas_last_error.restype = ctypes.c_char_p
    lib.vmas_host_waits.restype = _i32
    lib.vmas_host_waits.argtypes = []
    lib.vmas_test_hold.restype = _i32
    lib.vmas_test_hold.argtypes = [_i32, _i32, ctypes.c_int64, _vp]
    lib.vmas_balance_outputs.restype = _i32
    lib.vmas_balance_outputs.argtypes = [_i32, _vp, _vp]
    lib.vmas_test_exact_math.restype = _i32
    lib.vmas_test_exact_math.argtypes = [_i32, _vp, _vp, _vp, ctypes.c_int64, _vp]
    lib.vmas_test_fast_trig.restype = _i32
    lib.vmas_test_fast_trig.argtypes = [_i32, _vp, _vp, ctypes.c_int64, _vp]
    lib.vmas_discovery_outputs.restype = _i32
    lib.vmas_discovery_outputs.argtypes = [_i32, _vp, _vp]
    lib.vmas_transport_outputs.restype = _i32
    lib.vmas_transport_outputs.argtypes = [_i32, _vp, _vp]
    lib.vmas_flocking_outputs.restype = _i32
    lib.vmas_flocking_outputs.argtypes = [_i32, _vp, _vp]
    lib.vmas_distance_vjp.restype = _i32
    lib.vmas_distance_vjp.argtypes = [_i32, _i32, _i32, _vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    lib.vmas_cast_rays_vjp.restype = _i32
    lib.vmas_cast_rays_vjp.argtypes = [_i32, _i32, _i32, _vp, _i32, _i32, _vp, _i32, _i32, _vp, _i32, _vp, _i32,
                                       ctypes.c_float, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    lib.vmas_world_step_vjp.restype = _i32
    lib.vmas_world_step_vjp.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    lib.vmas_spawn_targets.restype = _i32
    lib.vmas_spawn_targets.argtypes = [_i32, _vp, ctypes.POINTER(ctypes.c_uint64), _vp]
    lib.vmas_spawn_scratch_words.restype = ctypes.c_int64
    lib.vmas_spawn_scratch_words.argtypes = [_i32, _i32]
    lib.vmas_spawn_channel_create.restype = _i32
    lib.vmas_spawn_channel_create.argtypes = [_i32, ctypes.POINTER(_vp)]
    lib.vmas_spawn_channel_destroy.restype = _i32
    lib.vmas_spawn_channel_destroy.argtypes = [_vp]
    lib.vmas_spawn_channel_in.restype = _i32
    lib.vmas_spawn_channel_in.argtypes = [_vp, ctypes.POINTER(_vp)]
    lib.vmas_spawn_channel_arm.restype = _i32
    lib.vmas_spawn_channel_arm.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
    lib.vmas_spawn_channel_wait.restype = _i32
    lib.vmas_spawn_channel_wait.argtypes = [_vp, ctypes.c_uint32, ctypes.POINTER(_i32), _i32, _vp]
    lib.vmas_spawn_profile.restype = _i32
    lib.vmas_spawn_profile.argtypes = [_vp, ctypes.c_int64]
    lib.vmas_copy_spans.restype = _i32
    lib.vmas_copy_spans.argtypes = [_i32, _vp, _i32, _vp]
    lib.vmas_copy_spans_draw.restype = _i32
    lib.vmas_copy_spans_draw.argtypes = [_i32, _vp, _i32, ctypes.c_int64, _vp, _i32, ctypes.c_uint64, ctypes.c_uint64,
                                         _vp, _i32, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64), _vp]
    lib.vmas_stream_abort_capture.restype = _i32
    lib.vmas_stream_abort_capture.argtypes = [_vp]
    lib.vmas_graph_launch.restype = _i32
    lib.vmas_graph_launch.argtypes = [_vp, _vp]
    lib.vmas_graph_chain_build.restype = _i32
    lib.vmas_graph_chain_build.argtypes = [_vp, _i32, ctypes.POINTER(_vp)]
    lib.vmas_graph_chain_launch.restype = _i32
    lib.vmas_graph_chain_launch.argtypes = [_vp, _vp]
    lib.vmas_graph_chain_free.restype = _i32
    lib.vmas_graph_chain_nodes.restype = _i32
    lib.vmas_graph_chain_nodes.argtypes = [_vp]
    lib.vmas_graph_chain_fused.restype = _i32
    lib.vmas_graph_chain_fused.argtypes = [_vp]
    lib.vmas_graph_chain_set_writeback.restype = _i32
    lib.vmas_graph_chain_set_writeback.argtypes = [_vp, ctypes.c_int64]
    lib.vmas_graph_chain_launch_wb.restype = _i32
    lib.vmas_graph_chain_launch_wb.argtypes = [_vp, _vp]
    lib.vmas_test_tail_draw.restype = _i32
    lib.vmas_test_tail_draw.argtypes = [_i32, _vp, _i32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64, _i32, _vp, _vp]
    lib.vmas_graph_chain_launch_tail.restype = _i32
    lib.vmas_graph_chain_launch_tail.argtypes = [_vp, _i32, _vp, _i32, ctypes.c_int64, _vp, _i32, ctypes.c_uint64,
                                                 ctypes.c_uint64, _vp, _i32, ctypes.c_int64, _vp, _vp]
    lib.vmas_graph_chain_free.argtypes = [_vp]
    lib.vmas_world_create.restype = _i32
    lib.vmas_world_create.argtypes = [_vp, _vp, _vp, _vp, ctypes.POINTER(_vp)]
    lib.vmas_world_destroy.restype = _i32
    lib.vmas_world_destroy.argtypes = [_vp]
    lib.vmas_world_step.restype = _i32
    lib.vmas_world_step.argtypes = [_vp, _vp, _vp, _vp]
    lib.vmas_world_set_timing.restype = _i32
    lib.vmas_world_set_timing.argtypes = [_vp, _i32]
    lib.vmas_world_get_timing.restype = _i32
    lib.vmas_world_get_timing.argtypes = [_vp, _i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    lib.vmas_cast_rays.restype = _i32
    lib.vmas_cast_rays.argtypes = [
        _i32, _i32, _i32, _vp, _i32, _i32, _vp, _i32, _i32, _vp, _i32, _vp, _i32, _f32, _vp, _vp,
    ]
    lib.vmas_check_actions.restype = _i32
    lib.vmas_check_actions.argtypes = [_i32, _i32, _vp, _i32, _vp, _vp]
    lib.vmas_apply_actions.restype = _i32
    lib.vmas_apply_actions.argtypes = [_i32, _i32, _vp, _i32, _vp, _vp, _vp]
    lib.vmas_apply_actions_launch.restype = _i32
    lib.vmas_apply_actions_launch.argtypes = [_i32, _i32, _vp, _i32, _vp, ctypes.POINTER(ctypes.c_uint32), _vp]
    lib.vmas_apply_actions_flags.restype = _i32
    lib.vmas_apply_actions_flags.argtypes = [_i32, ctypes.c_uint32, _i32, _vp, _vp]
    lib.vmas_uniform_columns.restype = _i32
    lib.vmas_uniform_columns.argtypes = [_i32, ctypes.c_int64, _vp, _i32, ctypes.c_uint64, ctypes.c_uint64, _i32,
                                         ctypes.POINTER(ctypes.c_uint64), _vp]
    lib.vmas_uniform_columns_snap.restype = _i32
    lib.vmas_uniform_columns_snap.argtypes = [_i32, ctypes.c_int64, _vp, _i32, ctypes.c_uint64, ctypes.c_uint64, _i32,
                                              ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64), _vp]
    lib.vmas_assert_create.restype = _i32
    lib.vmas_assert_create.argtypes = [_i32, _i32, ctypes.POINTER(_vp)]
    lib.vmas_assert_destroy.restype = _i32
    lib.vmas_assert_destroy.argtypes = [_vp]
    lib.vmas_assert_publish.restype = _i32
    lib.vmas_assert_publish.argtypes = [_vp, _i32, _vp, ctypes.c_int64, _vp]
    lib.vmas_assert_wait.restype = _i32
    lib.vmas_assert_wait.argtypes = [_vp, _i32, ctypes.c_uint32, ctypes.POINTER(_i32), _vp]
    lib.vmas_assert_publish_range.restype = _i32
    lib.vmas_assert_publish_range.argtypes = [_vp, _i32, _vp, ctypes.c_int64, ctypes.c_int64, _i32, _i32, _vp, _vp, _vp]
    lib.vmas_flocking_target_action.restype = _i32
    lib.vmas_flocking_target_action.argtypes = [_i32, _vp, _i32, _f32, _vp, _vp]
    lib.vmas_distance.restype = _i32
    lib.vmas_distance.argtypes = [_i32, _i32, _i32, _vp, _vp, _vp, _i32, _i32, _vp, _vp]
    lib.vmas_spawn_resolve.restype = _i32
    lib.vmas_spawn_resolve.argtypes = [
        _i32, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _i32, _i32, _f32, _vp, _vp,
        ctypes.POINTER(_i32), ctypes.POINTER(_i32), _vp,
    ]
    lib.vmas_aux_last_error.restype = ctypes.c_char_p
    lib.vmas_jit_world_create.restype = _i32
    lib.vmas_jit_world_create.argtypes = [_vp, _vp, _vp, _vp, ctypes.POINTER(_vp)]
    lib.vmas_jit_world_destroy.restype = _i32
    lib.vmas_jit_world_destroy.argtypes = [_vp]
    lib.vmas_jit_world_step.restype = _i32
    lib.vmas_jit_world_step.argtypes = [_vp, _vp, _vp, _vp]
    lib.vmas_jit_world_set_timing.restype = _i32
    lib.vmas_jit_world_set_timing.argtypes = [_vp, _i32]
    lib.vmas_jit_world_get_timing.restype = _i32
    lib.vmas_jit_world_get_timing.argtypes = [_vp, _i32, ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_int64)]
    lib.vmas_jit_world_source.restype = _i32
    lib.vmas_jit_world_source.argtypes = [_vp, _vp, ctypes.c_int64]
    lib.vmas_jit_compile_check.restype = _i32
    lib.vmas_jit_compile_check.argtypes = [_vp, _vp, _vp, _vp, _vp, ctypes.c_int64]
    lib.vmas_jit_world_profile.restype = _i32
    lib.vmas_jit_world_profile.argtypes = [_vp, _vp, ctypes.c_int64]
    lib.vmas_jit_world_passes.restype = _i32
    lib.vmas_jit_world_passes.argtypes = [_vp, ctypes.POINTER(_i32)]
    lib.vmas_jit_world_device_timing.restype = _i32
    lib.vmas_jit_world_device_timing.argtypes = [_vp, _i32, ctypes.POINTER(ctypes.c_double),
                                                 ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]
    lib.vmas_jit_world_check.restype = _i32
    lib.vmas_jit_world_check.argtypes = [_vp]
    lib.vmas_jit_world_grid.restype = _i32
    lib.vmas_jit_world_grid.argtypes = [_vp]
    lib.vmas_jit_world_set_params.restype = _i32
    lib.vmas_jit_world_set_params.argtypes = [_vp, _vp, _vp, _vp, _vp]
    lib.vmas_jit_stats.restype = _i32
    lib.vmas_jit_stats.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    lib.vmas_jit_last_error.restype = ctypes.c_char_p
    lib.vmas_jit_world_epilogue.restype = _i32
    lib.vmas_jit_world_epilogue.argtypes = [_vp]
    lib.vmas_jit_program_outputs.restype = _i32
    lib.vmas_jit_program_outputs.argtypes = [_vp, _i32, _vp, _vp]
    ver = lib.vmas_abi_version()
    if ver != VMAS_ABI_VERSION:
        raise NativeLibraryError(f"ABI version mismatch: library {ver}, python {VMAS_ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load_library().vmas_last_error().decode(errors="replace")
        raise NativeLibraryError(f"{what} failed ({rc}): {msg}")


def check_jit(rc: int, what: str) -> None:
    """Error check of the world-specialised step entry points (csrc/vmas_jit.hip)."""
    if rc < 0:
        msg = load_library().vmas_jit_last_error().decode(errors="replace")
        raise NativeLibraryError(f"{what} failed ({rc}): {msg}")


def check_aux(rc: int, what: str) -> None:
    """Error check of the auxiliary entry points (csrc/vmas_spawn.hip)."""
    if rc != 0:
        msg = load_library().vmas_aux_last_error().decode(errors="replace")
        raise NativeLibraryError(f"{what} failed ({rc}): {msg}")


def jit_stats():
    """(hipRTC compiles so far, code objects in the bounded cache) of this process."""
    c, n = ctypes.c_int64(0), ctypes.c_int64(0)
    load_library().vmas_jit_stats(ctypes.byref(c), ctypes.byref(n))
    return c.value, n.value


# ---- the host half of a graph-mode step (csrc/vmas_host.cpp, the _vmas_host torch extension) -----
HOST_EXT_PATH = Path(__file__).resolve().parent / "_vmas_host.so"
_host = None


def load_host():
    """Load (once) and return the _vmas_host extension: the per-step host work of a replayed step
    (fresh outputs + the post-replay copy launch, the random-action draw) in C++.  Raises
    NativeLibraryError if it is missing -- graph mode on a GPU has no Python stand-in for it."""
    global _host
    if _host is not None:
        return _host
    if not HOST_EXT_PATH.exists():
        raise NativeLibraryError(
            f"{HOST_EXT_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    import importlib.util

    load_library()  # (first: the extension calls into this library through the pointers below)
    spec = importlib.util.spec_from_file_location("_vmas_host", HOST_EXT_PATH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    if mod.ABI_VERSION != VMAS_ABI_VERSION:
        raise NativeLibraryError(f"_vmas_host ABI {mod.ABI_VERSION} != library ABI {VMAS_ABI_VERSION}")
    _host = mod
    return mod


_fn_addrs = {}


def fn_addr(name: str) -> int:
    """Address of a C entry point of the loaded library (handed to _vmas_host; cached: the library
    stays loaded for the process's life)."""
    a = _fn_addrs.get(name)
    if a is None:
        a = _fn_addrs[name] = ctypes.cast(getattr(load_library(), name), ctypes.c_void_p).value
    return a
