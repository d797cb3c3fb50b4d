"""HIP-graph replay of ``Environment.step`` (opt-in: ``make_env(..., graph_step=True)``).

The reference's step is an eager tensor program: per step ~70 small kernels for balance
(scenario rewards / observations / dones around the physics launch), each launched from Python.
On the MI355X that host work, not the GPU, sets the step time.  Once a world is warm this module
captures everything after the action check -- ``env_process_action``, ``pre_step``,
``World.step`` (the k_world launch and its fixed-point control words), ``post_step`` and the
scenario's rewards / observations / infos / dones -- into ONE HIP graph
(``torch.cuda.CUDAGraph``: stream capture, hipGraphInstantiate, hipGraphLaunch) and replays it.

What a replay must honour, and how:
  * Actions.  The native action kernel (one launch, one host wait for the NaN / range flags, as
    the reference's asserts) runs eagerly before the replay and writes every agent's ``u`` into
    ONE persistent buffer, so the captured program reads the current actions.
  * State carried across steps by re-binding.  The reference creates new tensors every step
    (integration, core.py:2866-2907; scenario attributes such as balance's ``global_shaping``).
    A captured program reads the tensors that were bound when it was captured (X) and writes
    tensors of the graph pool (Y).  At capture the attributes of the simulator's objects (env,
    scenario, world, entities, entity states, agent actions, joint constraints) are diffed:
    every attribute re-bound from X to Y is a carried tensor, and before each replay its current
    value is copied Y -> X (one multi-tensor copy, grouped by storage: the engine's whole output
    buffer is one copy).
  * Changes made between steps.  In-place edits of Y (``reset_at`` -> ``set_pos(batch_index)``)
    travel with that copy.  A tracked attribute re-bound by the caller (``reset()``, ``set_pos``
    without an index) is copied into the captured tensor and the attribute pointed back at it.
    Entity / world parameter changes (mass, shape, substeps, ...) drop the graph; the next step
    runs eagerly and captures again.
  * Outputs.  The returned observations / rewards / dones / infos are fresh copies (the
    reference clones them too), made by one multi-tensor copy after the replay.  The same launch
    adds one to the step counter (``steps += 1``) when nothing in the step reads it (no
    ``max_steps``): one kernel node fewer per step.
  * Asserts on device tensors inside the step (a scripted agent's action range check,
    core.py:977-980) are captured as device checks (``_DeviceAsserts``); a failed one rolls the
    replayed step back -- the tensors the step modifies in place (found by version counters at
    capture) from a per-step backup, the carried tensors from their pre-step copies, the device
    generator -- and raises from the same step() call.
  * What cannot be captured -- a host sync inside the step (``.item()``, ``bool(t.any())``,
    the spawn sampler's rejection loop), a host-to-device copy
    of pageable memory, discrete or communication actions -- makes the capture fail; the
    simulator's objects are rolled back (nothing ran: capture only records) and the env stays
    eager.  ``env.graph_status`` says which.
  * Per-step host state.  A replay runs no Python, so host state the step changes would be
    frozen at its capture-time value.  The last eager step before the capture is watched: if it
    draws from a host RNG (torch CPU, numpy or Python ``random``, outside the host holes, which
    run eagerly in a replay too) or changes a plain Python number / string attribute of the
    tracked objects (a Python-int step counter), the env stays eager (``graph_reason`` says
    why).  Host state kept elsewhere (module globals, objects the tracker does not visit) stays
    a documented requirement: the benchmark scenarios keep all per-step state in device
    tensors; tests/test_graph.py checks replay == eager bit for bit.
"""
from __future__ import annotations

import ctypes
import gc
import operator
import os
import random
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch
from torch import Tensor

from ... import _native as N
from ..core import Agent

_VERSION = operator.attrgetter("_version")  # a tensor's version counter (map() without a Python frame)

WARM_STEPS = 2  # eager steps before the capture (JIT compile, engine tables, allocator warm)


def _tracked_objects(env) -> List[Any]:
    w = env.world
    objs = [env, env.scenario, w]
    for e in w.entities:
        objs.append(e)
        objs.append(e._state)
        a = getattr(e, "_action", None)
        if a is not None:
            objs.append(a)
        for sensor in getattr(e, "_sensors", None) or ():  # Lidar._last_measurement is re-bound per step
            objs.append(sensor)
    for jc in w._joints.values():
        objs.append(jc)
    seen = set()
    out = []
    for o in objs:
        if id(o) not in seen and hasattr(o, "__dict__"):
            seen.add(id(o))
            out.append(o)
    return out


def _package_scenario_class(scenario) -> bool:
    """The scenario's class is one of this package's own (its make_world defined in the class
    itself, in a file of the package's scenarios directory).  (make_env loads scenario modules
    afresh, without a package name: by source file.)"""
    scn_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                           "scenarios") + os.sep
    cls = type(scenario)
    return (cls.__qualname__ == "Scenario" and "make_world" in cls.__dict__
            and os.path.abspath(cls.make_world.__code__.co_filename).startswith(scn_dir))


def _own_scenario(scenario) -> bool:
    """The scenario is one of this package's own classes, unmodified: only then does the step's
    code hold the contracts DirectOutputs and the write-only attributes rely on."""
    if not _package_scenario_class(scenario):
        return False
    # a step-time method overridden on the instance (a monkeypatched reward / post_step ...) may
    # read a write-only attribute before the class's own code re-binds it
    inst = getattr(scenario, "__dict__", {})
    return not any(m in inst for m in _STEP_METHODS)


_STEP_METHODS = ("reward", "observation", "done", "info", "pre_step", "post_step", "process_action",
                 "env_process_action", "extra_render")

# The scenarios whose step code the replay trusts beyond the watched eager step (write-only
# attributes, direct outputs): the four benchmark scenarios, each held to its eager step by
# tests/test_graph.py (not every file of the scenarios directory -- the debug scenarios
# are replayed like a user's scenario).
_TRUSTED_FILES = ("balance.py", "transport.py", "discovery.py", "flocking.py")


def _trusted_scenario(scenario) -> bool:
    if not _own_scenario(scenario):
        return False
    f = os.path.abspath(type(scenario).make_world.__code__.co_filename)
    scn_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "scenarios")
    return os.path.dirname(f) == scn_dir and os.path.basename(f) in _TRUSTED_FILES


def _write_only(o, k: str, scn_cls=None) -> bool:
    """Attribute k of o is declared write-only within a step by o's own class (not inherited: a
    subclass may read it): `_vmas_graph_write_only`, a set of attribute names each step re-binds
    before anything in the step reads it -- or, for an attribute the scenario sets on its agents,
    by the scenario class (`_vmas_graph_write_only_agents`).  The replays then need no carry of its
    previous value."""
    if k in type(o).__dict__.get("_vmas_graph_write_only", ()):
        return True
    return (scn_cls is not None and isinstance(o, Agent)
            and k in scn_cls.__dict__.get("_vmas_graph_write_only_agents", ()))


def _host_rng_states():
    return torch.random.get_rng_state(), np.random.get_state(), random.getstate()


def _host_rng_changed(a, b) -> Optional[str]:
    if not torch.equal(a[0], b[0]):
        return "torch CPU generator"
    if a[1][0] != b[1][0] or not np.array_equal(a[1][1], b[1][1]) or tuple(a[1][2:]) != tuple(b[1][2:]):
        return "numpy global generator"
    if a[2] != b[2]:
        return "python random"
    return None


_PLAIN = (bool, int, float, str)


def _fingerprint(v, depth: int = 0):
    """What a step could change in place inside a Python container: its length and its plain
    values, tensors by identity (a tensor appended or re-bound inside a list), numpy arrays by
    content; None for anything else (not compared)."""
    t = type(v)
    if t in _PLAIN or v is None:
        return v
    if isinstance(v, Tensor):
        return ("tensor", id(v))
    if isinstance(v, np.ndarray):
        return ("ndarray", v.shape, str(v.dtype), v.tobytes() if v.size <= 4096 else hash(v.tobytes()))
    if depth >= 3:
        return None
    if t in (list, tuple) or isinstance(v, (list, tuple)):
        return (t.__name__, len(v), tuple(_fingerprint(x, depth + 1) for x in v[:256]))
    if isinstance(v, dict):
        items = list(v.items())[:256]
        return ("dict", len(v), tuple((repr(k), _fingerprint(x, depth + 1)) for k, x in items))
    if isinstance(v, (set, frozenset)):
        return (t.__name__, len(v))
    return None


def _plain_attrs(objs, strict: bool = False) -> Dict[Tuple[int, str], Any]:
    """Plain Python number / string attributes of the tracked objects (Python-side step state);
    strict (a scenario outside the trusted set): also the contents of Python containers and numpy
    arrays held by them (a history list appended to in place, a numpy counter ...)."""
    out = {}
    for o in objs:
        for k, v in o.__dict__.items():
            if type(v) in _PLAIN:
                out[(id(o), k)] = v
            elif strict and not isinstance(v, Tensor):
                fp = _fingerprint(v)
                if fp is not None:
                    out[(id(o), k)] = fp
    return out


def _tensors(tree, acc: List[Tensor]):
    if isinstance(tree, Tensor):
        acc.append(tree)
    elif isinstance(tree, (list, tuple)):
        for x in tree:
            _tensors(x, acc)
    elif isinstance(tree, dict):
        for x in tree.values():
            _tensors(x, acc)
    return acc


def _rebuild(tree, it):
    if isinstance(tree, Tensor):
        return next(it)
    if isinstance(tree, list):
        return [_rebuild(x, it) for x in tree]
    if isinstance(tree, tuple):
        return tuple(_rebuild(x, it) for x in tree)
    if isinstance(tree, dict):
        return {k: _rebuild(v, it) for k, v in tree.items()}
    return tree


class _CapturableConstants:
    """While a step is captured: ``torch.tensor(data, device=<gpu>)`` / ``torch.as_tensor`` of
    host data (scenario constants such as transport's colour vectors, built every step) would be
    a pageable host->device copy, which stream capture forbids.  They are built on the host,
    written into a pinned arena allocated before the capture, and copied with a captured memcpy
    from there; the arena lives as long as the graph, so every replay copies the same values."""

    ARENA_BYTES = 1 << 16

    def __init__(self):
        self.arena = torch.empty(self.ARENA_BYTES, dtype=torch.uint8).pin_memory()
        self.used = 0

    def _wrap(self, orig):
        def fn(data, *args, dtype=None, device=None, **kw):
            if device is not None and not isinstance(data, Tensor) and torch.device(device).type == "cuda" \
                    and not args and not kw.get("requires_grad", False):
                host = orig(data, dtype=dtype)
                n = host.numel() * host.element_size()
                start = (self.used + 15) & ~15
                if start + n > self.ARENA_BYTES:
                    raise GraphUnsupported("too many host constants in the captured step")
                self.used = start + n
                slot = self.arena[start: start + n].view(host.dtype).view(host.shape)
                slot.copy_(host)
                out = torch.empty(host.shape, dtype=host.dtype, device=device)
                out.copy_(slot, non_blocking=True)
                return out
            return orig(data, *args, dtype=dtype, device=device, **kw)

        return fn

    def __enter__(self):
        self.saved = (torch.tensor, torch.as_tensor)
        torch.tensor = self._wrap(self.saved[0])
        torch.as_tensor = self._wrap(self.saved[1])
        return self

    def __exit__(self, *exc):
        torch.tensor, torch.as_tensor = self.saved
        return False


def _bytes(t: Tensor) -> Tensor:
    """A contiguous tensor as a flat uint8 view."""
    return t.reshape(-1).view(torch.uint8)


def _storage_key(t: Tensor) -> int:
    return t.untyped_storage().data_ptr()


class GraphUnsupported(RuntimeError):
    pass


def _assert_unwatched(ok: Tensor, msg: str):
    """The trial step's sink: the reference's eager assert, not counted as a host sync of the
    step (a captured step defers it to the device, _DeviceAsserts)."""
    mode = torch.cuda.get_sync_debug_mode()
    torch.cuda.set_sync_debug_mode(0)
    try:
        holds = bool(ok)
    finally:
        torch.cuda.set_sync_debug_mode(mode)
    assert holds, msg


class _DeviceAsserts:
    """Asserts on device tensors inside a captured step (a scripted agent's action range check,
    core.py:977-980).  At capture each one becomes a native kernel (vmas_assert_publish) that
    publishes the condition with a per-replay epoch into mapped host memory; after a replay the
    host waits for every slot's word of that replay (the kernels run at the start of the graph,
    so the wait overlaps the rest of it) and raises the reference's AssertionError, in order,
    from the same step() call, after rolling the replayed step back (StepGraph._rollback: the
    world is left as the eager step leaves it when the assert fires)."""

    MAX_SLOTS = 64
    # channels of dropped graphs: freed at the next creation (outside any capture), never from
    # __del__, which the garbage collector may run while another env's step is being captured
    # (freeing device / pinned memory during a capture aborts the process)
    _graveyard: List[ctypes.c_void_p] = []

    def __init__(self, dev):
        from ... import _native as N

        self.N = N
        self.lib = N.load_library()
        if not torch.cuda.is_current_stream_capturing():
            while _DeviceAsserts._graveyard:
                self.lib.vmas_assert_destroy(_DeviceAsserts._graveyard.pop())
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        h = ctypes.c_void_p()
        N.check_aux(self.lib.vmas_assert_create(idx, self.MAX_SLOTS, ctypes.byref(h)), "vmas_assert_create")
        self.h = h
        self.msgs: List[str] = []
        self.keep: List[Tensor] = []
        self.seq = 0

    def capture_sink(self, ok: Tensor, msg: str):
        if len(self.msgs) >= self.MAX_SLOTS:
            raise GraphUnsupported("too many device asserts in the captured step")
        ok = ok.reshape(-1)
        if ok.dtype is not torch.bool or not ok.is_contiguous():
            ok = ok.to(torch.bool).contiguous()
        stream = ctypes.c_void_p(torch.cuda.current_stream(ok.device).cuda_stream)
        self.N.check_aux(self.lib.vmas_assert_publish(self.h, len(self.msgs), ok.data_ptr(), ok.numel(), stream),
                         "vmas_assert_publish")
        self.keep.append(ok)
        self.msgs.append(msg)

    def capture_range(self, u: Tensor, mult: Tensor, rng: Tensor, msg: str) -> bool:
        """A scripted action's range check ((u / mult).abs() <= rng).all(), evaluated and
        published by one captured kernel (vmas_assert_publish_range); False (nothing done) when
        the operands are not the fp32 [B, n] / [n] device tensors it takes."""
        if len(self.msgs) >= self.MAX_SLOTS:
            raise GraphUnsupported("too many device asserts in the captured step")
        if (u.dim() != 2 or any(t.dtype is not torch.float32 or t.device != u.device for t in (u, mult, rng))
                or mult.shape != (u.shape[1],) or rng.shape != (u.shape[1],) or not mult.is_contiguous()
                or not rng.is_contiguous()):
            return False
        stream = ctypes.c_void_p(torch.cuda.current_stream(u.device).cuda_stream)
        self.N.check_aux(self.lib.vmas_assert_publish_range(self.h, len(self.msgs), u.data_ptr(), u.stride(0),
                                                            u.stride(1), u.shape[0], u.shape[1], mult.data_ptr(),
                                                            rng.data_ptr(), stream), "vmas_assert_publish_range")
        self.keep += [u, mult, rng]
        self.msgs.append(msg)
        return True

    def after_replay(self, dev, raise_: bool = True):
        """Waits for this replay's words; raises the first violated assert (raise_) or only keeps
        the sequence in step (a replay that is rolled back for another reason)."""
        if not self.msgs:
            return
        self.seq = (self.seq + 1) & 0xFFFFFFFF or 1
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        bad = ctypes.c_int32(0)
        first = None
        for slot, msg in enumerate(self.msgs):
            self.N.check_aux(self.lib.vmas_assert_wait(self.h, slot, self.seq, ctypes.byref(bad), stream),
                             "vmas_assert_wait")
            if bad.value and first is None:
                first = msg
        if raise_:
            assert first is None, first

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h is not None and h.value:
            _DeviceAsserts._graveyard.append(h)


def _reset_generator_capture_state(dev):
    """After a failed capture torch's CUDA generator may still consider itself captured (the
    capture epilogue never ran), which makes every later random op raise.  One tiny successful
    capture runs the prologue / epilogue pair again; the caller restores the RNG state after."""
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            torch.empty(1, device=dev).uniform_()
        del g
    except Exception:  # noqa: BLE001 -- best effort; the eager step reports any real problem
        pass


class _KernelChain:
    """A raw-launched step graph that is a chain of at most MAX_NODES kernel nodes, replayed as
    plain launches of those kernels on the stream (csrc/vmas_kernels.hip vmas_graph_chain_build):
    on MI355X a replayed graph costs the GPU ~5 us more than its kernels launched on the stream,
    and the post-replay launch after it starts ~2.3 us later (tools/launch_gap_probe.py,
    profiles/r05/run7_launch_gap) -- ~7 us of a ~56 us C2 step.  The launches are the captured
    nodes' own (function, grid, argument block), in the chain's order, so a replay runs the same
    kernels on the same arguments as the graph would -- except that a world module's k_world node
    followed by the same module's scenario-program node (k_program_jit) becomes ONE launch of
    k_world with the program as its epilogue (Args.epi; csrc/vmas_programs.hpp), the same compiled
    code on the same values, per 64-env group after the group's step.  Holds the graph: the
    nodes' argument blocks belong to it."""

    MAX_NODES = int(os.environ.get("VMAS_GRAPH_CHAIN_MAX", "8"))

    def __init__(self, graph, handle, n_nodes, fused):
        self.graph = graph
        self.handle = handle
        self.addr = handle.value  # (handed to _vmas_host's post / post_draw, which launch it)
        self.n_nodes = n_nodes  # launches per replay
        self.fused = fused  # k_world + k_program_jit pairs run as one launch (the program as k_world's epilogue)

    @classmethod
    def build(cls, graph) -> Tuple[Optional["_KernelChain"], str]:
        try:
            raw = graph.raw_cuda_graph()
        except Exception as ex:  # noqa: BLE001 -- a graph not kept: replay it as a graph
            return None, f"graph not kept ({type(ex).__name__})"
        lib = N.load_library()
        out = ctypes.c_void_p()
        rc = lib.vmas_graph_chain_build(ctypes.c_void_p(raw), cls.MAX_NODES, ctypes.byref(out))
        if rc != 0 or not out.value:
            return None, lib.vmas_last_error().decode(errors="replace")
        return cls(graph, out, lib.vmas_graph_chain_nodes(out), lib.vmas_graph_chain_fused(out)), ""

    def set_writeback(self, backup_delta: int) -> bool:
        """The write-back variant of the chain's k_world launch (vmas_graph_chain_set_writeback):
        False when the chain has no k_world launch."""
        return N.load_library().vmas_graph_chain_set_writeback(self.handle, int(backup_delta)) == 0

    def __del__(self):
        h, self.handle = getattr(self, "handle", None), None
        if h is not None and h.value:
            try:
                N.load_library().vmas_graph_chain_free(h)
            except Exception:  # noqa: BLE001 -- interpreter shutdown
                pass


class _Segments:
    """Capture of a step that contains host holes: code that must run on the host every step
    because it waits on the device -- the spawn sampler's rejection loop (utils.py:272-319),
    whose number of tries, and so the generator's advance, depends on the device data.  Such
    code reaches the capture through ``world._hole_sink`` (``ScenarioUtils.find_random_pos_for_
    entity``).  The capture ends the current graph there, runs that graph for real, runs the
    hole eagerly (its waits are now allowed) and captures the rest of the step into the next
    graph, all graphs in one memory pool.  A replay runs graph 0, hole 0 (writing into the same
    output tensor the next graph reads), graph 1, ... -- the reference's order of device work
    and of generator use.  Without holes it is a single graph, captured as torch.cuda.graph
    does."""

    def __init__(self, side: torch.cuda.Stream):
        self.side = side
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.holes: List[Tuple[Any, tuple, Tensor]] = []
        self.cur: Optional[torch.cuda.CUDAGraph] = None
        self.ran = False

    def begin(self):
        # keep_graph: the captured hipGraph_t stays readable after instantiation (its kernel nodes
        # are what a chain replay launches, _KernelChain)
        self.cur = torch.cuda.CUDAGraph(keep_graph=StepGraph._CHAIN)
        self.cur.capture_begin(pool=self.pool)

    def end(self):
        g, self.cur = self.cur, None
        g.capture_end()
        self.graphs.append(g)

    def hole(self, fn, args):
        if not isinstance(args, tuple):
            raise GraphUnsupported("host hole arguments must be a tuple")
        self.end()
        self.ran = True
        self.graphs[-1].replay()  # the work before the hole, for real
        res = fn(*args)
        if not isinstance(res, Tensor):
            raise GraphUnsupported("a host hole must return one tensor")
        self.holes.append((fn, args, res))
        self.begin()
        return res


_STATE_KEYS = ("_pos", "_vel", "_rot", "_ang_vel", "_force", "_torque")
_WB_KEYS = ("_pos", "_vel", "_rot", "_ang_vel")  # (the fields k_world's state write-back covers)


class DirectOutputs:
    """Fused programs writing a replay's outputs straight into fresh tensors: no
    copy of the step's observations / rewards / done after the replay.

    During the capture a fused scenario launch asks for its outputs here (_fused.direct_outputs):
    per category (obs, rewards, done) one buffer in the graph's pool, split into the members it
    returns, and three device words its kernel adds to those pointers (out_delta).  After the
    capture a category is relocated only when the step returns each of its members as is and
    nothing modified them in place (version counters) -- an op of the captured step that reads a
    member to build another output would read the captured buffer, which no replay writes any
    more -- and the scenario is one of this package's own classes (whose steps read their
    outputs nowhere else).  Each replay then writes into a fresh buffer allocated one step ahead
    (its offset from the captured buffer stored into the category's word by the previous
    post-replay launch, a VMAS_COPY_STORE64 span); the step hands out views of it, and the
    caching allocator recycles it once the caller drops them, as the reference's fresh tensors.
    Categories left out keep their words at 0: the kernel writes the captured buffer, and the
    post-replay launch copies it out as before."""

    MAX_LAUNCHES = 16

    def __init__(self, dev):
        self.dev = torch.device(dev)
        # (allocated outside the capture: the post-replay launches write them)
        self.words = torch.zeros(3 * self.MAX_LAUNCHES, dtype=torch.int64, device=self.dev)
        self.regions: List[dict] = []
        self.launches = 0
        self.enabled: List[dict] = []

    def launch(self, specs):
        k = self.launches
        if k >= self.MAX_LAUNCHES:
            return None, [None, None, None]
        self.launches += 1
        out = []
        for c, spec in enumerate(specs):
            if spec is None:
                out.append(None)
                continue
            dt, shape, n = spec
            numel = n * int(np.prod(shape, dtype=np.int64))
            buf = torch.empty(numel * torch.empty((), dtype=dt).element_size(), dtype=torch.uint8, device=self.dev)
            members = list(buf.view(dt).view(n, *shape).unbind(0))
            self.regions.append({"buf": buf, "dtype": dt, "members": members,
                                 "word": self.words.data_ptr() + 8 * (3 * k + c)})
            out.append(members)
        return self.words.data_ptr() + 24 * k, out

    def finalize(self, out_tensors, scenario) -> None:
        """Which categories the replays relocate (see the class notes)."""
        own = _trusted_scenario(scenario)
        ids = {id(t) for t in out_tensors}
        self.enabled = [r for r in self.regions
                        if own and r["buf"]._version == 0 and all(id(m) in ids for m in r["members"])]

    def arm(self, stream) -> None:
        """Before the first replay: each relocated category's first fresh buffer and its word."""
        if not self.enabled:
            return
        tbl = np.zeros(len(self.enabled), dtype=N.COPY_SPAN_DTYPE)
        for i, r in enumerate(self.enabled):
            cur = torch.empty_like(r["buf"])
            r["box"] = [cur]  # (the buffer the next replay writes: OutputAlloc moves it on)
            tbl[i] = ((cur.data_ptr() - r["buf"].data_ptr()) % (1 << 64), r["word"], N.VMAS_COPY_STORE64)
        dev = self.dev.index if self.dev.index is not None else torch.cuda.current_device()
        N.copy_table_at(dev, tbl.ctypes.data, 0, len(tbl), stream)
        self._arm_tbl = tbl  # (the launch reads its arguments at enqueue time; kept for clarity)


class _FreshState:
    """Fresh entity-state tensors after every replay, made on first use.

    A replay writes the integrated state into the same graph-pool tensors Y every step, and the
    entity states stay bound to views of Y.  The reference creates new state tensors every step
    (core.py:2866-2907): a reference kept to ``entity.state.pos`` from an earlier step keeps that
    step's values.  So after each replay this holder is marked pending, and the first read of any
    entity state attribute (EntityState / AgentState getters) materialises the step: every carried
    state attribute is re-bound to a view of a fresh copy F of its Y storage (one vmas_copy_spans
    launch, stream-ordered between this replay and the next).  Until then a step costs nothing
    extra.  Before the next replay (StepGraph.before_actions) the attributes are bound back to Y;
    if F was written in place meanwhile (reset_at -> set_pos(batch_index)) F is copied back to Y
    first.  References the caller kept point into F and keep their values."""

    def __init__(self, graph: "StepGraph", items, persist_items=()):
        self.g = graph
        self.items = items  # [(state object's __dict__, key, the Y view bound after the capture)]
        # agents' action._u / a holonomic state._force: views of the persistent action buffer P
        # (the same views every step, not carried); fresh copies of P on first use, never copied
        # back (every step rewrites P from its actions)
        self.persist_items = list(persist_items)
        self.pending = False
        self.bound = None  # after materialize: ([(dict, key, y, f)], [(F, version, Y bytes, F bytes)])

    def materialize(self) -> None:
        self.pending = False
        if self.bound is not None:
            return
        by_storage: Dict[int, list] = {}
        for d, k, y in self.items:
            if d.get(k) is y:  # (an attribute the caller re-bound keeps the caller's tensor)
                by_storage.setdefault(_storage_key(y), []).append((d, k, y))
        items, stor, spans = [], [], []
        self._materialize_persist(items, spans)
        for _, group in by_storage.items():
            y0 = group[0][2]
            ys = y0.untyped_storage()
            nb = ys.nbytes()
            if all(y.dtype is torch.float32 for _, _, y in group) and nb % 4 == 0:
                f = torch.empty(nb // 4, dtype=torch.float32, device=y0.device)
                for d, k, y in group:
                    v = f.as_strided(y.shape, y.stride(), y.storage_offset())
                    d[k] = v
                    items.append((d, k, y, v))
            else:  # (mixed dtypes: one byte buffer, a view of it per attribute)
                f = torch.empty(nb, dtype=torch.uint8, device=y0.device)
                for d, k, y in group:
                    v = torch.empty(0, dtype=y.dtype, device=y.device).set_(
                        f.untyped_storage(), y.storage_offset(), y.shape, y.stride())
                    d[k] = v
                    items.append((d, k, y, v))
            spans.append((ys.data_ptr(), f.data_ptr(), nb))
            stor.append((f, ys.data_ptr(), nb, items[-len(group):]))
        if spans:
            N.copy_raw(self.g._dev_index(), spans, self.g._stream())
        self.bound = (items, [(f, tuple(map(_VERSION, [v for *_, v in its])), yp, nb) for f, yp, nb, its in stor])

    def _materialize_persist(self, items, spans) -> None:
        env = self.g.env
        pc = env._u_persist
        if not self.persist_items or pc is None:
            return
        P = pc[1]
        live = [(d, k, y) for d, k, y in self.persist_items
                if d.get(k) is y and y.untyped_storage().data_ptr() == P.untyped_storage().data_ptr()]
        if not live:
            return
        sh = env._ushadow
        if sh.active:  # (a draw already rewrote P: its snapshot, itself a fresh tensor, holds the step's values)
            for d, k, y in live:
                v = sh.view(y)
                d[k] = v
                items.append((d, k, y, v))
            return
        f = torch.empty(P.numel(), dtype=torch.float32, device=P.device)
        spans.append((P.data_ptr(), f.data_ptr(), 4 * P.numel()))
        base = P.storage_offset()
        for d, k, y in live:
            v = f.as_strided(y.shape, y.stride(), y.storage_offset() - base)
            d[k] = v
            items.append((d, k, y, v))

    def unbind(self) -> bool:
        """Bind the attributes back to Y before a replay; F copied back to Y where it was written
        in place.  Returns whether Y changed."""
        self.pending = False
        b, self.bound = self.bound, None
        if b is None:
            return False
        items, stor = b
        spans = []
        for f, vers, yp, nb in stor:
            its = [v for (_, _, _, v) in items if v.untyped_storage().data_ptr() == f.untyped_storage().data_ptr()]
            if tuple(map(_VERSION, its)) != vers:
                spans.append((f.data_ptr(), yp, nb))
        if spans:
            N.copy_raw(self.g._dev_index(), spans, self.g._stream())
        for d, k, y, v in items:
            if d.get(k) is v:
                d[k] = y
        return bool(spans)


class StepGraph:
    """Capture / replay state of one Environment (see the module docstring)."""

    def __init__(self, env):
        self.env = env
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.status = "warming"
        self.eager_steps = 0
        self.replays = 0
        self._out_tree = None
        self._out_tensors: List[Tensor] = []
        self._carry_dst: List[Tensor] = []  # X (read by the graph)
        self._carry_src: List[Tensor] = []  # Y (written by the graph)
        self._watch: List[Tuple[dict, str, Tensor]] = []  # (obj.__dict__, key, bound tensor)
        self._watch_cols = None  # the same as three parallel tuples (dicts, keys, tensors)
        self._first_replay = True
        self._asserts: Optional[_DeviceAsserts] = None
        self._inplace: List[Tensor] = []
        self._write_only_ys: List[Tensor] = []  # (re-bound, not carried: _write_only)
        self._bk_src: List[Tensor] = []
        self._bk_dst: List[Tensor] = []
        self._bk_u: Optional[Tensor] = None
        self._raw_exec: Optional[ctypes.c_void_p] = None
        self._chain: Optional[_KernelChain] = None
        self.chain_why = ""  # why a replay is not a kernel chain (diagnostics)
        self._segments: List[torch.cuda.CUDAGraph] = []  # one graph per stretch between host holes
        self._holes: List[Tuple[Any, tuple, Tensor]] = []  # (fn, args, output) run after segment i
        self._executed = None  # outputs of a capture step that already ran (segmented capture)
        self._carry_ys: List[Tensor] = []  # the Y tensors as bound (version counters)
        self._post: Optional[dict] = None  # what the last post-replay launch covered (_post_replay)
        self._direct: Optional[DirectOutputs] = None  # (the capture's directly written outputs)
        # launches captured with their host side deferred (world._deferred_sink: discovery's
        # DeferredRespawn): armed before every replay, finished after its host work is queued
        self._deferred: List[Any] = []
        # Environment.steps += 1 (ref environment.py:397) folded into the post-replay launch (an
        # increment span of vmas_copy_spans) instead of a kernel node of the graph: set while the
        # capture records body(), kept for the captured graph (_steps_folded)
        self._folding = False
        self._steps_folded = False
        self._steps_t = None
        self._fresh: Optional[_FreshState] = None  # fresh entity states on first use after a replay
        # the state write-back (_writeback_ready): the carry index of the engine's state buffer, and
        # None (not tried) / False (not possible) / {chain, backup}
        self._state_idx: Optional[int] = None
        self._wb = None

    # ---- the step -------------------------------------------------------------------------------
    def body(self):
        """Everything of Environment.step after the actions (environment.py:394-412)."""
        env = self.env
        for agent in env.world.agents:
            env.scenario.env_process_action(agent)
        env.scenario.pre_step()
        env.world.step()
        env.scenario.post_step()
        if not self._folding:
            env.steps += 1
        return env._get_from_scenario(get_observations=True, get_infos=True, get_rewards=True, get_dones=True)

    def before_actions(self):
        """Bring the tensors a replay reads up to date, BEFORE the step's actions are applied (as
        the eager step orders it): tensors re-bound by the caller are copied into the captured
        ones, carried state is copied forward.  (A tracked tensor may alias the action buffer --
        a holonomic agent's force is a view of u -- so the fresh actions must land last.)"""
        # (copied: this call wrote tracked tensors, which may alias the persistent action buffer:
        # random actions applied into it by their draw are then stale -- Environment._take_preapplied)
        self.copied = False
        if self.graph is None:
            return
        fr = self._fresh
        if fr is not None and fr.bound is not None and fr.unbind():
            self.copied = True  # (Y written from F: the carry Y -> X runs again)
            self._post = None
        self.env.world.engine.check_device_errors()
        if not self._still_valid():
            self.drop("world or entity parameters changed")
            return
        env = self.env
        if self._steps_folded and (env.max_steps is not None or (env.steps is not self._steps_t and not self._fold_steps_ok())):
            # (max_steps set: the done program reads steps)
            self.drop("max_steps set or Environment.steps re-bound after the capture")
            return
        w = self._watch_cols
        # (every watched attribute still bound to its tensor: two C-level passes, no Python loop)
        if w is not None and all(map(operator.is_, map(dict.get, w[0], w[1]), w[2])):
            w = None
        for d, k, t in (self._watch if w is not None else ()):
            cur = d.get(k, None)
            if cur is not t:
                if not isinstance(cur, Tensor) or cur.shape != t.shape or cur.dtype != t.dtype:
                    self.drop(f"attribute {k} re-bound to a tensor of another shape")
                    return
                with torch.no_grad():
                    try:
                        t.copy_(cur)
                    except RuntimeError:
                        # the captured tensor is a broadcast view (a user's set_pos(t.expand(B, 2))
                        # keeps the expanded tensor): not writable per element -- the same values
                        # keep the capture, others drop it (the env recaptures)
                        if not torch.equal(cur, t):
                            self.drop(f"attribute {k} re-bound: its captured tensor is a broadcast view")
                            return
                d[k] = t
                self.copied = True
        if not self._first_replay and not self._carry_current():
            self.copied = True
            self._post = None
            with torch.no_grad():
                if self._carry_dst:
                    N.copy_spans(self._dev_index(), list(zip(self._carry_dst, self._carry_src)), self._stream())
                for x, y in self._carry_other:
                    x.copy_(y)

    def step(self):
        """Run the post-action part of a step (actions already applied; before_actions ran before
        them); returns its results."""
        if self.graph is None:
            if self.status in ("warming", "dropped"):
                if self.eager_steps >= WARM_STEPS:
                    if self._capture():
                        if self._executed is not None:  # a segmented capture ran the step already
                            out, self._executed = self._clone_outputs(), None
                            self._asserts.after_replay(self.env.device)
                            return out
                        return self._replay()
                elif self.eager_steps == WARM_STEPS - 1:
                    self.eager_steps += 1
                    return self._trial()
            self.eager_steps += 1
            return self.body()
        return self._replay()

    def _trial(self):
        """The last eager step before the capture, watched for host waits: torch's synchronising
        ops (sync debug mode "warn") and the native library's (vmas_host_waits).  A step that waits
        on the device cannot be captured -- a wait inside a capture invalidates it -- so such an
        env stays eager without attempting one."""
        import warnings

        from ... import _native as N

        lib = N.load_library()
        w0 = lib.vmas_host_waits()
        mode = torch.cuda.get_sync_debug_mode()
        consts = _CapturableConstants()  # host constants go through a pinned arena, as in capture
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            torch.cuda.set_sync_debug_mode(1)
            self.env.world._assert_sink = _assert_unwatched
            hole_waits = [0]

            def hole(fn, args):  # a host hole runs eagerly in a captured step: its waits are allowed
                m = torch.cuda.get_sync_debug_mode()
                torch.cuda.set_sync_debug_mode(0)
                h0 = lib.vmas_host_waits()
                try:
                    return fn(*args)
                finally:
                    hole_waits[0] += (lib.vmas_host_waits() - h0) & 0xFFFFFFFF
                    torch.cuda.set_sync_debug_mode(m)

            rng_cur = [_host_rng_states()]
            rng_used = [None]
            # device generator use outside the holes: a captured step that draws device random
            # numbers besides the respawn keeps the respawn as a host hole (a deferred
            # respawn reads the generator before the replay, so it would share those numbers)
            dgen = torch.cuda.default_generators[torch.device(self.env.device).index or 0]
            d_off0, hole_adv = dgen.get_offset(), [0]

            def hole(fn, args, _inner=hole):  # host RNG use inside a hole is replayed eagerly too
                if rng_used[0] is None:
                    rng_used[0] = _host_rng_changed(rng_cur[0], _host_rng_states())
                o0 = dgen.get_offset()
                try:
                    return _inner(fn, args)
                finally:
                    rng_cur[0] = _host_rng_states()
                    hole_adv[0] += dgen.get_offset() - o0

            self.env.world._hole_sink = hole
            objs = _tracked_objects(self.env)
            # (strict for a class outside the package: the package's scenarios keep their own
            # Python-side caches of the fused programs, keyed by tensor versions, which are not step state)
            strict = not _package_scenario_class(self.env.scenario)
            plain0 = _plain_attrs(objs, strict)
            try:
                with consts:
                    out = self.body()
            finally:
                self.env.world._assert_sink = None
                self.env.world._hole_sink = None
                torch.cuda.set_sync_debug_mode(mode)
            if rng_used[0] is None:
                rng_used[0] = _host_rng_changed(rng_cur[0], _host_rng_states())
            self._device_rng_outside_holes = (dgen.get_offset() - d_off0 - hole_adv[0]) != 0
            plain1 = _plain_attrs(objs, strict)
            changed = sorted(k for k in set(plain0) | set(plain1) if plain0.get(k) != plain1.get(k))
        self._trial_consts = consts  # the arena outlives the copies that read it
        # torch's warning: "called a synchronizing CUDA operation" (not the notice that the mode
        # is a prototype, which set_sync_debug_mode emits itself)
        syncs = [str(r.message).splitlines()[0] for r in rec
                 if "synchronizing" in str(r.message) and "prototype" not in str(r.message)]
        native = ((lib.vmas_host_waits() - w0) & 0xFFFFFFFF) - hole_waits[0]
        if syncs or native:
            self.status = "eager"
            self.why = ("host sync in the step: " + (syncs[0] if syncs else f"{native} native host wait(s)"))[:300]
        elif rng_used[0] is not None:
            self.status = "eager"
            self.why = f"the step draws from a host RNG ({rng_used[0]}): a replay would repeat its numbers"
        elif changed:
            names = {id(o): type(o).__name__ for o in objs}
            self.status = "eager"
            self.why = ("the step changes Python-side state a replay would freeze: "
                        + ", ".join(f"{names.get(i, '?')}.{k}" for i, k in changed[:4]))[:300]
        return out

    _AHEAD_DEFERRED = os.environ.get("VMAS_GRAPH_DRAW_AHEAD_DEFERRED", "1") != "0"  # (A/B knob)

    def _ahead_offset_word(self):
        """Where a draw made ahead in the post-replay launch reads its generator offset: 0 (the
        host passes it) without deferred launches; with one spawn channel (discovery's respawn,
        whose host side advances the generator only after this launch is queued) the device word
        the respawn launch leaves it in (VMAS_SPAWN_OFF_END_WORD); None: no draw ahead."""
        if not self._deferred:
            return 0
        if len(self._deferred) != 1 or not self._AHEAD_DEFERRED:
            return None
        mx = getattr(getattr(self._deferred[0], "chan", None), "mx", None)
        return None if mx is None else mx.data_ptr() + 4 * N.VMAS_SPAWN_OFF_END_WORD

    def _finish_deferred(self, apply: bool = True, out=None):
        """The host side of the captured deferred launches (discovery's respawn).  One that had to
        be redone on the host (DeferredRespawn.finish) changed state the graph's observations had
        already read: the step's observations in ``out`` are recomputed eagerly.  A draw made ahead
        at the device offset the respawn left gets that offset now -- the generator's, once the
        respawn's tries are accounted -- or is dropped when the respawn was redone (its offset
        word is then not what the host loop leaves)."""
        err, redone = None, False
        for d in self._deferred:
            try:
                redone |= bool(d.finish(apply))
            except Exception as ex:  # noqa: BLE001 -- drain every channel, then raise the first
                err = err or ex
        sp = getattr(self.env, "_spec", None)
        if sp is not None and sp[3] is None:
            if err is not None or redone or not apply:
                self.env._spec = None
            else:
                self.env._spec = sp[:3] + (sp[0][5].get_offset(),) + sp[4:]
        if err is not None:
            raise err
        if redone and out is not None:
            env = self.env
            obs = env._get_from_scenario(get_observations=True, get_rewards=False, get_infos=False,
                                         get_dones=False)[0]
            dst = out[0]
            for a, b in (zip(dst.values(), obs.values()) if isinstance(dst, dict) else zip(dst, obs)):
                for x, y in zip(_tensors(a, []), _tensors(b, [])):
                    x.copy_(y)

    def drop(self, why: str):
        fr, self._fresh = self._fresh, None
        if fr is not None:  # (eager steps read the attributes as bound: F views hold the values)
            fr.pending = False
            for d, k, y in fr.items + fr.persist_items:
                if d.get("_fresh") is fr:
                    d.pop("_fresh")
        self._finish_deferred(apply=False)
        self._deferred = []
        self.graph = None
        self._raw_exec = None
        self._chain = None
        self._segments, self._holes = [], []
        self.status = "dropped"
        self.why = why
        self.eager_steps = 0
        self._out_tree = None
        self._out_tensors = []
        self._carry_dst, self._carry_src, self._watch = [], [], []
        self._state_idx, self._wb = None, None
        self._watch_cols = None
        self._carry_ys, self._post = [], None
        self._steps_folded = False

    # ---- capture --------------------------------------------------------------------------------
    _FOLD_STEPS = os.environ.get("VMAS_GRAPH_FOLD_STEPS", "1") != "0"  # (A/B knob)

    def _fold_steps_ok(self) -> bool:
        """Whether the capture leaves `steps += 1` to the post-replay launch: nothing in the
        captured step reads steps (no max_steps: the done program reads it, ref
        environment.py:415-418) and it is a contiguous fp32 tensor on the step's device."""
        st = getattr(self.env, "steps", None)
        return (self._FOLD_STEPS and self.env.max_steps is None and isinstance(st, Tensor)
                and st.dtype is torch.float32 and st.is_contiguous() and st.device.type == "cuda")

    def _capture(self) -> bool:
        env = self.env
        eng = env.world.engine
        objs = _tracked_objects(env)
        snap = [(o, dict(o.__dict__)) for o in objs]
        # version counters of every tracked tensor: those the step modifies in place are what a
        # speculative replay has to back up (see replay_speculative)
        versions = {}
        for _, d in snap:
            for v in d.values():
                if isinstance(v, Tensor):
                    versions[id(v)] = (v, v._version)
        dev = env.device
        rng = torch.cuda.get_rng_state(dev)
        consts = _CapturableConstants()
        side = torch.cuda.Stream(dev)
        prev_stream = torch.cuda.current_stream(dev)
        from .. import _engine

        _engine.drain_deferred()  # engines collected during an earlier capture
        env._raw_outputs = True
        asserts = _DeviceAsserts(dev)
        # No garbage collection inside the capture: a finalizer run there (another env's graph,
        # engine or device buffers) would free device memory while the stream is captured, which
        # aborts the process.  Collect now, then keep the collector off until the capture ends.
        gc.collect()
        gc_was_on = gc.isenabled()
        gc.disable()
        # contents of every tracked tensor: a capture that hits a host hole runs the segments
        # before the hole for real, so a failure after that has state to restore
        # (a view with a zero stride over a dimension of size > 1 -- the LIDAR's expanded angle
        # row -- cannot be written in place, so the step cannot have changed it)
        contents = [(t, t.clone()) for t, _ in versions.values()
                    if not any(st == 0 and n > 1 for st, n in zip(t.stride(), t.shape))]
        segs = _Segments(side)
        self._direct = DirectOutputs(dev) if self._DIRECT else None
        deferred: List[Any] = []

        def deferred_sink(d):  # captured here; armed / finished around each replay
            d.capture()
            deferred.append(d)

        try:
            env.world._assert_sink = asserts.capture_sink
            env.world._assert_range_sink = asserts.capture_range
            env.world._hole_sink = segs.hole
            # (the deferred form only when the step draws no other device random numbers)
            env.world._deferred_sink = None if getattr(self, "_device_rng_outside_holes", True) else deferred_sink
            env.world._direct_out = self._direct
            torch.cuda.synchronize(dev)
            self._folding = self._fold_steps_ok()
            with torch.cuda.stream(side), consts:
                segs.begin()
                out = self.body()
                segs.end()
                if segs.holes:  # the last segment too: the capture step has then run the step
                    segs.graphs[-1].replay()
            prev_stream.wait_stream(side)
            g = segs.graphs[0]
            self._consts = consts
            self._asserts = asserts
            self._sig = eng.graph_token()
            if self._direct is not None and not segs.holes:  # (a segmented step keeps its copies)
                self._direct.finalize(_tensors(out, []), env.scenario)
            self._plan(objs, snap, out)
            if self._direct is not None:
                self._direct.arm(N.stream_ptr(self._dev_index()))
            self._inplace = [t for t, v in versions.values() if t._version != v]
            ids = {id(t) for t in self._inplace}
            self._inplace += [y for y in self._write_only_ys if id(y) not in ids]
            self._bk_src: List[Tensor] = []
            self._bk_dst: List[Tensor] = []
            self._bk_u = None
        except Exception as ex:  # noqa: BLE001 -- any capture failure means "stay eager"
            # a capture invalidated by a forbidden call may be left open: end it, so that the
            # eager step that follows can launch
            N.load_library().vmas_stream_abort_capture(ctypes.c_void_p(side.cuda_stream))
            # capture_end may raise with the capture stream current: go back to the caller's
            torch.cuda.set_stream(prev_stream)
            torch.cuda.synchronize(dev)
            _reset_generator_capture_state(dev)
            for o, d in snap:
                o.__dict__.clear()
                o.__dict__.update(d)
            if segs.ran:  # segments before a hole ran for real: put the tensors back
                with torch.no_grad():
                    for t, c in contents:
                        t.copy_(c)
                torch.cuda.synchronize(dev)
            torch.cuda.set_rng_state(rng, dev)
            self.status = "eager"
            self.why = f"{type(ex).__name__}: {str(ex).splitlines()[0] if str(ex) else ''}"[:300]
            self.graph = None
            self._direct = None
            self._folding = False
            return False
        finally:
            if gc_was_on:
                gc.enable()
            env._raw_outputs = False
            env.world._assert_sink = None
            env.world._assert_range_sink = None
            env.world._hole_sink = None
            env.world._deferred_sink = None
            env.world._direct_out = None
        del contents
        self._steps_folded, self._folding = self._folding, False
        self._steps_t = env.steps
        persist = []
        pc = env._u_persist
        if pc is not None and pc[2] is not None:
            pkey = _storage_key(pc[1])
            for ag in env.world.agents:
                for o, k in ((ag._action, "_u"), (ag._state, "_force")):
                    t = o.__dict__.get(k)
                    if isinstance(t, Tensor) and _storage_key(t) == pkey:
                        persist.append((o.__dict__, k, t))
        if (self._fresh_items or persist) and self._FRESH_STATES:
            self._fresh = _FreshState(self, self._fresh_items, persist)
            for d, _, _ in self._fresh_items + persist:
                d["_fresh"] = self._fresh
        self._deferred = deferred
        self.graph = g
        self._segments, self._holes = segs.graphs, segs.holes
        self._raw_exec = None
        self._chain = None
        self.replays = 0
        self.status = "graph"
        self.why = ""
        self._first_replay = not segs.holes
        self._executed = out if segs.holes else None
        self._post = None
        return True

    def _plan(self, objs, snap, out):
        carry: List[Tuple[Tensor, Tensor]] = []
        names: List[str] = []
        state_field: List[bool] = []  # (an entity state's pos / vel / rot / ang_vel: what k_world integrates)
        fresh = []  # carried entity-state attributes: re-bound to fresh tensors on first use (_FreshState)
        # re-bound attributes no step reads before re-binding them (the package's own scenarios and
        # sensors declare them): not carried; a rollback restores them from the backups (_inplace)
        own = self._WRITE_ONLY and _trusted_scenario(self.env.scenario)
        self._write_only_ys = []
        for o, before in snap:
            after = o.__dict__
            for k, v0 in before.items():
                if not isinstance(v0, Tensor):
                    continue
                v1 = after.get(k, None)
                if v1 is v0:
                    continue
                if not isinstance(v1, Tensor) or v1.shape != v0.shape or v1.dtype != v0.dtype \
                        or v1.device != v0.device:
                    raise GraphUnsupported(f"attribute {type(o).__name__}.{k} changes type/shape in the step")
                if (_storage_key(v1) == _storage_key(v0) and v1.storage_offset() == v0.storage_offset()
                        and v1.stride() == v0.stride()):
                    continue  # a new view of the same memory (e.g. force = u[:, :2] every step)
                if own and _write_only(o, k, type(self.env.scenario)):  # (no step reads X: no carry, see _write_only)
                    self._write_only_ys.append(v1)
                    continue
                carry.append((v0, v1))
                names.append(f"{type(o).__name__}.{k}")
                state_field.append(k in _WB_KEYS and hasattr(type(o), "_fresh"))
                if k in _STATE_KEYS and hasattr(type(o), "_fresh"):  # (an EntityState / AgentState)
                    fresh.append((after, k, v1))
        self._carry_ys = [y for _, y in carry]
        self._carry_names = names  # (reporting: tools/post_table_probe.py)
        x_keys = {_storage_key(x): n for (x, _), n in zip(carry, names)}
        for (_, y), n in zip(carry, names):
            if _storage_key(y) in x_keys:
                raise GraphUnsupported(f"{n} is re-bound onto the storage that {x_keys[_storage_key(y)]} held "
                                       "before the step")
        # group carried pairs by (X storage, Y storage): same offsets / strides / storage size ->
        # one whole-storage copy (the engine's output buffer: every dynamic field at once)
        groups: Dict[Tuple[int, int], List[Tuple[Tensor, Tensor]]] = {}
        state_only: Dict[Tuple[int, int], bool] = {}
        for (x, y), sf in zip(carry, state_field):
            key = (_storage_key(x), _storage_key(y))
            groups.setdefault(key, []).append((x, y))
            state_only[key] = state_only.get(key, True) and sf
        dst, src = [], []
        state_pair = None  # (the whole-storage copy of the engine's state buffer: k_world can write it back)
        for key, pairs in groups.items():
            x0, y0 = pairs[0]
            sx, sy = x0.untyped_storage(), y0.untyped_storage()
            whole = (len(pairs) > 1 and sx.nbytes() == sy.nbytes()
                     and all(x.storage_offset() == y.storage_offset() and x.stride() == y.stride()
                             for x, y in pairs))
            if whole:
                dst.append(torch.empty(0, dtype=torch.uint8, device=x0.device).set_(sx))
                src.append(torch.empty(0, dtype=torch.uint8, device=y0.device).set_(sy))
                if state_only[key] and state_pair is None:
                    state_pair = (dst[-1], src[-1])
            else:
                for x, y in pairs:
                    dst.append(x)
                    src.append(y)
        # one multi-tensor copy kernel: contiguous pairs as flat byte views (one dtype), the rest
        # (non-contiguous views) copied one by one
        self._carry_dst, self._carry_src, self._carry_other = [], [], []
        self._state_idx, self._wb = None, None
        for x, y in zip(dst, src):
            if x.is_contiguous() and y.is_contiguous() and x.dtype == y.dtype:
                if state_pair is not None and x is state_pair[0]:
                    self._state_idx = len(self._carry_dst)
                self._carry_dst.append(_bytes(x))
                self._carry_src.append(_bytes(y))
            else:
                self._carry_other.append((x, y))
        # every tensor attribute of the tracked objects as bound after the capture: the caller
        # re-binding one of them between steps is detected by identity
        self._watch = []
        for o in objs:
            d = o.__dict__
            for k, v in d.items():
                if isinstance(v, Tensor):
                    self._watch.append((d, k, v))
        self._watch_cols = (tuple(d for d, _, _ in self._watch), tuple(k for _, k, _ in self._watch),
                            tuple(t for _, _, t in self._watch))
        self._fresh_items = fresh
        self._out_tree = out
        # an output marked constant (BaseScenario.done's all-False view of one element made outside
        # the capture, which no replay writes) is copied from a contiguous copy made once here:
        # part of the post-replay launch instead of a strided torch copy per step
        self._out_tensors = [t.contiguous() if getattr(t, "_vmas_constant", False) and not t.is_contiguous() else t
                             for t in _tensors(out, [])]

    def _still_valid(self) -> bool:
        return self.env.world.engine.graph_token() == self._sig

    # ---- replay ---------------------------------------------------------------------------------
    def _launch(self, defer_chain: bool = False, wb: bool = False):
        """One replay.  The first goes through torch (its prologue refreshes the generator state
        that captured random ops read); if it did not advance the device generator, the graph
        draws no random numbers and later replays launch the instantiated graph directly
        (vmas_graph_launch), without the prologue's two fill kernels."""
        if self._fresh is not None:  # (this replay's states: fresh tensors on first use)
            self._fresh.pending = True
        for d in self._deferred:  # the generator state the captured launches read
            d.arm()
        if self._holes:  # segmented step: graph, host hole, graph, ... (torch replays)
            for i, seg in enumerate(self._segments):
                seg.replay()
                if i < len(self._holes):
                    fn, args, res = self._holes[i]
                    fn(*args, out=res)
            return
        if self._chain is not None:  # the graph's kernels as plain launches (_KernelChain)
            if defer_chain:  # (launched by the post-replay call: _post_replay(chain=...))
                return self._chain
            self._launch_chain(self._chain, wb)
            return
        if self._raw_exec is not None:
            N.check(N.load_library().vmas_graph_launch(self._raw_exec, N.stream_ptr(self._dev_index())),
                    "vmas_graph_launch")
            return
        dev = self.env.device
        gen = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
        before = gen.get_offset()
        self.graph.replay()
        if self.replays == 0 and gen.get_offset() == before and self._RAW_LAUNCH:
            self._raw_exec = ctypes.c_void_p(self.graph.raw_cuda_graph_exec())
            self._chain, self.chain_why = _KernelChain.build(self.graph) if self._CHAIN else (None, "off")

    _RAW_LAUNCH = os.environ.get("VMAS_GRAPH_RAW_LAUNCH", "1") != "0"  # (A/B knob)
    # a replay whose graph is a short chain of kernel nodes launches them on the stream instead
    # (_KernelChain); 0: hipGraphLaunch (A/B knob)
    _CHAIN = os.environ.get("VMAS_GRAPH_CHAIN", "1") != "0"
    # a pre-applied replay's kernel chain launched by the post-replay C++ call (_vmas_host post /
    # post_draw) instead of its own ctypes call; 0: launched from Python first (A/B knob)
    _CHAIN_IN_POST = os.environ.get("VMAS_GRAPH_CHAIN_IN_POST", "1") != "0"
    # fused programs write the step's outputs into fresh tensors (DirectOutputs); 0: copied out
    _DIRECT = os.environ.get("VMAS_GRAPH_DIRECT_OUTPUTS", "1") != "0"
    # fresh entity-state tensors on first use after each replay (_FreshState); 0: the states stay
    # views of the graph's buffers (an alias kept across a step then sees later steps' values)
    _FRESH_STATES = os.environ.get("VMAS_GRAPH_FRESH_STATES", "1") != "0"
    # declared write-only attributes (_write_only) are not carried between replays; 0: carried
    _WRITE_ONLY = os.environ.get("VMAS_GRAPH_WRITE_ONLY", "1") != "0"

    def _replay(self):
        asserts = self._asserts is not None and bool(self._asserts.msgs)
        if asserts:  # a failed device assert rolls the step back: back up what it modifies in place
            self.backup(None)
            rng = torch.cuda.get_rng_state(self.env.device)
        self._first_replay = False
        self._launch()
        self.replays += 1
        if asserts:  # (the post-replay carry overwrites X, which a rollback restores Y from)
            try:
                self._asserts.after_replay(self.env.device)
            except AssertionError:
                self._finish_deferred(apply=False)
                self._rollback(rng, restore_actions=False)
                raise
        out = self._post_replay()
        self._finish_deferred(out=out)
        return out

    # ---- speculative replay ---------------------------------------------------------------------
    def backup(self, u_buf: Optional[Tensor]):
        """Copies of the tensors the step modifies in place (found by version counters at
        capture) -- and, before the action kernel of a speculative step, of the persistent action
        buffer -- so that a step can be undone (one multi-tensor copy kernel)."""
        if not self._bk_dst or (u_buf is not None and self._bk_u is not u_buf):
            self._bk_src = [*self._inplace] + ([u_buf] if u_buf is not None else [])
            self._bk_dst = [torch.empty_like(t) for t in self._bk_src]
            self._bk_u = u_buf
            self._post = None
        n = len(self._bk_src) if u_buf is not None else len(self._inplace)
        if n and not self._backup_current(n):
            with torch.no_grad():
                pairs = list(zip(self._bk_dst[:n], self._bk_src[:n]))
                if all(d.is_contiguous() and s.is_contiguous() for d, s in pairs):
                    N.copy_spans(self._dev_index(), pairs, self._stream())
                else:
                    torch._foreach_copy_(self._bk_dst[:n], self._bk_src[:n])

    def rollback_free(self) -> bool:
        """No device assert in the captured step: a step whose actions pass by construction (drawn
        and applied by get_random_actions) can then never be rolled back."""
        return self._asserts is None or not self._asserts.msgs

    def replay_preapplied(self):
        """One replay of a step whose actions were drawn and applied by the draw's own launch and
        that has no device asserts (rollback_free): the speculative replay without its backups and
        generator snapshot, which only a rollback reads."""
        self._first_replay = False
        wb = self._writeback_ready()
        chain = self._launch(defer_chain=self._CHAIN_IN_POST, wb=wb)
        self.replays += 1
        out = self._post_replay(chain=chain, wb=wb)
        self._finish_deferred(out=out)
        return out

    # The state write-back (a rollback-free replay only): the chain's k_world writes the integrated
    # state into its own inputs X as well as into the outputs Y (vmas_graph_chain_set_writeback; a
    # re-run fixed-point pass reads the pre-step state from a backup the first pass stores), so the
    # post-replay launch drops the whole-storage carry Y -> X of the engine's state buffer -- at C2 4.46
    # of its 5.8 MB (VERDICT r5 "Next" #2).  Only when that carry group holds nothing but entity
    # states' pos / vel / rot / ang_vel (exactly what k_world integrates and writes back) and the replay
    # is a kernel chain.  A speculative replay (a rollback restores Y from X) keeps the carry.  Only for
    # the trusted (benchmark) scenarios: X is overwritten INSIDE the step, so no kernel after k_world
    # may read the pre-step state -- their programs read the integrated state only; a user's reward
    # may keep last step's position (self.prev = agent.state.pos) and read it after World.step.
    # Measured (profiles/r06/run3_writeback, run6_writeback_size): the write-back's stores cost
    # k_world more than the carry costs the post-replay launch once the carried state is large --
    # C2's 4.5 MB carry: step 49.5 -> 48.0 us; C5 shard's 7.1 MB: 62.3 -> 63.2 us; C5 full's 57 MB:
    # 337 -> 362 us -- so it is used only up to VMAS_GRAPH_WRITEBACK_MAX_MB of carried state.
    _WRITEBACK = os.environ.get("VMAS_GRAPH_WRITEBACK", "1") != "0"  # (A/B knob)
    _WRITEBACK_MAX_BYTES = float(os.environ.get("VMAS_GRAPH_WRITEBACK_MAX_MB", "6")) * (1 << 20)

    def _writeback_ready(self) -> bool:
        w = self._wb
        if w is not None and w is not False and w["chain"] is self._chain:
            return True
        if w is False or self._chain is None:
            return False
        self._wb = False
        if (not self._WRITEBACK or self._state_idx is None or self._carry_other
                or not _trusted_scenario(self.env.scenario)):
            return False
        x = self._carry_dst[self._state_idx]
        if x.numel() * x.element_size() > self._WRITEBACK_MAX_BYTES:
            return False
        backup = torch.empty_like(x)  # (the first pass's copy of the pre-step state, same offsets)
        if not self._chain.set_writeback(backup.data_ptr() - x.data_ptr()):
            return False
        self._wb = {"chain": self._chain, "backup": backup}
        return True

    def replay_speculative(self, flags_ok):
        """Replays the step while the action kernel's flags are still in flight, then waits for
        them (flags_ok(): the host wait of the eager path, now overlapping the replay).  Passing
        flags: the replay's outputs, as _replay.  A failed flag: the step is rolled back -- the
        in-place-modified tensors and the action buffer from the backup, then every carried
        tensor from its pre-step copy, the device generator state -- and None is returned (the
        caller then raises the reference's AssertionError through the eager action check).  A
        scripted agent's failed assert rolls back everything but the policy agents' actions
        (set, as in the reference, before the scripted agents act) and raises."""
        dev = self.env.device
        rng = torch.cuda.get_rng_state(dev)
        self._first_replay = False
        self._launch()
        self.replays += 1
        # the host side of the post-replay copies (fresh output tensors, span table) while the
        # action kernel's flags are still in flight; nothing is launched before they pass
        prep = self._post_prepare()
        if not flags_ok():
            self._asserts.after_replay(dev, raise_=False)
            self._finish_deferred(apply=False)
            self._rollback(rng, restore_actions=True)
            return None
        try:
            self._asserts.after_replay(dev)
        except AssertionError:
            self._finish_deferred(apply=False)
            self._rollback(rng, restore_actions=False)
            raise
        # only now: the post-replay carry overwrites X, which a rollback restores Y from
        out = self._post_replay(prep)
        self._finish_deferred(out=out)
        return out

    def _rollback(self, rng: Tensor, restore_actions: bool):
        self._post = None
        n = len(self._bk_src) if restore_actions else len(self._inplace)
        with torch.no_grad():
            if n:
                torch._foreach_copy_(self._bk_src[:n], self._bk_dst[:n])
            if self._carry_dst:  # carried tensors: Y <- X (X holds the pre-step values)
                torch._foreach_copy_(self._carry_src, self._carry_dst)
            for x, y in self._carry_other:
                y.copy_(x)
        torch.cuda.set_rng_state(rng, self.env.device)

    # ---- copies after a replay -----------------------------------------------------------------
    def _launch_chain(self, chain, wb: bool = False) -> None:
        lib = N.load_library()
        fn = lib.vmas_graph_chain_launch_wb if wb else lib.vmas_graph_chain_launch
        N.check(fn(chain.handle, N.stream_ptr(self._dev_index())), "vmas_graph_chain_launch")

    _chain_fn_addr = None

    @classmethod
    def _chain_fn(cls, wb: bool = False) -> int:
        if cls._chain_fn_addr is None:
            cls._chain_fn_addr = (N.fn_addr("vmas_graph_chain_launch"), N.fn_addr("vmas_graph_chain_launch_wb"))
        return cls._chain_fn_addr[1 if wb else 0]

    def _dev_index(self) -> int:
        dev = torch.device(self.env.device)
        return dev.index if dev.index is not None else torch.cuda.current_device()

    def _stream(self):
        return N.stream_ptr(self._dev_index())

    def _carry_current(self) -> bool:
        """The last post-replay launch carried Y -> X and no Y was modified since (version
        counters: a native replay bumps none, a caller's in-place edit or the re-bind copy of
        before_actions bumps them)."""
        p = self._post
        return p is not None and p["carry_ver"] == tuple(map(_VERSION, self._carry_ys))

    def _backup_current(self, n: int) -> bool:
        p = self._post
        return (p is not None and p["bk_n"] >= n and self._carry_current()
                and p["bk_ver"] == tuple(map(_VERSION, self._inplace)))

    def _post_spans(self, wb: bool = False):
        """Per capture: the carry spans (Y -> X, contiguous byte views) and the backup spans of
        the next step (in-place tensors and the action buffer -> their backups; a backup whose
        tensor lies inside a carry destination X is taken from the matching bytes of Y, which
        is what X holds once the carry has run).  None if a backup straddles a carry destination
        or is not contiguous (then the backups stay in backup())."""
        carry = [(y.data_ptr(), x.data_ptr(), x.numel()) for i, (x, y) in enumerate(zip(self._carry_dst, self._carry_src))
                 if not (wb and i == self._state_idx)]  # (wb: k_world wrote the state back itself)
        bk = []
        n = len(self._bk_src) if self._bk_dst else 0
        for t, d in zip(self._bk_src[:n], self._bk_dst[:n]):
            if not (t.is_contiguous() and d.is_contiguous()):
                return carry, None, 0
            lo, nb = t.data_ptr(), t.numel() * t.element_size()
            src = lo
            for y, x, cn in carry:
                if lo < x + cn and x < lo + nb:  # overlaps carry destination X
                    if not (x <= lo and lo + nb <= x + cn):
                        return carry, None, 0
                    src = y + (lo - x)
            bk.append((src, d.data_ptr(), nb))
        return carry, bk, n

    def _post_prepare(self):
        """The host half of _post_replay: (span table, fresh output views, non-contiguous rest)."""
        t = self._post_table()
        if t["steps_row"] is not None:
            self._steps_current(t)
        views, rest = self._clone_alloc(t)
        return t, views, rest

    def _post_replay(self, prep=None, chain=None, wb: bool = False):
        """After a replay, in ONE native launch (vmas_copy_spans): the fresh copies of the
        outputs, the carry of the re-bound state to the next step (Y -> X, which before_actions
        then skips while no Y changes) and the next step's backups (which backup() then skips
        while no in-place tensor changes).  The outputs are copied before the carry when one
        of them lies in a carry destination (two launches).  The span table is built once per
        (capture, backup buffers): a step only writes its fresh outputs' addresses into it."""
        t = self._post_table(wb) if prep is None else None
        if chain is not None and (t is None or t["plain"] or t.get("host") is None):
            self._launch_chain(chain, wb)  # (a replay's kernel chain not yet launched: now, before anything else)
            chain = None
        if t is not None and not t["plain"]:
            # the common case in one C++ call (csrc/vmas_host.cpp OutputAlloc.post): the replay's
            # kernel chain (chain: not launched yet), fresh outputs, their addresses into the table,
            # the launch(es)
            if t["steps_row"] is not None:
                self._steps_current(t)
            host = t.get("host") or self._host_alloc(t)
            ch = (chain.addr, self._chain_fn(wb)) if chain is not None else (0, 0)
            mid, hi = (t["n_out"] if t["clash"] else 0), t["n_all"]
            # (with a deferred launch -- discovery's respawn, whose host side advances the generator
            # after this -- the draw reads its offset where the respawn launch leaves it)
            off_dev = self._ahead_offset_word()
            ahead = (self.env._draw_ahead_plan() if (hi - mid <= 96 and not t["n_bk"] and off_dev is not None)
                     else None)
            if ahead is not None:  # (+ the next step's random actions in the same launch)
                st, drawer, P = ahead
                # (a single fused launch: these items as its tail, _tail_ok)
                tail = N.fn_addr("vmas_graph_chain_launch_tail") if ch[0] and not mid and self._tail_ok(t) else 0
                views, acts, snap, seed, off, inc = N.load_host().post_draw(
                    host, drawer, mid, hi, P.data_ptr(), P.numel(), N.fn_addr("vmas_copy_spans_draw"), off_dev, *ch,
                    tail, int(wb))
                self.env._drew_ahead(st, acts, snap, seed, off, inc)
            else:
                views = host.post(mid, hi, *ch)
            rest = [(views[k], s) for k, s in t["loose"]]
            self._clone_finish(rest)
            self._post = {"carry_ver": tuple(map(_VERSION, self._carry_ys)),
                          "bk_ver": tuple(map(_VERSION, self._inplace)), "bk_n": t["n_bk"]}
            fn, consts = self._clone_build
            return fn(views, consts)
        t, views, rest = prep if prep is not None else self._post_prepare()
        dev, st = self._dev_index(), self._stream()
        tbl, n_out, n_all = t["addr"], t["n_out"], t["n_all"]
        if t["plain"]:  # non-contiguous carries / backups: the old order
            N.copy_table_at(dev, tbl, 0, n_out, st)
            t["host"].commit()
            self._clone_finish(rest)
            self._post = None
        else:
            if t["clash"]:
                N.copy_table_at(dev, tbl, 0, n_out, st)
                N.copy_table_at(dev, tbl, n_out, n_all, st)
            else:
                N.copy_table_at(dev, tbl, 0, n_all, st)
            t["host"].commit()
            self._clone_finish(rest)
            self._post = {"carry_ver": tuple(map(_VERSION, self._carry_ys)),
                          "bk_ver": tuple(map(_VERSION, self._inplace)), "bk_n": t["n_bk"]}
        fn, consts = self._clone_build
        return fn(views, consts)

    # The post-replay launch's items as the tail of the replay's one fused k_world launch
    # (csrc/vmas_tail.hpp, vmas_graph_chain_launch_tail): one launch per step instead of two.  A copy
    # then runs inside the launch that wrote its source, possibly on another XCD, so it is admitted
    # only when that source is written through: k_world's state outputs (stored sc1) and the
    # tensors a trusted scenario's program writes through (`_vmas_tail_sources()`: balance's global
    # shaping, position and ground rewards; transport's per-package distance, on-goal flag, colour and
    # shaping).  Store words and the step counter need nothing.
    _TAIL = os.environ.get("VMAS_GRAPH_TAIL", "1") != "0"  # (A/B knob)

    def _tail_ok(self, t) -> bool:
        ok = t.get("tail_ok")
        if ok is None:
            ok = t["tail_ok"] = self._tail_admit(t)
        return ok

    def _tail_admit(self, t) -> bool:
        ch, sc = self._chain, self.env.scenario
        srcs = getattr(sc, "_vmas_tail_sources", None)
        if (not self._TAIL or ch is None or ch.n_nodes != 1 or not ch.fused or srcs is None or t["plain"]
                or not _trusted_scenario(sc)):
            return False
        ranges = []
        try:
            tensors = list(srcs())
        except Exception:  # noqa: BLE001 -- (an attribute the declaration names is not bound: no tail)
            return False
        for v in tensors:
            if not isinstance(v, Tensor) or not v.is_contiguous() or v.device.type != "cuda":
                return False
            ranges.append((v.data_ptr(), v.data_ptr() + v.numel() * v.element_size()))
        if self._state_idx is not None:  # (the engine's output buffer: k_world's sc1 stores)
            y = self._carry_src[self._state_idx]
            ranges.append((y.data_ptr(), y.data_ptr() + y.numel()))
        for r in t["tbl"]:
            n, src = int(r["nbytes"]), int(r["src"])
            if n == N.VMAS_COPY_STORE64 or src == 0 or n == 0:
                continue
            if not any(lo <= src and src + n <= hi for lo, hi in ranges):
                return False
        return True

    def _post_table(self, wb: bool = False):
        """The post-replay span table (N.COPY_SPAN_DTYPE rows): the contiguous outputs (their
        destinations are filled per step by _clone_alloc), then the carry and backup spans."""
        ts = self._out_tensors
        if getattr(self, "_clone_src_of", None) is not ts:
            self._clone_plan()
            self._clone_src_of = ts
        cname = "_post_cache_wb" if wb else "_post_cache"  # (a table per variant: with / without the state carry)
        c = getattr(self, cname, None)  # (objects compared by identity, not id())
        if (c is not None and c[0] is ts and c[1] is self._bk_dst and c[2] == len(self._bk_dst)
                and c[3] == len(self._bk_src)):
            return c[4]
        out_rows = [(x.data_ptr(), 0, x.numel() * x.element_size()) for _, _, srcs in self._clone_group_srcs
                    for x in srcs if x.is_contiguous()]
        direct = self._direct.enabled if self._direct is not None else []
        direct_rows = []
        for r in direct:  # (the next replay's buffer offset: written by OutputAlloc.alloc)
            direct_rows.append(len(out_rows))
            out_rows.append((0, r["word"], N.VMAS_COPY_STORE64))
        steps_row = None
        if self._steps_folded:  # (last output row: the launch of the outputs always covers it)
            st = self.env.steps
            steps_row = len(out_rows)
            out_rows.append((0, st.data_ptr(), st.numel() * 4))
        carry, bk, n_bk = self._post_spans(wb)
        plain = bool(self._carry_other) or bk is None
        extra = [] if plain else carry + bk
        tbl = np.zeros(len(out_rows) + len(extra), dtype=N.COPY_SPAN_DTYPE)
        for i, row in enumerate(out_rows + extra):
            tbl[i] = row
        clash = any(lo < x + cn and x < lo + nb for lo, _, nb in out_rows if nb > 0 for _, x, cn in carry)
        t = {"tbl": tbl, "addr": tbl.ctypes.data, "n_out": len(out_rows), "n_all": len(out_rows) + len(extra),
             "plain": plain,
             "clash": clash, "n_bk": n_bk, "steps_row": steps_row, "steps": self.env.steps if self._steps_folded else None,
             "direct_rows": direct_rows,
             "contig": [[x.is_contiguous() for x in srcs] for _, _, srcs in self._clone_group_srcs]}
        setattr(self, cname, (ts, self._bk_dst, len(self._bk_dst), len(self._bk_src), t))
        return t

    def _steps_current(self, t) -> None:
        """Point the table's increment row at env.steps as bound now (reset() re-binds it)."""
        st = self.env.steps  # (checked by before_actions: fp32, contiguous, on the device)
        if t["steps"] is not st:
            t["tbl"][t["steps_row"]]["dst"] = st.data_ptr()
            t["tbl"][t["steps_row"]]["nbytes"] = st.numel() * 4
            t["steps"] = st

    def _host_alloc(self, t):
        """The table's OutputAlloc (csrc/vmas_host.cpp): per (dtype, shape) group one allocation
        split into its members, the contiguous members' addresses into the table's output rows."""
        groups, row, loose, start = [], 0, [], 0
        for (dt, shape, n), (_, _, srcs), contig in zip(self._clone_groups, self._clone_group_srcs, t["contig"]):
            ks = [k for k, c in enumerate(contig) if c]
            groups.append((srcs[0], list(shape), n, row, ks))
            loose += [(start + k, srcs[k]) for k, c in enumerate(contig) if not c]
            row += len(ks)
            start += n
        direct = self._direct.enabled if self._direct is not None else []
        regions = [(r["buf"], r["box"], r["members"][0], row,
                    [(list(m.shape), list(m.stride()), m.storage_offset()) for m in r["members"]])
                   for r, row in zip(direct, t["direct_rows"])]
        host = N.load_host().OutputAlloc(self._dev_index(), groups, t["tbl"], t["addr"], N.fn_addr("vmas_copy_spans"),
                                         N.fn_addr("vmas_aux_last_error"), regions)
        t["host"], t["loose"] = host, loose
        return host

    def _clone_alloc(self, t):
        """Fresh output tensors for one step, their addresses written into the table's output
        rows: (views in the plan's order, the non-contiguous (dst, src) rest)."""
        host = t.get("host") or self._host_alloc(t)
        views = host.alloc()
        return views, [(views[k], s) for k, s in t["loose"]]

    def _clone_alloc_py(self, t):
        """_clone_alloc in Python (kept as the statement of what OutputAlloc.alloc does)."""
        plan = t.get("alloc")
        if plan is None:  # per table: each group's rows and the byte offsets of its contiguous members
            plan, row = [], 0
            dev = self._out_tensors[0].device
            for (dt, shape, n), (_, _, srcs), contig in zip(self._clone_groups, self._clone_group_srcs, t["contig"]):
                step = int(np.prod(shape, dtype=np.int64)) * torch.empty((), dtype=dt).element_size()
                ks = [k for k, c in enumerate(contig) if c]
                plan.append(((n,) + shape, dt, dev, row, row + len(ks), np.array(ks, dtype=np.uint64) * np.uint64(step),
                             [(k, srcs[k]) for k, c in enumerate(contig) if not c]))
                row += len(ks)
            t["alloc"] = plan
        views = ()
        dst = t["tbl"]["dst"]
        rest = []
        for shape, dt, dev, r0, r1, offs, loose in plan:
            buf = torch.empty(shape, dtype=dt, device=dev)
            vs = buf.unbind(0)
            views += vs
            if r1 > r0:
                np.add(offs, buf.data_ptr(), out=dst[r0:r1], casting="unsafe")
            for k, src in loose:
                rest.append((vs[k], src))
        return views, rest

    def _clone_plan(self):
        """Outputs grouped by (dtype, shape): per group one allocation [n, *shape] whose unbind
        gives the n fresh tensors, all filled by the post-replay copy launch; the result tree rebuilt by a
        function generated for its structure.  Built once per capture (the replay's output tensors
        are fixed), so a step makes a handful of host calls instead of several per output."""
        ts = self._out_tensors
        direct = self._direct.enabled if self._direct is not None else []
        dmember = {id(m): (ri, mi) for ri, r in enumerate(direct) for mi, m in enumerate(r["members"])}
        groups: Dict[Tuple[torch.dtype, Tuple[int, ...]], List[int]] = {}
        for i, t in enumerate(ts):
            if id(t) not in dmember:  # (directly written: views of the replay's fresh buffer)
                groups.setdefault((t.dtype, tuple(t.shape)), []).append(i)
        plan = sorted(groups.items(), key=lambda kv: str(kv[0][0]))  # same dtypes adjacent
        self._clone_groups = [(dt, shape, len(idx)) for (dt, shape), idx in plan]
        order = [i for _, idx in plan for i in idx]  # position in the concatenated views -> output
        pos = {i: p for p, i in enumerate(order)}
        # the direct categories' members follow the groups' views (OutputAlloc.alloc's order)
        base, at = [], len(order)
        for r in direct:
            base.append(at)
            at += len(r["members"])
        for i, t in enumerate(ts):
            if id(t) in dmember:
                ri, mi = dmember[id(t)]
                pos[i] = base[ri] + mi
        # per (dtype, shape) group, in view order: its sources
        self._clone_group_srcs, start = [], 0
        for _, idx in plan:
            self._clone_group_srcs.append((start, start + len(idx), [ts[i] for i in idx]))
            start += len(idx)
        consts: List[Any] = []
        counter = [0]

        def expr(t):
            if isinstance(t, Tensor):
                counter[0] += 1
                return f"v[{pos[counter[0] - 1]}]"
            if isinstance(t, list):
                return "[" + ", ".join(expr(x) for x in t) + "]"
            if isinstance(t, tuple):
                return "(" + "".join(expr(x) + ", " for x in t) + ")"
            if isinstance(t, dict):
                items = []
                for k, x in t.items():
                    consts.append(k)
                    items.append(f"c[{len(consts) - 1}]: {expr(x)}")
                return "{" + ", ".join(items) + "}"
            consts.append(t)
            return f"c[{len(consts) - 1}]"

        body = expr(self._out_tree)
        fn = eval("lambda v, c: " + body)  # noqa: S307 -- generated from the output tree's structure only
        self._clone_build = (fn, consts)

    @staticmethod
    def _clone_finish(rest):
        for v, t in rest:
            v.copy_(t)

    def _clone_outputs(self):
        """Fresh copies of the replay's outputs (the reference returns fresh tensors too)."""
        t = self._post_table()
        if t["steps_row"] is not None:
            self._steps_current(t)
        views, rest = self._clone_alloc(t)
        N.copy_table_at(self._dev_index(), t["addr"], 0, t["n_out"], self._stream())
        t["host"].commit()
        self._clone_finish(rest)
        fn, consts = self._clone_build
        return fn(views, consts)
