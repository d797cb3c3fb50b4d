"""MI355X-native engine with the surface of VMAS (VectorizedMultiAgentSimulator) 1.5.0.

``make_env`` / ``Environment`` / ``BaseScenario`` / ``World`` keep the reference's API; the
physics step, LIDAR ray casting and distance queries run in ``libvmas_mi355x.so`` (hand-written
HIP kernels for gfx950, with a host backend of the same arithmetic for ``device="cpu"``).
"""
from .make_env import make_env
from .simulator.environment import Wrapper

__version__ = "1.5.0"


def render_interactively(*args, **kwargs):
    raise NotImplementedError("interactive rendering is not part of the MI355X engine")


scenarios = sorted(["balance", "transport", "discovery", "flocking"])
"""Benchmark scenarios restated for the engine."""

debug_scenarios = sorted(["pollock", "waterfall"])
"""Parity fixtures (all shape pairs; joints)."""

mpe_scenarios = []

__all__ = ["make_env", "render_interactively", "scenarios", "debug_scenarios", "mpe_scenarios", "Wrapper"]
