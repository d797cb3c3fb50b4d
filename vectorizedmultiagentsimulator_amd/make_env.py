# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""make_env (restates vmas/make_env.py:13-100)."""
from __future__ import annotations

from typing import Optional, Union

from . import scenarios
from .simulator.environment import Environment, Wrapper
from .simulator.scenario import BaseScenario
from .simulator.utils import DEVICE_TYPING


def make_env(
    scenario: Union[str, BaseScenario],
    num_envs: int,
    device: DEVICE_TYPING = "cpu",
    continuous_actions: bool = True,
    wrapper: Optional[Union[Wrapper, str]] = None,
    max_steps: Optional[int] = None,
    seed: Optional[int] = None,
    dict_spaces: bool = False,
    multidiscrete_actions: bool = False,
    clamp_actions: bool = False,
    grad_enabled: bool = False,
    terminated_truncated: bool = False,
    wrapper_kwargs: Optional[dict] = None,
    graph_step: Optional[bool] = None,
    **kwargs,
):
    """Create a vectorized environment.

    Same arguments as the reference's ``vmas.make_env``.  ``device`` may be ``"cpu"`` (host
    backend of the native engine) or a ROCm device such as ``"cuda"`` / ``"cuda:0"`` (gfx950
    kernels).  ``scenario`` is a scenario file name from ``scenarios/`` or a BaseScenario.
    ``graph_step`` (not in the reference): True replays each step as one HIP graph once the world
    is warm, with the same results (ROCm devices; simulator/environment/_graph.py); False keeps
    the eager step; None (default) picks the graph where it is known to be exact -- a ROCm device,
    continuous actions, no autograd, one of this package's scenarios (Environment._auto_graph_step).
    """
    if isinstance(scenario, str):
        if not scenario.endswith(".py"):
            scenario += ".py"
        scenario = scenarios.load(scenario).Scenario()
    env = Environment(
        scenario,
        num_envs=num_envs,
        device=device,
        continuous_actions=continuous_actions,
        max_steps=max_steps,
        seed=seed,
        dict_spaces=dict_spaces,
        multidiscrete_actions=multidiscrete_actions,
        clamp_actions=clamp_actions,
        grad_enabled=grad_enabled,
        terminated_truncated=terminated_truncated,
        graph_step=graph_step,
        **kwargs,
    )
    if wrapper is not None and isinstance(wrapper, str):
        wrapper = Wrapper[wrapper.upper()]
    if wrapper_kwargs is None:
        wrapper_kwargs = {}
    return wrapper.get_env(env, **wrapper_kwargs) if wrapper is not None else env
