"""Import alias for drop-in use: ``vmas.X`` is ``vectorizedmultiagentsimulator_amd.X``.

Scenario code written against the reference (``from vmas import make_env``, ``from
vmas.simulator.core import Agent, World``, ``from vmas.simulator.scenario import BaseScenario``
...; reference vmas/__init__.py) runs unchanged on this package: every ``vmas.<sub>`` module is
the same module object as ``vectorizedmultiagentsimulator_amd.<sub>`` (one class identity, one
engine), so isinstance checks and scenario registries agree between the two names.  Do not
install this next to the reference package: it takes its name."""
import importlib
import importlib.abc
import importlib.util
import sys

import vectorizedmultiagentsimulator_amd as _impl
from vectorizedmultiagentsimulator_amd import *  # noqa: F401,F403 -- the reference's top-level names
from vectorizedmultiagentsimulator_amd import __all__  # noqa: F401

_PREFIX, _TARGET = __name__ + ".", _impl.__name__ + "."


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """Resolves ``vmas.<sub>`` to the already-importable ``vectorizedmultiagentsimulator_amd.<sub>``."""

    def find_spec(self, name, path=None, target=None):
        if not name.startswith(_PREFIX):
            return None
        real = _TARGET + name[len(_PREFIX):]
        if importlib.util.find_spec(real) is None:
            return None
        return importlib.util.spec_from_loader(name, self, is_package=hasattr(importlib.import_module(real), "__path__"))

    def create_module(self, spec):
        return importlib.import_module(_TARGET + spec.name[len(_PREFIX):])

    def exec_module(self, module):  # the real module is already executed
        pass


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())
