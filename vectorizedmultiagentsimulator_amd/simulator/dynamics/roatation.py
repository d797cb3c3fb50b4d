# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""The reference's module name for rotation-only dynamics (vmas/simulator/dynamics/roatation.py,
sic): ``from vmas.simulator.dynamics.roatation import Rotation`` resolves here."""
from .rotation import Rotation  # noqa: F401
