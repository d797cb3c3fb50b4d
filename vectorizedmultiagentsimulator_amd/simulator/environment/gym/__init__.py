"""Gym / Gymnasium wrappers of an Environment (ref vmas/simulator/environment/gym/__init__.py).
Importing this package needs `gym`, as in the reference."""
from .gym import GymWrapper  # noqa: F401
