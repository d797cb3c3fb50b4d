# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""PID velocity controller (vmas/simulator/controllers/velocity_controller.py:15-134): turns a
desired velocity in ``agent.action.u`` into a force, u = kP (e + I(e) + D(e)) * mass, e = desired -
current velocity.

Parameters (``ctrl_params``), as the reference reads them:
* ``pid_form="standard"``: (gain, integral time, derivative time), times in units of dt;
* ``pid_form="parallel"``: (kP, kI, kD) with integral time kP / kI and derivative time kD / kP.
An integral time of 0 disables the integrator; otherwise the accumulated error is clamped at the
anti-windup limit 0.5 * f_max * T_i / (dt * kP), f_max = the smaller of the agent's max_f and
f_range (a warning when neither is set)."""
import math
import warnings
from typing import Optional

import torch

from ..utils import TorchUtils


class VelocityController:
    def __init__(self, agent, world, ctrl_params=(1, 0, 0), pid_form: str = "standard"):
        self.agent = agent
        self.world = world
        self.dt = world.dt
        self.ctrl_gain = ctrl_params[0]
        if pid_form == "standard":
            self.integralTs = ctrl_params[1]
            self.derivativeTs = ctrl_params[2]
        elif pid_form == "parallel":
            self.integralTs = 0.0 if ctrl_params[1] == 0 else self.ctrl_gain / ctrl_params[1]
            self.derivativeTs = ctrl_params[2] / self.ctrl_gain
        else:
            raise Exception("PID form is either standard or parallel.")
        self.use_integrator = self.integralTs != 0
        if self.use_integrator:
            limits = [x for x in (self.agent.max_f, self.agent.f_range) if x is not None]
            fmax = min(limits) if limits else None
            if fmax is not None:
                self.integrator_windup_cutoff = 0.5 * fmax * self.integralTs / (self.dt * self.ctrl_gain)
            else:
                self.integrator_windup_cutoff = None
                warnings.warn("Force limits not specified. Integrator can wind up!")
        self.reset()

    def reset(self, index: Optional[int] = None):
        if index is None:
            shape = (self.world.batch_dim, self.world.dim_p)
            self.accum_errs = torch.zeros(shape, device=self.world.device)
            self.prev_err = torch.zeros(shape, device=self.world.device)
        else:
            self.accum_errs = TorchUtils.where_from_index(index, 0.0, self.accum_errs)
            self.prev_err = TorchUtils.where_from_index(index, 0.0, self.prev_err)

    def integralError(self, err):
        if not self.use_integrator:
            return 0
        self.accum_errs += self.dt * err
        if self.integrator_windup_cutoff is not None:
            self.accum_errs = self.accum_errs.clamp(-self.integrator_windup_cutoff, self.integrator_windup_cutoff)
        return (1.0 / self.integralTs) * self.accum_errs

    def rateError(self, err):
        rate = self.derivativeTs * (err - self.prev_err) / self.dt
        self.prev_err = err
        return rate

    def process_force(self):
        self.accum_errs = self.accum_errs.to(self.world.device)
        self.prev_err = self.prev_err.to(self.world.device)
        err = self.agent.action.u - self.agent.state.vel
        u = self.ctrl_gain * (err + self.integralError(err) + self.rateError(err))
        u *= self.agent.mass
        self.agent.action.u = u
