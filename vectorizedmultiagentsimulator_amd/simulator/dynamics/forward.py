# Derived from VMAS, Copyright (c) 2022-2024 ProrokLab (https://www.proroklab.org/), licensed under
# GPL-3.0; modified for this MI355X build.  See NOTICE.md.
"""Forward-only dynamics (dynamics/forward.py:9-20): a thrust along the agent's heading."""
import torch

from ..utils import TorchUtils, X
from .common import Dynamics


class Forward(Dynamics):
    @property
    def needed_action_size(self) -> int:
        return 1

    def process_action(self):
        a = self.agent
        force = torch.zeros(a.batch_dim, 2, device=a.device, dtype=torch.float)
        force[:, X] = a.action.u[:, 0]
        a.state.force = TorchUtils.rotate_vector(force, a.state.rot)
