"""Seeding (reference ``utils/utils.py:28-35``).

The reference set ``cudnn.deterministic=True`` *and* ``benchmark=True`` (contradictory, A14).
Here ``deterministic`` is one explicit switch: our HIP kernels are deterministic by construction
(no float atomics in reductions that feed parameters), and for the stock torch backend it maps to
``torch.use_deterministic_algorithms`` / MIOpen deterministic mode.
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch


def set_seed(seed: int, deterministic: bool = False):
    random.seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = deterministic
    torch.backends.cudnn.benchmark = not deterministic
