"""Import shims for the reference (majidsina/rlmd at /root/reference).

Test infrastructure only: used by ``make_golden.py`` in the build container to
generate golden vectors from the reference's own code.  The reference never
travels to the GPU box; only the ``.npz`` fixtures produced here do.

The shims are ordinary-error workarounds recorded in SURVEY.md §8c:
  * ``gym`` (0.24 in the reference's requirements) is absent: provide a stub
    with ``gym.Env`` and ``gym.spaces.Box`` (sample = uniform over [low, high]);
  * NumPy 2 removed ``np.float_`` / ``np.bool8``: alias them;
  * ``tools/eval_episodes.py:33`` imports ``pybullet_envs``: empty stub.
"""
import os
import sys
import types

import numpy as np

REF = "/root/reference"


def install() -> None:
    if not hasattr(np, "float_"):
        np.float_ = np.float64
    if not hasattr(np, "bool8"):
        np.bool8 = np.bool_

    if "gym" not in sys.modules:
        gym = types.ModuleType("gym")
        spaces = types.ModuleType("gym.spaces")

        class Env:
            pass

        class Box:
            def __init__(self, low, high, shape=None, dtype=np.float32):
                self.shape = tuple(shape) if shape is not None else np.shape(low)
                self.dtype = np.dtype(dtype)
                self.low = np.full(self.shape, low, dtype=self.dtype)
                self.high = np.full(self.shape, high, dtype=self.dtype)

            def sample(self):
                return np.random.uniform(self.low, self.high).astype(self.dtype)

        spaces.Box = Box
        gym.Env = Env
        gym.spaces = spaces
        sys.modules["gym"] = gym
        sys.modules["gym.spaces"] = spaces

    if "pybullet_envs" not in sys.modules:
        sys.modules["pybullet_envs"] = types.ModuleType("pybullet_envs")

    if REF not in sys.path:
        sys.path.insert(0, REF)
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
