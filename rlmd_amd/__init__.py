"""rlmd_amd — MI355X-native vectorised hot path of majidsina/rlmd.

Batched multiplicative-gamble environments, an on-device replay ring and
SAC / TD3 ``learn()`` as hand-written HIP kernels for gfx950, exposed through
the C ABI of ``librlmd_amd.so`` (include/rlmd_abi.h) and this Python facade
with the reference's class and method names.
"""
from . import _abi  # noqa: F401  (fails loudly if the .so is missing)

__all__ = ["envs", "agent", "trainer"]
