"""reservoir_amd -- MI355X-native reservoir sampling behind the lgbt.princess.reservoir API.

    from reservoir_amd import Sampler
    s = Sampler(100)(lambda user: user.id)          # Sampler.apply
    d = Sampler.distinct(100)(lambda user: user.id) # Sampler.distinct

The compute engine is libreservoir_hip.so (hand-written gfx950 HIP kernels behind the C ABI in
include/reservoir_hip.h); this package is the host-side mirror of the reference interface.
"""
from ._native import (  # noqa: F401
    IllegalArgumentException,
    IllegalStateException,
    NullPointerException,
    ReservoirError,
)
from .sampler import GpuSampler, Sampler, identity  # noqa: F401
from .stream import AbruptStageTerminationException, Sample  # noqa: F401

__all__ = [
    "Sampler", "GpuSampler", "Sample", "identity", "IllegalArgumentException",
    "IllegalStateException", "NullPointerException", "ReservoirError",
    "AbruptStageTerminationException",
]
