"""cglgan -- MI355X-native CGL-GAN worker step (HIP kernels for gfx950 behind a C ABI).

The compute path is ``lib/libcglgan_hip.so``; importing this package loads it and fails
loudly if it is missing (no CPU fallback).  See DESIGN.md.
"""
from . import _lib
from ._lib import version
from .specs import (MIXGEN_HEAD_LAYER, RING_HEAD_LAYER, MlpModel, mixgen_worker, mnist_discriminator,
                    mnist_generator, ring_discriminator, ring_generator)
from .step import GanStep
from . import model

__all__ = ["GanStep", "MlpModel", "mnist_generator", "mnist_discriminator", "mixgen_worker", "ring_generator",
           "ring_discriminator", "MIXGEN_HEAD_LAYER", "RING_HEAD_LAYER", "version", "model"]
