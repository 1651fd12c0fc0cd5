"""Ops layer: native gfx950 kernels behind autograd-aware functions."""
from ._ext import C, native_available, use_native, check_gpu_native  # noqa: F401
