"""goworld_amd — MI355X-native, tick-batched AOI engine for GoWorld.

The product is libgwaoi.so (hand-written HIP for gfx950 behind the C ABI in include/gwaoi.h);
this package is its host-side mirror of go-aoi's AOIManager interface plus a numpy-facing handle.
"""
from ._lib import GwaoiError, load  # noqa: F401

__all__ = ["GwaoiError", "load", "Engine", "aoi"]


def __getattr__(name):
    if name == "Engine":
        from .engine import Engine
        return Engine
    if name == "aoi":
        from . import aoi
        return aoi
    raise AttributeError(name)
