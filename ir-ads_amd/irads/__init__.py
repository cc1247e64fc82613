"""irads — MI355X-native (gfx950) hot path of IR-ADS's multimodal segmentation.

``irads.native`` binds libirads.so (C ABI: include/irads.h); ``irads.ops`` holds the
autograd wrappers used by the reference-compatible ``semseg`` / ``detrex`` / ``modules``
packages that live next to it.
"""
from . import native  # noqa: F401

__all__ = ["native", "ops"]
