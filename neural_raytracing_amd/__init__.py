"""MI355X-native re-implementation of the pytorch3d/pathtracer ray-march render path.

Host API: ``neural_raytracing_amd.pathtracer`` mirrors ``pytorch3d.pathtracer`` (pathtrace,
integrators, SDF shapes, BSDFs, lights, cameras).  Compute: ``libnrt_hip.so`` (include/nrt.h),
hand-written HIP kernels for gfx950 bound with ctypes.
"""
from ._lib import NrtError, get_precision, load, set_precision  # noqa: F401

__all__ = ["NrtError", "get_precision", "set_precision", "load"]
