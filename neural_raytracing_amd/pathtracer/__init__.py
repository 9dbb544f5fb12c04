"""Drop-in mirror of ``pytorch3d.pathtracer`` on the MI355X HIP path."""
from . import bsdf, cameras, integrators, lights, samplers, shapes  # noqa: F401
from .main import pathtrace, pathtrace_sample  # noqa: F401
