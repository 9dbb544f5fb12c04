"""Drop-in mirror of ``pytorch3d.pathtracer`` on the MI355X HIP path."""
from . import bsdf, cameras, integrators, lights, samplers, shapes  # noqa: F401
from .integrators import Debug, Depth, Direct, NeRFIntegrator, Path, Silhouette  # noqa: F401
from .interaction import (DirectionSample, Interaction, MixedInteraction,  # noqa: F401
                          SurfaceInteraction)
from .main import pathtrace, pathtrace_sample  # noqa: F401
from .neural_blocks import SkipConnMLP  # noqa: F401
from .samplers import Sampler  # noqa: F401
from .scene import mesh_intersect, mesh_intersect_test  # noqa: F401
from .utils import LossSampler  # noqa: F401
from .warps import (square_to_cos_hemisphere, square_to_cos_hemisphere_pdf,  # noqa: F401
                    square_to_uniform_disk_concentric, square_to_uniform_sphere,
                    square_to_uniform_sphere_pdf)
