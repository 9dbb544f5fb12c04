from .integrators import (BasisBRDF, Debug, Depth, Direct, Illumination, Integrator,  # noqa: F401
                          Luminance, Mask, NeRFIntegrator, NeRFReproduce, NeuralApprox, Path,
                          Silhouette)
