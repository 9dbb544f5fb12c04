from .integrators import (Debug, Depth, Direct, Integrator, Mask, NeRFIntegrator,  # noqa: F401
                          NeRFReproduce, Path)
