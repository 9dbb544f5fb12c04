from .bsdfs import (BSDF, ComposeSpatialVarying, Conductor, Diffuse, NeuralBSDF,  # noqa: F401
                    identity, identity_div_pi)
