from .bsdfs import (BSDF, Bidirectional, ComposeSpatialVarying, Conductor, Diffuse,  # noqa: F401
                    NeuralBSDF, Phong, Plastic, identity, identity_div_pi)
